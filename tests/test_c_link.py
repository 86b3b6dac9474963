"""A plain C program built against include/cndp_fib.h and linked to
libcndp_gpu.so (tests/c_link/l3fwd_fib_demo.c): the FIB usage of
examples/cndpfwd/l3-fwd.c:78-117 -- a DUMMY FIB with 48-bit next hops, one
cne_fib_lookup_bulk per 256-address burst -- checked against a longest-prefix
match over the same rules.  Without a GPU the lookups return -ENODEV with the
default next hop (exit 77); on the GPU every answer must be right (exit 0)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
DEMO = os.path.join(HERE, "c_link", "l3fwd_fib_demo")


def _run():
    if not os.path.exists(DEMO):
        pytest.skip("c_link demo not built (build() makes it)")
    return subprocess.run([DEMO], capture_output=True, text=True, timeout=120)


def test_c_program_links_and_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = _run()
    assert r.returncode == 77, r.stdout + r.stderr


@pytest.mark.gpu
def test_c_program_fib_lookups_on_gpu(gpu):
    r = _run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
