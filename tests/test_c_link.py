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


RATE = os.path.join(HERE, "c_link", "fib_rate")


def test_fib_rate_default_selection():
    """tests/c_link/fib_rate, the default selection only: cnet's rt4 / arp /
    nd6 FIBs looked up through cne_fib_lookup_bulk from plain C in 1-, 4- and
    256-key calls on the host image, every answer checked (brute-force LPM for
    rt4 and arp, the whole-array call for the rest)."""
    import json
    if not os.path.exists(RATE):
        pytest.skip("fib_rate not built (build() makes it)")
    r = subprocess.run([RATE, "--ms", "20"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout)
    assert res["wrong"] == 0 and len(res["points"]) == 9


@pytest.mark.gpu
def test_fib_rate_both_selections(gpu):
    """The same through CNE_FIB_LOOKUP_GPU as well: every GPU answer equals the
    host image's."""
    import json
    r = subprocess.run([RATE, "--gpu", "--ms", "20"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout)
    assert res["wrong"] == 0 and {p["sel"] for p in res["points"]} == {"default", "gpu"}
