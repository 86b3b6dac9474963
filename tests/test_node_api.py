"""Graph-node control API of libcndp_gpu.so (include/cndp_node.h), CPU only.

Reference functions restated (CNDP v25.08.0):
  cne_node_ip4_route_add     lib/usr/clib/nodes/ip4_lookup.c:259-289 (+ setup_fib :292-311)
  cne_node_ip4_rewrite_add   lib/usr/clib/nodes/ip4_rewrite.c:282-312
  ip4_rewrite_set_next       lib/usr/clib/nodes/ip4_rewrite.c:266-277
  cne_node_ip4_add_input     lib/cnet/ipv4/ip4_input.c:263-272
  cne_node_ip6_add_input     lib/cnet/ipv6/ip6_input.c:263-274
  cne_fib6_get_rib           lib/usr/clib/fib/cne_fib6.c:202-205

The prototype tests need /root/reference (this container only) and gcc; the
GPU box skips them.  The table tests check the node FIB's host image with the
oracle's lookup arithmetic; tests/test_gpu_parity.py runs the same ladder
through the GPU lookup.
"""
import ctypes
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from cndp_amd import native as N
from cndp_amd.fib import Fib, Fib6, NodeFib, cne_node_ip4_route_add, node_ip4_add_input, node_ip6_add_input

REF = "/root/reference"
INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
need_ref = pytest.mark.skipif(not (os.path.isdir(REF) and shutil.which("gcc")),
                              reason="needs the reference tree and gcc (build container only)")


def _gcc_syntax(src: str, tmp_path, incs=()):
    f = tmp_path / "proto_check.c"
    f.write_text(src)
    cmd = ["gcc", "-fsyntax-only", "-std=gnu11", "-Wno-address-of-packed-member"]
    for d in incs:
        cmd += ["-I", d]
    cmd += ["-I", INC, str(f)]
    return subprocess.run(cmd, capture_output=True, text=True)


@need_ref
def test_prototypes_match_reference_node_ip4_api(tmp_path):
    """node_ip4_api.h includes only cne_common.h, so it compiles here: include
    it, then this library's header, and let the compiler compare every
    prototype (a mismatch is a 'conflicting types' error)."""
    src = "#include <node_ip4_api.h>\n#include \"cndp_node.h\"\n#include \"cndp_gpu.h\"\n"
    r = _gcc_syntax(src, tmp_path, [f"{REF}/lib/include", f"{REF}/lib/usr/clib/nodes"])
    assert r.returncode == 0, r.stderr
    # negative control: a wrong prototype must be caught the same way
    bad = src + "int cne_node_ip4_route_add(uint32_t, uint8_t, uint32_t, enum cne_node_ip4_lookup_next);\n"
    r = _gcc_syntax(bad, tmp_path, [f"{REF}/lib/include", f"{REF}/lib/usr/clib/nodes"])
    assert r.returncode != 0 and "conflicting types" in r.stderr


def _ref_decl(path: str, name: str) -> str:
    """The reference's declaration of `name` (text up to ';'), CNDP_API removed."""
    with open(path) as f:
        txt = f.read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    m = re.search(r"(^|;|\})\s*((?:CNDP_API\s+)?[A-Za-z_][\w\s\*]*?\b" + name + r"\s*\([^;{]*\)\s*;)", txt, re.M)
    assert m, (path, name)
    return m.group(2).replace("CNDP_API", "")


# headers that cannot be compiled here (cne_fib.h -> cne_inet.h -> cne_inet4.h ->
# <bsd/string.h>, libbsd is absent): their declarations are lifted as text and
# compiled after this library's headers, which checks them the same way
TEXT_CHECKS = [
    ("lib/usr/clib/fib/cne_fib.h", ["cne_fib_create", "cne_fib_free", "cne_fib_add", "cne_fib_delete",
                                     "cne_fib_lookup_bulk", "cne_fib_get_dp", "cne_fib_get_rib",
                                     "cne_fib_select_lookup"]),
    ("lib/usr/clib/fib/cne_fib6.h", ["cne_fib6_create", "cne_fib6_free", "cne_fib6_add", "cne_fib6_delete",
                                      "cne_fib6_lookup_bulk", "cne_fib6_get_dp", "cne_fib6_get_rib",
                                      "cne_fib6_select_lookup"]),
    ("lib/cnet/ipv4/ip4_node_api.h", ["cne_node_ip4_add_input"]),
    ("lib/cnet/ipv6/ip6_node_api.h", ["cne_node_ip6_add_input"]),
    ("lib/usr/clib/nodes/ip4_rewrite_priv.h", ["ip4_rewrite_set_next"]),
    ("lib/usr/clib/nodes/node_ip4_api.h", ["cne_node_ip4_route_add", "cne_node_ip4_rewrite_add"]),
]


@need_ref
def test_prototypes_match_reference_text(tmp_path):
    decls = []
    for rel, names in TEXT_CHECKS:
        for nm in names:
            decls.append(_ref_decl(os.path.join(REF, rel), nm))
    src = "#include \"cndp_node.h\"\n#include \"cndp_gpu.h\"\n" + "\n".join(decls) + "\n"
    r = _gcc_syntax(src, tmp_path)
    assert r.returncode == 0, r.stderr + "\n" + src
    assert len(decls) == sum(len(n) for _, n in TEXT_CHECKS)


def test_headers_compile_as_c_and_cxx(tmp_path):
    if not shutil.which("gcc") or not shutil.which("g++"):
        pytest.skip("no host compiler")
    src = '#include "cndp_fib.h"\n#include "cndp_node.h"\n#include "cndp_gpu.h"\nint main(void){return 0;}\n'
    (tmp_path / "h.c").write_text(src)
    (tmp_path / "h.cc").write_text(src)
    for cc, fn in (("gcc", "h.c"), ("g++", "h.cc")):
        r = subprocess.run([cc, "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I", INC, str(tmp_path / fn)],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def _host_lookup4(fib, ips):
    from oracle import oracle as O
    t24, t8 = fib.image()
    return O.dir24_8_lookup(t24, t8, ips)


def test_route_add_before_node_init_is_a_noop():
    """ip4_lookup.c:278-286: without a FIB (node not initialised) nothing is added, rc 0."""
    NodeFib.fini()
    L = N.lib()
    assert L.cndp_node_ip4_lookup_fib() is None
    assert cne_node_ip4_route_add(0x0A000000, 8, 3, N.IP4_LOOKUP_NEXT_REWRITE) == 0
    nf = NodeFib()
    try:
        assert nf.stats()["routes"] == 0
        assert L.cndp_node_ip4_lookup_init() == 0          # idempotent (init_once)
        assert L.cndp_node_ip4_lookup_fib() == nf.h
    finally:
        NodeFib.fini()


def test_node_fib_ladder_through_route_add():
    """fib_test.c:239-288 check_fib, routes added through the exported
    cne_node_ip4_route_add (val = edge << 16 | nh, nh = depth, edge REWRITE),
    misses on the node FIB's default (PKT_DROP << 16, ip4_lookup.c:302)."""
    from test_oracle_golden import _ladder4
    NodeFib.fini()
    nf = NodeFib()
    try:
        _ladder4(lambda ips: _host_lookup4(nf, np.asarray(ips, np.uint32)),
                 lambda ip, d, nh: cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE),
                 nf.delete, def_nh=N.IP4_LOOKUP_NEXT_PKT_DROP << 16)
        # the edge rides in bits 16..23 of the value, the id in 0..15
        assert cne_node_ip4_route_add(0xC6120000, 24, 0x1234, N.IP4_LOOKUP_NEXT_PKT_DROP) == 0
        assert _host_lookup4(nf, np.array([0xC6120007], np.uint32))[0] == (1 << 16) | 0x1234
        # setup_fib's limits: 1024 routes (rib pool 2048 nodes), 256 tbl8 groups
        st = nf.stats()
        assert st["routes"] == 1
    finally:
        NodeFib.fini()


def test_node_fib_tbl8_limit():
    """The node FIB reserves at most 256 tbl8 groups (ip4_lookup.c:27): the 257th
    /24 holding a /25 fails with -ENOSPC from cne_fib_add."""
    NodeFib.fini()
    NodeFib()
    try:
        rc = [cne_node_ip4_route_add((10 << 24) | (k << 8), 25, k, 0) for k in range(257)]
        assert rc[:256] == [0] * 256
        assert rc[256] == -28
    finally:
        NodeFib.fini()


def test_rewrite_add_semantics():
    """ip4_rewrite.c:266-312 argument checks, in the reference's order."""
    L = N.lib()
    L.cndp_node_ip4_rewrite_reset()
    data = (ctypes.c_uint8 * 56)(*range(56))
    assert L.cne_node_ip4_rewrite_add(64, data, 12, 0) == -22       # next_hop >= 64
    assert L.cne_node_ip4_rewrite_add(0, data, 57, 0) == -22        # rewrite_len > 56
    assert L.cne_node_ip4_rewrite_add(0, data, 12, 3) == -22        # port 3 has no edge yet
    assert L.ip4_rewrite_set_next(32, 1) == -22                     # CNE_MAX_ETHPORTS
    assert L.ip4_rewrite_set_next(3, 5) == 0
    assert L.cne_node_ip4_rewrite_add(7, data, 12, 3) == 0
    assert L.cne_node_ip4_rewrite_add(8, data, 12, 40) == -22       # out of the port table
    out = (ctypes.c_uint8 * 56)()
    ln, tx, en = ctypes.c_uint16(), ctypes.c_uint16(), ctypes.c_uint16()
    assert L.cndp_node_ip4_rewrite_get(7, out, ctypes.byref(ln), ctypes.byref(tx), ctypes.byref(en)) == 0
    assert (ln.value, tx.value, en.value) == (12, 5, 1)
    assert bytes(out)[:12] == bytes(range(12))
    assert L.cndp_node_ip4_rewrite_get(8, out, ctypes.byref(ln), ctypes.byref(tx), ctypes.byref(en)) == 0
    assert en.value == 0
    # a later set_next does not touch entries already added (tx_node is copied)
    assert L.ip4_rewrite_set_next(3, 9) == 0
    L.cndp_node_ip4_rewrite_get(7, out, ctypes.byref(ln), ctypes.byref(tx), ctypes.byref(en))
    assert tx.value == 5
    L.cndp_node_ip4_rewrite_reset()
    assert L.cndp_node_ip4_rewrite_get(7, out, None, None, None) == -2


def test_add_input_edges():
    """ip4_input.c:263-272 / ip6_input.c:263-274: nh = idx | edge << 24, with
    PROTO for depth 32 -- for IPv6 too (the reference tests 32, not 128)."""
    f = Fib("in4", N.CNE_FIB_DIR24_8, default_nh=1025, max_routes=64, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=64)
    assert node_ip4_add_input(f, 0x0A000001, 32, 5) == 0
    assert node_ip4_add_input(f, 0x0B000000, 8, 6) == 0
    got = _host_lookup4(f, np.array([0x0A000001, 0x0B123456, 0x0C000000], np.uint32))
    assert list(got) == [(2 << 24) | 5, (1 << 24) | 6, 1025]
    f6 = Fib6("in6", N.CNE_FIB_TRIE, default_nh=1025, max_routes=64, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1024)
    a = bytes.fromhex("20010db8000000000000000000000001")
    b = bytes.fromhex("20010db9000000000000000000000000")
    assert node_ip6_add_input(f6, a, 128, 7) == 0
    assert node_ip6_add_input(f6, b, 32, 8) == 0
    t24, t8 = f6.image()

    def lk(ip):
        e = int(t24[(ip[0] << 16) | (ip[1] << 8) | ip[2]])
        j = 3
        while e & 1:
            e = int(t8[(e >> 1) * 256 + ip[j]])
            j += 1
        return e >> 1
    assert lk(a) == (1 << 24) | 7        # /128: FORWARD (the quirk keeps PROTO for /32 only)
    assert lk(b[:15] + b"\x09") == (2 << 24) | 8
    # errors are cne_fib_add's
    assert node_ip4_add_input(f, 0, 33, 1) == -22


def test_fib6_get_rib():
    L = N.lib()
    assert L.cne_fib6_get_rib(None) is None
    f6 = Fib6("r6", N.CNE_FIB_TRIE)
    assert L.cne_fib6_get_rib(f6.h)


def test_lookup_without_gpu_fills_default():
    """CNE_FIB_LOOKUP_GPU selected and no usable device: the lookup cannot run,
    so every next hop is the FIB default (callers like l3-fwd.c:85 ignore the
    code) and -ENODEV returns."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    f = Fib("nogpu", N.CNE_FIB_DIR24_8, default_nh=77, max_routes=16, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=16,
            lookup=N.CNE_FIB_LOOKUP_GPU)
    ips = np.arange(300, dtype=np.uint32)
    out = np.full(300, 0xDEAD, np.uint64)
    assert f._L.cne_fib_lookup_bulk(f.h, ips.ctypes.data, out.ctypes.data, 300) == -19
    assert np.all(out == 77)
