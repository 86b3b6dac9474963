"""C-ABI boundary + host control plane, CPU only (no kernel launches).

The FIB control plane (RIB + DIR-24-8 / trie build) runs on the host, so its
table images can be checked here with the oracle's lookup arithmetic; the
GPU lookups over the same images are checked in test_gpu_parity.py.
Reference tests mirrored: test/testcne/fib_test.c (create/add/delete
invalid-argument cases, check_fib ladder), fib6_test.c, lpm6_data_test.h.
"""
import ctypes
import os

import numpy as np
import pytest

from cndp_amd import native as N
from cndp_amd.fib import Fib, Fib6, node_ip4_route_add
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_library_exports_every_declared_symbol():
    L = N.lib()
    names = N.exported_symbols()
    assert "cne_fib_create" in names and "cndp_gpu_classify" in names
    for name in names:
        assert hasattr(L, name), name
    assert L.cndp_gpu_version().startswith(b"cndp_amd")
    assert L.cndp_gpu_get_stat(None, N.CNDP_STAT_CNET_WORKLIST) == -22  # -EINVAL, no context


def test_no_oracle_in_product():
    """The product library must not link or reference the checker."""
    with open(N.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"liboracle" not in blob and b"orc_classify" not in blob
    root = os.path.dirname(N.HERE)
    for dp, _, files in os.walk(os.path.join(root, "cndp_amd")):
        for fn in files:
            if fn.endswith((".py", ".c", ".h", ".hip")):
                with open(os.path.join(dp, fn)) as f:
                    txt = f.read()
                assert "from oracle" not in txt and "import oracle" not in txt, fn


def _conf(type_, def_nh=0, max_routes=1 << 10, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256):
    c = N.FibConf()
    c.type, c.default_nh, c.max_routes = type_, def_nh, max_routes
    c.dir24_8.nh_sz, c.dir24_8.num_tbl8 = nh_sz, num_tbl8
    return c


def test_create_invalid():
    """fib_test.c test_create_invalid (:34-74)."""
    L = N.lib()
    c = _conf(N.CNE_FIB_DUMMY)
    assert not L.cne_fib_create(None, ctypes.byref(c))
    assert not L.cne_fib_create(b"x", None)
    c.max_routes = 0
    assert not L.cne_fib_create(b"x", ctypes.byref(c))
    c = _conf(N.CNE_FIB_DIR24_8 + 1)
    assert not L.cne_fib_create(b"x", ctypes.byref(c))
    c = _conf(N.CNE_FIB_DIR24_8, nh_sz=N.CNE_FIB_DIR24_8_8B + 1)
    assert not L.cne_fib_create(b"x", ctypes.byref(c))
    c = _conf(N.CNE_FIB_DIR24_8, num_tbl8=0)
    assert not L.cne_fib_create(b"x", ctypes.byref(c))
    c = _conf(N.CNE_FIB_DIR24_8, nh_sz=N.CNE_FIB_DIR24_8_1B, num_tbl8=128)  # > max_nh(1B)=127
    assert not L.cne_fib_create(b"x", ctypes.byref(c))
    c = _conf(N.CNE_FIB_DIR24_8, nh_sz=N.CNE_FIB_DIR24_8_1B, def_nh=128, num_tbl8=64)
    assert not L.cne_fib_create(b"x", ctypes.byref(c))
    # IPv6: DIR24_8 type is rejected, TRIE 1B does not exist
    c = _conf(N.CNE_FIB_DIR24_8)
    assert not L.cne_fib6_create(b"x", ctypes.byref(c))
    c = _conf(N.CNE_FIB_TRIE, nh_sz=0)
    assert not L.cne_fib6_create(b"x", ctypes.byref(c))
    c = _conf(N.CNE_FIB_TRIE + 1)
    assert not L.cne_fib6_create(b"x", ctypes.byref(c))


def test_add_del_invalid():
    """fib_test.c test_add_del_invalid (:129-166) and test_get_invalid."""
    L = N.lib()
    assert L.cne_fib_add(None, 0, 24, 100) < 0
    assert L.cne_fib_delete(None, 0, 24) < 0
    f = Fib("x", N.CNE_FIB_DUMMY)
    assert f.add(0, 33, 100) < 0
    assert f.delete(0, 33) < 0
    assert L.cne_fib_get_dp(None) is None
    assert L.cne_fib_get_rib(None) is None
    d = Fib("y", N.CNE_FIB_DIR24_8, nh_sz=N.CNE_FIB_DIR24_8_1B, num_tbl8=64)
    assert d.add(10 << 24, 8, 128) == -22  # next hop > max_nh(1B) -> -EINVAL
    assert d.delete(10 << 24, 8) == -2     # -ENOENT
    L.cne_fib_free(None)
    f6 = Fib6("z", N.CNE_FIB_TRIE, nh_sz=N.CNE_FIB_TRIE_2B, num_tbl8=64)
    assert f6.add(bytes(16), 129, 1) < 0
    assert f6.delete(bytes(16), 64) == -2


def test_select_lookup():
    f = Fib("x", N.CNE_FIB_DIR24_8)
    for t in (N.CNE_FIB_LOOKUP_DEFAULT, N.CNE_FIB_LOOKUP_DIR24_8_SCALAR_MACRO, N.CNE_FIB_LOOKUP_GPU):
        assert f.select_lookup(t) == 0
    assert f.select_lookup(N.CNE_FIB_LOOKUP_TRIE_SCALAR) < 0
    # the AVX-512 selectors: -EINVAL, as the reference at its default 256-bit
    # SIMD width (dir24_8.c:63-69, trie.c:47-53, cne_vect_generic.h:205)
    assert f.select_lookup(N.CNE_FIB_LOOKUP_DIR24_8_VECTOR_AVX512) == -22
    assert Fib6("z", N.CNE_FIB_TRIE).select_lookup(N.CNE_FIB_LOOKUP_TRIE_VECTOR_AVX512) == -22
    # cne_fib.c:206-221: a DUMMY FIB selects nothing of the reference's; the
    # GPU extension is accepted
    assert Fib("d", N.CNE_FIB_DUMMY).select_lookup(N.CNE_FIB_LOOKUP_DEFAULT) < 0
    assert Fib("d", N.CNE_FIB_DUMMY).select_lookup(N.CNE_FIB_LOOKUP_GPU) == 0
    f6 = Fib6("y", N.CNE_FIB_TRIE)
    assert f6.select_lookup(N.CNE_FIB_LOOKUP_TRIE_SCALAR) == 0
    assert f6.select_lookup(N.CNE_FIB_LOOKUP_DIR24_8_SCALAR_MACRO) < 0
    assert Fib6("d6", N.CNE_FIB_DUMMY).select_lookup(N.CNE_FIB_LOOKUP_GPU) == 0


# ---- cne_fib_lookup_bulk with the reference's default selection -----------
# cne_fib.c:86 / cne_fib6.c:92 bind the scalar loop of dir24_8.h:118-148 /
# trie.h:119-138 at create time; this library answers those calls on the
# calling thread from the host image (no GPU involved), so they run here.

@pytest.mark.parametrize("kind", [("dummy", N.CNE_FIB_DUMMY, 0, 127), ("1B", N.CNE_FIB_DIR24_8, 0, 127),
                                  ("2B", N.CNE_FIB_DIR24_8, 1, 255), ("4B", N.CNE_FIB_DIR24_8, 2, 256),
                                  ("8B", N.CNE_FIB_DIR24_8, 3, 256)])
def test_ladder4_default_lookup(kind):
    """fib_test.c check_fib (:239-348) through cne_fib_lookup_bulk as created."""
    from test_oracle_golden import _ladder4
    _, t, nh_sz, ntbl8 = kind
    f = Fib("lad", t, default_nh=100, max_routes=1 << 16, nh_sz=nh_sz, num_tbl8=ntbl8)
    _ladder4(f.lookup_bulk, f.add, f.delete)


@pytest.mark.parametrize("nh_sz", [0, 1, 2, 3])
def test_default_lookup_vs_bruteforce(nh_sz):
    rng = np.random.default_rng(40 + nh_sz)
    maxnh = (1 << ((8 << nh_sz) - 1)) - 1
    f = Fib("b", N.CNE_FIB_DIR24_8, default_nh=min(7, maxnh), max_routes=4096, nh_sz=nh_sz,
            num_tbl8=min(127, maxnh) if nh_sz == 0 else 512)
    routes = {}
    for _ in range(400):
        d = int(rng.integers(8, 33))
        ip = int(rng.integers(0, 2**32))
        ip = 0x0A000000 | (ip & 0x00FFFFFF) if rng.random() < 0.7 else ip
        ip &= (0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF
        nh = int(rng.integers(0, maxnh + 1))
        if f.add(ip, d, nh) == 0:
            routes[(ip, d)] = nh
    ips = rng.integers(0, 2**32, size=20000, dtype=np.uint64).astype(np.uint32)
    ips[::2] = 0x0A000000 | (ips[::2] & 0x00FFFFFF)
    want = O.lpm4_bruteforce([(ip, d, nh) for (ip, d), nh in routes.items()], min(7, maxnh), ips)
    for n in (1, 3, 4, 15, 16, 17, 256, 20000):  # below, at and past the prefetch distance
        assert np.array_equal(f.lookup_bulk(ips[:n]), want[:n]), n
    for t in (N.CNE_FIB_LOOKUP_DIR24_8_SCALAR_MACRO, N.CNE_FIB_LOOKUP_DIR24_8_SCALAR_UNI,
              N.CNE_FIB_LOOKUP_DEFAULT):
        assert f.select_lookup(t) == 0
        assert np.array_equal(f.lookup_bulk(ips), want)


def test_default_lookup6_golden():
    """lpm6_data_test.h's 1000 rules and the reference's expected next hops,
    through cne_fib6_lookup_bulk as created, for every trie width and DUMMY."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "lpm6_1000.npz"))
    for t, nh_sz in ((N.CNE_FIB_TRIE, N.CNE_FIB_TRIE_2B), (N.CNE_FIB_TRIE, N.CNE_FIB_TRIE_4B),
                     (N.CNE_FIB_TRIE, N.CNE_FIB_TRIE_8B), (N.CNE_FIB_DUMMY, 0)):
        f6 = Fib6("l6", t, default_nh=0, max_routes=2000, nh_sz=nh_sz, num_tbl8=1 << 14)
        for ip, d, nh in zip(g["rule_ip"], g["rule_depth"], g["rule_nh"]):
            assert f6.add(bytes(ip), int(d), int(nh)) == 0
        for n in (1, 4, 256, len(g["ip"])):
            assert np.array_equal(f6.lookup_bulk(g["ip"][:n]), g["nh"][:n].astype(np.uint64))


def test_default_lookup_while_routes_change():
    """cnet adds ARP and route entries while graphs forward: one thread adds and
    deletes routes while three call cne_fib_lookup_bulk (no lock on the lookup,
    as in dir24_8.h).  A /24 under a /16 is the only thing that ever changes for
    the probe keys, so every answer is one of the two next hops; afterwards the
    lookups equal brute-force LPM over the final routes."""
    import threading
    f = Fib("churn", N.CNE_FIB_DIR24_8, default_nh=3, max_routes=8192, nh_sz=N.CNE_FIB_DIR24_8_4B,
            num_tbl8=1024)
    assert f.add(0x0B000000, 16, 50) == 0
    rng = np.random.default_rng(78)
    probe = (0x0B000000 | rng.integers(0, 1 << 16, size=4096, dtype=np.uint64)).astype(np.uint32)
    stop = threading.Event()
    bad = []

    def reader():
        k = 0
        while not stop.is_set():
            n = (4, 256, 4096)[k % 3]
            got = f.lookup_bulk(probe[:n])
            ok = (got >= 50) & (got < 50 + 1 + 3000)
            if not ok.all():
                bad.append(got[~ok][:4])
                return
            k += 1

    th = [threading.Thread(target=reader) for _ in range(3)]
    for t in th:
        t.start()
    routes = {(0x0B000000, 16): 50}
    try:
        for k in range(3000):
            d = int(rng.choice([24, 25, 28, 32]))
            ip = (0x0B000000 | int(rng.integers(0, 1 << 16))) & (0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF
            if k % 4 == 3 and len(routes) > 1:
                keys = [r for r in routes if r[1] > 16]
                dip, dd = keys[int(rng.integers(0, len(keys)))]
                assert f.delete(dip, dd) == 0
                del routes[(dip, dd)]
            elif f.add(ip, d, 51 + k) == 0:
                routes[(ip, d)] = 51 + k
    finally:
        stop.set()
        for t in th:
            t.join()
    assert not bad, bad[:3]
    want = O.lpm4_bruteforce([(ip, d, nh) for (ip, d), nh in routes.items()], 3, probe)
    assert np.array_equal(f.lookup_bulk(probe), want)


def _host_lookup4(fib, ips):
    t24, t8 = fib.image()
    if t24.dtype == np.uint32:
        return O.dir24_8_lookup(t24, t8, ips)
    ips = np.asarray(ips, np.uint64)
    e = t24[(ips >> 8).astype(np.int64)].astype(np.uint64)
    ext = (e & 1) == 1
    idx = ((e >> 1) * 256 + (ips & 0xFF)).astype(np.int64)
    e = np.where(ext, t8[np.where(ext, idx, 0)].astype(np.uint64), e)
    return e >> 1


def _host_lookup6(fib6, ips):
    t24, t8 = fib6.image()
    ips = np.asarray(ips, np.uint8).reshape(-1, 16)
    out = np.zeros(len(ips), np.uint64)
    for i, ip in enumerate(ips):
        e = int(t24[(int(ip[0]) << 16) | (int(ip[1]) << 8) | int(ip[2])])
        j = 3
        while e & 1:
            e = int(t8[(e >> 1) * 256 + int(ip[j])])
            j += 1
        out[i] = e >> 1
    return out


@pytest.mark.parametrize("kind", [("dummy", N.CNE_FIB_DUMMY, 0, 127), ("1B", N.CNE_FIB_DIR24_8, 0, 127),
                                  ("2B", N.CNE_FIB_DIR24_8, 1, 255), ("4B", N.CNE_FIB_DIR24_8, 2, 256),
                                  ("8B", N.CNE_FIB_DIR24_8, 3, 256)])
def test_ladder4_host_image(kind):
    """fib_test.c test_lookup (:290-348): check_fib on every FIB flavour."""
    from test_oracle_golden import _ladder4
    _, t, nh_sz, ntbl8 = kind
    f = Fib("lad", t, default_nh=100, max_routes=1 << 16, nh_sz=nh_sz, num_tbl8=ntbl8)
    _ladder4(lambda ips: _host_lookup4(f, ips), f.add, f.delete)


@pytest.mark.parametrize("seed", [11, 12])
def test_random_add_delete_host_image(seed):
    """Random route churn: product table image == brute-force LPM."""
    rng = np.random.default_rng(seed)
    f = Fib("churn", N.CNE_FIB_DIR24_8, default_nh=5, max_routes=4096, nh_sz=N.CNE_FIB_DIR24_8_4B,
            num_tbl8=1024)
    live = {}
    for step in range(600):
        if live and rng.random() < 0.3:
            key = list(live)[int(rng.integers(0, len(live)))]
            assert f.delete(*key) == 0
            del live[key]
        else:
            d = int(rng.integers(0, 33)) if rng.random() < 0.3 else int(rng.integers(20, 33))
            ip = int(rng.integers(0, 2**32)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF if d else 0)
            if rng.random() < 0.5:
                ip = (0x0A000000 | (ip & 0x0003FFFF)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF if d else 0)
            nh = int(rng.integers(0, 1 << 20))
            assert f.add(ip, d, nh) == 0
            live[(ip, d)] = nh
    routes = [(ip, d, nh) for (ip, d), nh in live.items()]
    ips = rng.integers(0, 2**32, size=8192, dtype=np.uint64).astype(np.uint32)
    ips[::2] = 0x0A000000 | (ips[::2] & 0x0003FFFF)
    assert np.array_equal(_host_lookup4(f, ips), O.lpm4_bruteforce(routes, 5, ips))
    st = f.stats()
    assert st["routes"] == len(live)


def test_enospc_reservation():
    """dir24_8.c:405-409: a /25+ route in a fresh /24 needs a free tbl8 slot."""
    f = Fib("sp", N.CNE_FIB_DIR24_8, default_nh=0, max_routes=4096, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=64)
    for k in range(64):
        assert f.add((10 << 24) | (k << 8), 25, k + 1) == 0
    assert f.add((10 << 24) | (64 << 8), 25, 99) == -28  # -ENOSPC
    assert f.add((10 << 24) | (3 << 8) | 128, 25, 7) == 0  # same /24 as an existing one: fine
    assert f.delete((10 << 24) | (5 << 8), 25) == 0
    assert f.add((10 << 24) | (64 << 8), 25, 99) == 0


def test_rib_node_budget():
    """cne_rib node pool = 2 * max_routes (cne_fib.c:131-132): insert fails with -1."""
    f = Fib("nb", N.CNE_FIB_DIR24_8, default_nh=0, max_routes=4, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=64)
    rc = [f.add(k << 24, 8, k) for k in range(1, 10)]
    assert rc[:4] == [0, 0, 0, 0]
    assert -1 in rc


def test_lpm6_1000_rules_host_image():
    g = np.load(os.path.join(GOLD, "lpm6_1000.npz"))
    f6 = Fib6("l6", N.CNE_FIB_TRIE, default_nh=0, max_routes=2000, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 16)
    for ip, d, nh in zip(g["rule_ip"], g["rule_depth"], g["rule_nh"]):
        assert f6.add(bytes(ip), int(d), int(nh)) == 0
    sel = slice(0, 3000)
    assert np.array_equal(_host_lookup6(f6, g["ip"][sel]), g["nh"][sel].astype(np.uint64))


def test_ladder6_host_image():
    """fib6_test.c check_fib (:243-300) on the trie image."""
    def mask_ip(d):
        v = (1 << 128) - (1 << (128 - d)) if d else 0
        return v
    ip_add = 128 << 120
    ip_arr = []
    for i in range(128):
        v = ip_add | (((1 << 128) - 1) ^ mask_ip(128 - i))
        ip_arr.append(np.frombuffer(v.to_bytes(16, "big"), np.uint8))
    missing = np.frombuffer(((127 << 120) | ((1 << 120) - 1)).to_bytes(16, "big"), np.uint8)
    f6 = Fib6("l6", N.CNE_FIB_TRIE, default_nh=100, max_routes=1 << 10, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 12)
    arr = np.stack(ip_arr + [missing])

    def desc(n):
        got = list(_host_lookup6(f6, arr))
        exp = [128 - i for i in range(n)] + [100] * (128 - n) + [100]
        assert got == exp, n

    def asc(n):
        got = list(_host_lookup6(f6, arr))
        exp = [n] * (128 - n + 1) + [n - 1 - k for k in range(n - 1)] + [100]
        assert got == exp, n

    desc(0)
    for i in range(1, 129, 9):
        pass
    for i in range(1, 129):
        assert f6.add(ip_add.to_bytes(16, "big"), i, i) == 0
    asc(128)
    for i in range(128, 1, -1):
        assert f6.delete(ip_add.to_bytes(16, "big"), i) == 0
        if i % 16 == 0:
            asc(i - 1)
    assert f6.delete(ip_add.to_bytes(16, "big"), 1) == 0
    desc(0)
    for i in range(128):
        assert f6.add(ip_add.to_bytes(16, "big"), 128 - i, 128 - i) == 0
    desc(128)
    st = f6.stats()
    for i in range(1, 129):
        assert f6.delete(ip_add.to_bytes(16, "big"), i) == 0
        if i % 16 == 0:
            desc(128 - i)
    assert f6.stats()["tbl8_used"] == 0
    assert st["routes"] == 128


def test_l3fwd_routes_image_matches_oracle():
    from cndp_amd import pktgen
    f = Fib("rt4", N.CNE_FIB_DIR24_8, default_nh=1 << 16, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B,
            num_tbl8=256)
    routes = pktgen.l3fwd_routes()
    for ip, d, nh in routes:
        assert node_ip4_route_add(f, ip, d, nh, 0) == 0
    vals = [(ip, d, nh) for ip, d, nh in routes]
    t24, t8 = O.dir24_8_build(vals, 1 << 16, 256)
    rng = np.random.default_rng(3)
    ips = rng.integers(0, 2**32, size=1 << 16, dtype=np.uint64).astype(np.uint32)
    ips[::2] = (10 << 24) | (ips[::2] & 0x0004FFFF)
    assert np.array_equal(_host_lookup4(f, ips), O.dir24_8_lookup(t24, t8, ips))


def test_frames_alloc_argument_checks():
    """cndp_gpu_frames_alloc rejects a zero size, unknown flags and a NULL
    out pointer before it touches a device (CPU-safe)."""
    L = N.lib()
    p = ctypes.c_void_p(1)
    assert L.cndp_gpu_frames_alloc(-1, 0, 0, ctypes.byref(p)) == -22 and p.value is None
    assert L.cndp_gpu_frames_alloc(-1, 4096, 0x10, ctypes.byref(p)) == -22
    assert L.cndp_gpu_frames_alloc(-1, 4096, 0, None) == -22
    assert L.cndp_gpu_frames_free(None) == 0
    import torch
    from cndp_amd import pktgen
    t = pktgen.frame_slab(1000, "cpu")
    assert t.dtype == torch.uint8 and t.numel() == 1000 and int(t.sum()) == 0
