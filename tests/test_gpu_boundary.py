"""GPU tests of the drop-in boundary: the node control API driving the GPU
paths, the host-array FIB lookups (per-burst callers, many threads), and the
stream order of a context's scratch.  Everything goes through the C-ABI."""
import ctypes
import threading

import numpy as np
import pytest
import torch

from cndp_amd import native as N
from cndp_amd import pktgen
from oracle import oracle as O

from helpers import CNET_DEF, assert_same, cnet_fibs, l3fwd_fib, l3fwd_oracle_tables, oracle_classify

pytestmark = pytest.mark.gpu


def test_node_fib_ladder_gpu(gpu):
    """fib_test.c:239-288 check_fib through the exported cne_node_ip4_route_add
    on the library-owned node FIB, looked up by the GPU cne_fib_lookup_bulk."""
    from test_oracle_golden import _ladder4
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    NodeFib.fini()
    nf = NodeFib()
    assert nf.select_lookup(N.CNE_FIB_LOOKUP_GPU) == 0
    try:
        _ladder4(nf.lookup_bulk, lambda ip, d, nh: cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE),
                 nf.delete, def_nh=N.IP4_LOOKUP_NEXT_PKT_DROP << 16)
    finally:
        NodeFib.fini()


# both selections of cne_fib_select_lookup: the device mirror and the host
# image (CNE_FIB_LOOKUP_DEFAULT, what cne_fib_create binds)
SELECTIONS = pytest.mark.parametrize("sel", [N.CNE_FIB_LOOKUP_GPU, N.CNE_FIB_LOOKUP_DEFAULT],
                                     ids=["gpu", "host"])


def _routes_fib(seed, nh_sz=N.CNE_FIB_DIR24_8_4B, sel=N.CNE_FIB_LOOKUP_GPU):
    from cndp_amd.fib import Fib
    rng = np.random.default_rng(seed)
    f = Fib(f"t{seed}", N.CNE_FIB_DIR24_8, default_nh=9, max_routes=4096, nh_sz=nh_sz, num_tbl8=512,
            lookup=sel)
    routes = {}
    for _ in range(500):
        d = int(rng.integers(8, 33))
        ip = (0x0A000000 | int(rng.integers(0, 1 << 24))) & (0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF
        nh = int(rng.integers(0, 1 << 20))
        if f.add(ip, d, nh) == 0:
            routes[(ip, d)] = nh
    return f, [(ip, d, nh) for (ip, d), nh in routes.items()]


@SELECTIONS
def test_fib_lookup_bulk_many_threads(gpu, sel):
    """examples/cndpfwd/l3-fwd.c:85 calls cne_fib_lookup_bulk per burst from
    every forwarding thread on one FIB.  Eight threads start on a FIB that has
    no device mirror yet (the first lookups race to create it) and issue
    4-, 256- and 5000-key calls; every answer equals brute-force LPM."""
    f, routes = _routes_fib(21, sel=sel)
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 2**32, size=1 << 16, dtype=np.uint64).astype(np.uint32)
    keys[::2] = 0x0A000000 | (keys[::2] & 0x00FFFFFF)
    want = O.lpm4_bruteforce(routes, 9, keys)
    errors = []

    def worker(t):
        try:
            r = np.random.default_rng(100 + t)
            for it in range(60):
                n = (4, 256, 5000)[it % 3]
                lo = int(r.integers(0, keys.size - n))
                ips = keys[lo:lo + n].copy()
                out = np.zeros(n, np.uint64)
                rc = f._L.cne_fib_lookup_bulk(f.h, ips.ctypes.data, out.ctypes.data, n)
                if rc != 0 or not np.array_equal(out, want[lo:lo + n]):
                    errors.append((t, it, rc))
                    return
        except Exception as e:  # pragma: no cover - reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:4]


@SELECTIONS
def test_fib_lookup_bulk_large_and_v6(gpu, sel):
    """Calls above the mapped-staging size (DMA path, chunked) and IPv6."""
    f, routes = _routes_fib(22, sel=sel)
    rng = np.random.default_rng(6)
    ips = rng.integers(0, 2**32, size=(1 << 20) + 12345, dtype=np.uint64).astype(np.uint32)
    ips[::2] = 0x0A000000 | (ips[::2] & 0x00FFFFFF)
    got = f.lookup_bulk(ips)
    some = slice(0, None, 97)
    assert np.array_equal(got[some], O.lpm4_bruteforce(routes, 9, ips[some]))
    t24, t8 = f.image()
    assert np.array_equal(got, O.dir24_8_lookup(t24, t8, ips))
    import os
    from cndp_amd.fib import Fib6
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "lpm6_1000.npz"))
    f6 = Fib6("l6b", N.CNE_FIB_TRIE, default_nh=0, max_routes=2000, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 14,
              lookup=sel)
    for ip, d, nh in zip(g["rule_ip"], g["rule_depth"], g["rule_nh"]):
        assert f6.add(bytes(ip), int(d), int(nh)) == 0
    for n in (1, 4, 256, 20000):
        assert np.array_equal(f6.lookup_bulk(g["ip"][:n]), g["nh"][:n].astype(np.uint64))


def test_node_rewrite_table_drives_gpu_rewrite(gpu):
    """A context without a table of its own rewrites with the table filled
    through the exported ip4_rewrite_set_next / cne_node_ip4_rewrite_add
    (ip4_rewrite.c:266-312), and follows later changes to it."""
    from cndp_amd.classify import Classifier
    L = N.lib()
    L.cndp_node_ip4_rewrite_reset()
    fib, vals = l3fwd_fib()
    t4 = l3fwd_oracle_tables(vals)
    cl = Classifier(0)
    cl.set_fib(fib)
    tbl = np.zeros(64, O.REWRITE_NH)
    for p in range(4):
        assert L.ip4_rewrite_set_next(p, p + 1) == 0
    rng = np.random.default_rng(8)
    for nh in range(40):
        data = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        buf = ctypes.create_string_buffer(data, 12)
        assert L.cne_node_ip4_rewrite_add(nh, buf, 12, nh % 4) == 0
        tbl[nh]["rewrite_len"], tbl[nh]["tx_node"], tbl[nh]["enabled"] = 12, nh % 4 + 1, 1
        tbl[nh]["rewrite_data"][:12] = np.frombuffer(data, np.uint8)
    for step in range(2):
        fr = pktgen.packed_ipv4(30000, routes=pktgen.l3fwd_routes(), seed=40 + step)
        ref = oracle_classify(O.MODE_L3FWD, fr, tables4=t4)
        host = fr.slab.numpy().copy()
        ref_tx = O.ip4_rewrite(host, fr.n, ref["nh"], tbl, burst=256)
        dfr = pktgen.Frames(fr.slab.to(gpu), fr.n, stride=64)
        out = cl.classify(dfr, N.CNDP_MODE_L3FWD)
        tx = cl.ip4_rewrite(dfr, out["nh"], burst=256)
        torch.cuda.synchronize()
        assert np.array_equal(tx.cpu().numpy().view(np.uint16), ref_tx)
        assert np.array_equal(dfr.slab.cpu().numpy(), host)
        # change next hop 3 (new data, port 2) between the two batches
        data = bytes(range(100, 112))
        assert L.cne_node_ip4_rewrite_add(3, ctypes.create_string_buffer(data, 12), 12, 2) == 0
        tbl[3]["tx_node"] = 3
        tbl[3]["rewrite_data"][:12] = np.frombuffer(data, np.uint8)
    cl.close()
    L.cndp_node_ip4_rewrite_reset()


def test_scratch_stream_order(gpu):
    """One context, cnet calls alternating between two streams and the host
    path with no synchronisation in between: the speculation state carries
    from call to call exactly as if the calls ran one after another."""
    from cndp_amd.classify import Classifier
    from test_gpu_parity import _gtp_mix
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    cl = Classifier(0)
    cl.set_fib(fib, fib6)
    cl.set_tuning(cnet_spec=256)
    fr = _gtp_mix(256 * 200, routes, v6, gpu, seed=3)
    parts = 6
    cut = [k * (fr.n // parts) // 256 * 256 for k in range(parts)] + [fr.n]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs, refs = [], []
    st = np.zeros(1, np.uint16)
    host_slab = fr.slab.cpu().numpy()
    host_off = fr.offsets.cpu().numpy().astype(np.uint64)
    prts = [pktgen.Frames(fr.slab, cut[k + 1] - cut[k], offsets=fr.offsets[cut[k]:cut[k + 1]].contiguous())
            for k in range(parts)]
    outb = [cl.alloc_outputs(p.n, 64, device=gpu) for p in prts]
    torch.cuda.synchronize()
    for k in range(parts):
        lo, hi = cut[k], cut[k + 1]
        refs.append(oracle_classify(O.MODE_CNET, prts[k], tables4=t4, tables6=t6, spec_burst=256, spec_state=st))
        if k % 3 == 2:   # the host path (its own streams) in the middle of the chain
            o = cl.classify_host(host_slab, hi - lo, N.CNDP_MODE_CNET, offsets=host_off[lo:hi].copy())
        else:
            s = s1 if k % 3 == 0 else s2
            o = cl.classify(prts[k], N.CNDP_MODE_CNET, out=outb[k], stream=s.cuda_stream)
        outs.append(o)
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert_same(o, r)
    cl.close()


def test_scratch_stream_destroyed(gpu):
    """A caller-created HIP stream that ran a cnet call is handed back with
    cndp_gpu_stream_release and destroyed; the next calls (another such stream,
    then the null stream) order after its work and carry the speculation state
    exactly as if the calls ran one after another."""
    from cndp_amd.classify import Classifier
    from test_gpu_parity import _gtp_mix
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    cl = Classifier(0)
    cl.set_fib(fib, fib6)
    cl.set_tuning(cnet_spec=256)
    fr = _gtp_mix(256 * 120, routes, v6, gpu, seed=4)
    parts = 3
    cut = [k * (fr.n // parts) // 256 * 256 for k in range(parts)] + [fr.n]
    prts = [pktgen.Frames(fr.slab, cut[k + 1] - cut[k], offsets=fr.offsets[cut[k]:cut[k + 1]].contiguous())
            for k in range(parts)]
    outb = [cl.alloc_outputs(p.n, 64, device=gpu) for p in prts]
    st = np.zeros(1, np.uint16)
    refs = [oracle_classify(O.MODE_CNET, p, tables4=t4, tables6=t6, spec_burst=256, spec_state=st) for p in prts]
    torch.cuda.synchronize()
    outs = []
    L = N.lib()
    for k in range(parts):
        if k < parts - 1:
            s = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(s)) == 0
            outs.append(cl.classify(prts[k], N.CNDP_MODE_CNET, out=outb[k], stream=s.value))
            assert L.cndp_gpu_stream_release(cl.h, s) == 0
            assert hip.hipStreamDestroy(s) == 0
        else:
            outs.append(cl.classify(prts[k], N.CNDP_MODE_CNET, out=outb[k], stream=0))
    torch.cuda.synchronize()
    for o, r in zip(outs, refs):
        assert_same(o, r)
    assert L.cndp_gpu_stream_release(cl.h, None) == 0   # not the last user's: a no-op
    cl.close()


@SELECTIONS
def test_fib_add_while_lookup(gpu, sel):
    """cnet adds routes at run time while graphs walk: one thread adds and
    deletes routes (cne_fib_add / _delete) while three threads call
    cne_fib_lookup_bulk, which syncs the device mirror from the dirty ranges.
    The ranges change under the table's lock, so no sync copies a
    half-painted range or clears marks it did not copy: once the writer is
    done, every lookup equals brute-force LPM over the final routes."""
    from cndp_amd.fib import Fib
    f = Fib("churn", N.CNE_FIB_DIR24_8, default_nh=3, max_routes=8192, nh_sz=N.CNE_FIB_DIR24_8_4B,
            num_tbl8=1024, lookup=sel)
    rng = np.random.default_rng(77)
    keys = (0x0B000000 | rng.integers(0, 1 << 24, size=1 << 14, dtype=np.uint64)).astype(np.uint32)
    routes = {}
    stop = threading.Event()
    errors = []

    def reader():
        try:
            k = 0
            while not stop.is_set():  # per-burst and larger calls
                f.lookup_bulk(keys[:4096] if k % 2 else keys[:256])
                k += 1
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    th = [threading.Thread(target=reader) for _ in range(3)]
    for t in th:
        t.start()
    try:
        for k in range(3000):
            d = int(rng.choice([16, 20, 24, 24, 28, 32]))
            ip = (0x0B000000 | int(rng.integers(0, 1 << 24))) & (0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF
            if k % 5 == 4 and routes:
                (dip, dd) = list(routes)[int(rng.integers(0, len(routes)))]
                assert f.delete(dip, dd) == 0
                del routes[(dip, dd)]
            elif f.add(ip, d, k + 10) == 0:
                routes[(ip, d)] = k + 10
    finally:
        stop.set()
        for t in th:
            t.join()
    assert not errors, errors
    want = O.lpm4_bruteforce([(ip, d, nh) for (ip, d), nh in routes.items()], 3, keys)
    assert np.array_equal(f.lookup_bulk(keys), want)
    # per-burst calls on staging slots of their own see the same mirror
    for o in range(0, 4096, 1024):
        assert np.array_equal(f.lookup_bulk(keys[o:o + 1024]), want[o:o + 1024])
    ip, d = 0x0B123400, 24
    assert f.add(ip, d, 99) == 0
    routes[(ip, d)] = 99
    probe = np.array([ip | 7, ip | 200], np.uint32)
    want_p = O.lpm4_bruteforce([(ip, d, nh) for (ip, d), nh in routes.items()], 3, probe)
    assert 99 in list(want_p) or len(routes) > 1
    assert np.array_equal(f.lookup_bulk(probe), want_p)


@SELECTIONS
def test_fib_lookup_threads(gpu, sel):
    """examples/cndpfwd/l3-fwd.c:85 calls cne_fib_lookup_bulk per burst from
    every forwarding thread on one FIB.  Small calls take a staging slot of
    their own (stream, mapped staging, completion flag) and overlap; large
    ones take the DMA path under the table lock.  Eight threads (more than
    fit without waiting for a slot at times) mixing 4-, 256-, 4096- and
    20000-key calls on an IPv4 and an IPv6 FIB each get exactly the single-
    threaded answer, which is brute-force LPM."""
    from cndp_amd import pktgen
    from cndp_amd.fib import Fib, Fib6, node_ip4_route_add
    f = Fib("thr4", N.CNE_FIB_DIR24_8, default_nh=1 << 16, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B,
            num_tbl8=256, lookup=sel)
    routes = pktgen.l3fwd_routes()
    for ip, d, nh in routes:
        node_ip4_route_add(f, ip, d, nh, 0)
    f6 = Fib6("thr6", N.CNE_FIB_TRIE, default_nh=0, max_routes=1024, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15,
              lookup=sel)
    for ip, d, i in pktgen.v6_routes():
        f6.add(ip, d, i)
    rng = np.random.default_rng(5)
    keys = rng.integers(0, 2**32, size=20000, dtype=np.uint64).astype(np.uint32)
    keys[::2] = (10 << 24) | (keys[::2] & 0x0003FFFF)
    keys6 = rng.integers(0, 256, size=(20000, 16), dtype=np.uint8)
    keys6[::2, :4] = [0x20, 0x01, 0x0d, 0xb8]
    want4 = f.lookup_bulk(keys)
    assert np.array_equal(want4, O.lpm4_bruteforce([(ip, d, (0 << 16) | nh) for ip, d, nh in routes], 1 << 16, keys))
    want6 = f6.lookup_bulk(keys6)
    assert np.array_equal(want6, O.lpm6_bruteforce(pktgen.v6_routes(), 0, keys6))
    errors = []

    def worker(w):
        r = np.random.default_rng(100 + w)
        try:
            for it in range(60):
                n = int(r.choice([4, 256, 256, 4096, 20000]))
                o = int(r.integers(0, 20000 - n + 1))
                if (w + it) % 2:
                    got = f.lookup_bulk(keys[o:o + n])
                    ok = np.array_equal(got, want4[o:o + n])
                else:
                    got = f6.lookup_bulk(keys6[o:o + n])
                    ok = np.array_equal(got, want6[o:o + n])
                if not ok:
                    errors.append((w, it, n, o))
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    th = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]


def _sync_stats(f):
    b, c = ctypes.c_uint64(), ctypes.c_uint64()
    assert N.lib().cndp_fib_sync_stats(f.h, ctypes.byref(b), ctypes.byref(c)) == 0
    return b.value, c.value


@pytest.mark.parametrize("nh_sz", [N.CNE_FIB_DIR24_8_1B, N.CNE_FIB_DIR24_8_2B, N.CNE_FIB_DIR24_8_4B,
                                   N.CNE_FIB_DIR24_8_8B])
def test_fib_device_paint(gpu, nh_sz):
    """Route changes between GPU lookups are painted on the device (SURVEY §8(f)
    row 4): a /8 and /24s at both ends of the address space plus a /28 and a
    /32 inside one tbl8 group cost fill / copy commands over their own ranges
    (cndp_fib_sync_stats), not the 14.6 M-entry span between them; deletes the
    same; more than 1024 separate ranges take the bounding copy.  After every
    step all answers of the GPU selection equal brute-force LPM."""
    from cndp_amd.fib import Fib
    esz = 1 << nh_sz
    f = Fib(f"paint{nh_sz}", N.CNE_FIB_DIR24_8, default_nh=3, max_routes=4096, nh_sz=nh_sz, num_tbl8=64,
            lookup=N.CNE_FIB_LOOKUP_GPU)
    routes = {}
    rng = np.random.default_rng(11 + nh_sz)
    keys = rng.integers(0, 2**32, size=1 << 15, dtype=np.uint64).astype(np.uint32)

    def add(ip, d, nh):
        assert f.add(ip, d, nh) == 0
        routes[(ip, d)] = nh

    def check(extra=()):
        k = np.concatenate([keys, np.array([ip | off for (ip, d) in routes for off in (0, 1, 15, 255)]
                                           + list(extra), np.uint64).astype(np.uint32)])
        want = O.lpm4_bruteforce([(ip, d, nh) for (ip, d), nh in routes.items()], 3, k)
        assert np.array_equal(f.lookup_bulk(k), want)

    add(0x0A000000, 16, 4)
    check()                                  # the first lookup copies the new mirror whole
    b0, c0 = _sync_stats(f)
    assert b0 >= (1 << 24) * esz and c0 == 0
    add(0x01000000, 8, 5)
    add(0xDFFFFF00, 24, 6)
    add(0x00000100, 24, 7)
    add(0x0A010210, 28, 8)
    add(0x0A010221, 32, 9)
    check()
    b1, c1 = _sync_stats(f)
    assert 0 < c1 - c0 < 64 and b1 - b0 < 64 * 1024, (b1 - b0, c1 - c0)
    for key in ((0x01000000, 8), (0x0A010221, 32)):
        assert f.delete(*key) == 0
        del routes[key]
    check([0x01020304, 0x0A010221])
    b2, c2 = _sync_stats(f)
    assert 0 < c2 - c1 < 64 and b2 - b1 < 64 * 1024, (b2 - b1, c2 - c1)
    # 300 scattered /24s are painted; 1100 are more ranges than the log keeps:
    # the bounding copy
    for _ in range(300):
        ip, nh = int(rng.integers(0, 1 << 24)) << 8, int(rng.integers(0, 100))
        if (ip, 24) not in routes:
            add(ip, 24, nh)
    check()
    b2b, c2b = _sync_stats(f)
    assert c2b - c2 >= 250 and b2b - b2 < 64 * 1024
    b2, c2 = b2b, c2b
    for _ in range(1100):
        ip, nh = int(rng.integers(0, 1 << 24)) << 8, int(rng.integers(0, 100))
        if (ip, 24) not in routes:
            add(ip, 24, nh)
    check()
    b3, c3 = _sync_stats(f)
    assert c3 == c2 and b3 - b2 > 1 << 20


def test_fib6_device_paint(gpu):
    """The trie mirror under churn: the lpm6_1000 rules (lpm6_data_test.h) are
    loaded, looked up on the GPU (the new mirror is copied whole), then
    deleted and re-added in small batches between GPU lookups -- each sync
    paints only those routes' tbl24 / tbl8 ranges (cndp_fib6_sync_stats) --
    with every answer against brute-force LPM and the reference's golden next
    hops at the end."""
    import os
    from cndp_amd.fib import Fib6
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "lpm6_1000.npz"))
    f6 = Fib6("paint6", N.CNE_FIB_TRIE, default_nh=0, max_routes=2000, nh_sz=N.CNE_FIB_TRIE_4B,
              num_tbl8=1 << 14, lookup=N.CNE_FIB_LOOKUP_GPU)
    rules = [(bytes(ip), int(d), int(nh)) for ip, d, nh in zip(g["rule_ip"], g["rule_depth"], g["rule_nh"])]
    for ip, d, nh in rules:
        assert f6.add(ip, d, nh) == 0
    keys = g["ip"][:4000]
    assert np.array_equal(f6.lookup_bulk(keys), g["nh"][:4000].astype(np.uint64))

    def stats():
        b, c = ctypes.c_uint64(), ctypes.c_uint64()
        assert N.lib().cndp_fib6_sync_stats(f6.h, ctypes.byref(b), ctypes.byref(c)) == 0
        return b.value, c.value

    rng = np.random.default_rng(8)
    live = {(ip, d): nh for ip, d, nh in rules}
    b0, c0 = stats()
    painted = 0
    for step in range(6):
        pick = rng.choice(len(rules), size=5, replace=False)
        for k in pick:
            ip, d, nh = rules[k]
            if (ip, d) in live:
                assert f6.delete(ip, d) == 0
                del live[(ip, d)]
            else:
                assert f6.add(ip, d, nh) == 0
                live[(ip, d)] = nh
        want = O.lpm6_bruteforce([(ip, d, nh) for (ip, d), nh in live.items()], 0, keys)
        assert np.array_equal(f6.lookup_bulk(keys), want)
        b1, c1 = stats()
        painted += c1 > c0
        assert b1 - b0 < (1 << 20), (step, b1 - b0)  # never the 64 MiB+ bounding copy
        b0, c0 = b1, c1
    assert painted >= 4
    for (ip, d, nh) in rules:
        if (ip, d) not in live:
            assert f6.add(ip, d, nh) == 0
    assert np.array_equal(f6.lookup_bulk(g["ip"]), g["nh"].astype(np.uint64))
