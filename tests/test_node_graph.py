"""The GPU ip4_lookup graph node (cndp_amd/node/ip4_lookup_gpu.c), compiled
against the test-only graph stand-in (tests/node_harness) and driven the way
cne_graph_walk drives a node: bursts into process(), the source node once per
walk.  Checks the node registry (names, edges, source flag), the loud failure
without a GPU, and -- on the GPU -- that every mbuf leaves by the edge and with
the node_mbuf_priv1 the reference ip4_lookup gives it (ip4_lookup.c:48-256),
routes added through the exported cne_node_ip4_route_add."""
import ctypes
import os

import numpy as np
import pytest

from cndp_amd import native as N

HERE = os.path.dirname(os.path.abspath(__file__))
HARNESS = os.path.join(HERE, "node_harness", "libnode_harness.so")


def _harness():
    if not os.path.exists(HARNESS):
        pytest.skip("node harness not built (build() makes it)")
    N.lib()  # the same libcndp_gpu.so instance the harness links
    H = ctypes.CDLL(HARNESS)
    H.harness_node_info.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_char_p)]
    H.harness_process.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint16]
    H.harness_take.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32]
    H.harness_take.restype = ctypes.c_uint32
    H.harness_count.restype = ctypes.c_uint32
    H.harness_enqueue_calls.restype = ctypes.c_uint64
    return H


def test_node_registry():
    """Same node name and edges as ip4_lookup.c:345-359, plus the drain source
    node the "ip4*" pattern of l3fwd-graph (fwd.c:128) also picks up."""
    H = _harness()
    info = {}
    name = ctypes.create_string_buffer(64)
    fl, ne = ctypes.c_uint64(), ctypes.c_int()
    e0, e1 = ctypes.c_char_p(), ctypes.c_char_p()
    n = H.harness_node_info(0, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
    for i in range(n):
        H.harness_node_info(i, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
        info[name.value.decode()] = (fl.value, ne.value, e0.value, e1.value)
    assert info["ip4_lookup"] == (0, 2, b"ip4_rewrite", b"pkt_drop")
    assert info["ip4_lookup_gpu_drain"] == (1, 2, b"ip4_rewrite", b"pkt_drop")
    assert info["ip4_rewrite"] == (0, 1, b"pkt_drop", None)
    assert all(k.startswith("ip4") for k in info)


def test_node_init_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    H = _harness()
    assert H.harness_graph_create(0) == -19   # -ENODEV: there is no CPU path behind the node
    assert H.harness_priv1_offset() == 56      # offsetof(pktmbuf_t, udata64), set as ip4_lookup_node_init does


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, False, "driver_writes"])
def test_node_graph_walk(gpu, zero_copy):
    """driver_writes: zero-copy with each burst's mbuf headers written first as
    a graph on this lcore leaves them -- xskdev's data_len / data_off stores
    (xskdev.c:296-297) and pktdev_rx's soft parse (packet_type,
    pktdev_rx.c:36-101) -- so the device reads header lines held dirty in the
    host core's cache."""
    from cndp_amd import pktgen
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    from cndp_amd.mbuf import MbufPool
    from oracle import oracle as O
    import torch
    H = _harness()
    L = N.lib()
    NodeFib.fini()
    L.cndp_node_gpu_umem_reset()
    n = 30000
    pool = MbufPool(n)
    a = pktgen.packed_ipv4(n, routes=pktgen.l3fwd_routes(), seed=77)
    f = pktgen.fuzz_frames(n, seed=78, slot=64)
    slab = a.slab.view(n, 64).clone()
    fz = torch.zeros(n * 64, dtype=torch.uint8)
    fz[: f.slab.numel()] = f.slab
    slab[torch.arange(n) % 6 == 1] = fz.view(n, 64)[torch.arange(n) % 6 == 1]
    pool.fill(pktgen.Frames(slab.reshape(-1), n, stride=64))
    if zero_copy:
        assert L.cndp_node_gpu_umem_add(pool.base, pool.mem.nbytes) == 0
    dw = zero_copy == "driver_writes"
    H.harness_driver_writes.argtypes = [ctypes.c_int]
    H.harness_rx_parse.argtypes = [ctypes.c_int]
    H.harness_driver_writes(int(dw))
    H.harness_rx_parse(int(dw))
    os.environ["CNDP_GPU_BATCH"] = "2048"
    os.environ["CNDP_GPU_DEPTH"] = "3"
    try:
        assert H.harness_graph_create(3) == 0
        # routes after graph create, as l3fwd-graph does (fwd.c:160-201)
        routes = pktgen.l3fwd_routes()
        for ip, d, nh in routes:
            assert cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE) == 0
        rng = np.random.default_rng(1)
        order = rng.permutation(n)
        pos = 0
        while pos < n:
            b = int(min(n - pos, rng.choice([256, 256, 200, 31, 1])))
            ptrs = pool.ptrs(order[pos:pos + b])
            assert H.harness_process(b"ip4_lookup", ptrs, b) == b
            H.harness_walk_sources()
            pos += b
        for _ in range(100000):   # later walks drain the rest (flush on idle)
            if H.harness_count(0) + H.harness_count(1) == n:
                break
            H.harness_walk_sources()
        got = []
        for k in (0, 1):
            cnt = H.harness_count(k)
            buf = (ctypes.c_void_p * max(cnt, 1))()
            H.harness_take(k, buf, cnt)
            got.append(pool.index_of([x for x in buf[:cnt]]))
        assert H.harness_count(2) == 0
        assert len(got[0]) + len(got[1]) == n
    finally:
        H.harness_driver_writes(0)
        H.harness_rx_parse(0)
        H.harness_graph_destroy()
        os.environ.pop("CNDP_GPU_BATCH", None)
        os.environ.pop("CNDP_GPU_DEPTH", None)
        L.cndp_node_gpu_umem_reset()
    vals = [(ip, d, nh) for ip, d, nh in routes]
    t24, t8 = O.dir24_8_build(vals, N.IP4_LOOKUP_NEXT_PKT_DROP << 16, 256)
    d = pool.data_pos().astype(np.int64)
    bb = pool.mem
    dip = np.zeros(n, np.uint32)
    for k in range(4):
        dip = (dip << 8) | bb[d + 30 + k].astype(np.uint32)
    val = O.dir24_8_lookup(t24, t8, dip).astype(np.uint64)
    ttl = bb[d + 22].astype(np.uint64)
    ck = bb[d + 24].astype(np.uint64) | (bb[d + 25].astype(np.uint64) << 8)
    assert np.array_equal(pool.hdr["udata64"], (val & 0xFFFF) | (ttl << 16) | (ck << 32))
    if dw:  # the soft parse's packet_type, written by the host, survived the node
        et = (bb[d + 12].astype(np.uint32) << 8) | bb[d + 13]
        assert np.array_equal(pool.hdr["packet_type"], np.where(et == 0x0800, 0x90, np.where(et == 0x86DD, 0xE0, 0)))
    for k in (0, 1):
        assert np.all((val[got[k]] >> 16) == k)
        # each edge's stream keeps the arrival order (a subsequence of it)
        rank = np.empty(n, np.int64)
        rank[order] = np.arange(n)
        assert np.all(np.diff(rank[got[k]]) > 0)
    assert len(got[0]) > 0 and len(got[1]) > 0
    NodeFib.fini()


# ---- the cnet receive node (cndp_amd/node/eth_rx_gpu.c) -------------------
CNET_HARNESS = os.path.join(HERE, "node_harness", "libcnet_harness.so")
ETH_RX_EDGES = [b"pkt_drop", b"punt_kernel", b"punt_l2_kernel", b"gtpu_input", b"ip4_forward", b"ip4_proto",
                b"ip6_forward", b"ip6_proto", b"ptype"]


def _cnet_harness():
    if not os.path.exists(CNET_HARNESS):
        pytest.skip("cnet node harness not built (build() makes it)")
    N.lib()
    H = ctypes.CDLL(CNET_HARNESS)
    H.harness_node_info.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_char_p)]
    H.harness_node_edges.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    H.harness_take_edge.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32]
    H.harness_take_edge.restype = ctypes.c_uint32
    H.harness_rx_load.argtypes = [ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint32]
    H.harness_rx_left.restype = ctypes.c_uint32
    H.harness_cnet_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    H.harness_eth_rx_port.argtypes = [ctypes.c_uint32, ctypes.c_uint16]
    H.harness_walk_until.argtypes = [ctypes.c_uint64]
    H.harness_walk_until.restype = ctypes.c_double
    H.harness_total.restype = ctypes.c_uint64
    return H


def test_cnet_node_registry():
    """The node replacing lib/cnet/eth/eth_rx.c: registered as "eth_rx", a
    source node (eth_rx.c:171-190) that pkt_ctrl.c clones per port; its edges
    are the next nodes of ptype (ptype.c:213-230), ip4_input (ip4_input.c:274-287)
    and ip6_input (ip6_input.c:275-288), plus ptype itself, which keeps the
    replaced nodes reachable in the graph."""
    H = _cnet_harness()
    name = ctypes.create_string_buffer(64)
    fl, ne = ctypes.c_uint64(), ctypes.c_int()
    e0, e1 = ctypes.c_char_p(), ctypes.c_char_p()
    # (node 0; tests that register the replaced input nodes add more after it)
    assert H.harness_node_info(0, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1)) >= 1
    assert name.value == b"eth_rx" and fl.value == 1 and ne.value == len(ETH_RX_EDGES)
    names = (ctypes.c_char_p * 16)()
    k = H.harness_node_edges(0, names, 16)
    assert list(names[:k]) == ETH_RX_EDGES


def test_cnet_node_init_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from helpers import cnet_fibs
    H = _cnet_harness()
    assert H.harness_graph_create(0) == -22      # no cnet instance: -EINVAL
    fib, fib6 = cnet_fibs()[:2]
    H.harness_cnet_set(fib.h, fib6.h)
    assert H.harness_graph_create(0) == -19      # -ENODEV: no CPU path behind the node
    H.harness_graph_destroy()


def _edge_of_queue_code(e):
    """eth_rx_gpu.c rx_edge: the queue's CNDP_MQ_EDGE(node, e) -> this node's edge."""
    node, x = e >> 8, e & 0xFF
    if node == N.CNDP_MQ_NODE_IP4:
        return {1: 4, 2: 5}.get(x, 0)
    if node == N.CNDP_MQ_NODE_IP6:
        return {1: 6, 2: 7}.get(x, 0)
    return {1: 1, 2: 2, 5: 3}.get(x, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, "device_headers", False, "driver_writes",
                                       "driver_writes_device_headers"])
def test_cnet_node_graph_walk(gpu, zero_copy):
    """Graph walks over the GPU eth_rx node: it pulls 256-mbuf bursts from its
    port, and every mbuf leaves by the edge the reference's ptype /
    ip4_input / ip6_input would have sent it to, with the fields eth_rx and the
    input nodes write (the oracle over the same bursts, node state from 0).
    Zero-copy with the node's default host headers, and with the device
    reading them (CNDP_GPU_MQ_FLAGS=4, CNDP_MQ_F_DEVICE_HEADERS); driver_writes*:
    the same with the receive stub writing each mbuf's data_len / data_off as
    xskdev's receive does (xskdev.c:296-297), so eth_rx gets header lines
    dirty in the host core's cache, as in a real graph (eth_rx.c:111-131)."""
    from helpers import CNET_DEF, cnet_fibs
    from oracle import oracle as O
    from test_gpu_mq import _bursts, _cnet_expect, cnet_check, cnet_pool
    H = _cnet_harness()
    L = N.lib()
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    n, port = 24000, 3
    pool, orig = cnet_pool(n, routes, v6, bool(zero_copy))
    ref = _cnet_expect(pool, np.arange(n), _bursts(n, 0, "full"), t4, t6, 0, port)
    L.cndp_node_gpu_umem_reset()
    if zero_copy in ("device_headers", "driver_writes_device_headers"):
        os.environ["CNDP_GPU_MQ_FLAGS"] = str(N.CNDP_MQ_F_DEVICE_HEADERS)
    if zero_copy:
        L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes))
    H.harness_rx_driver_writes.argtypes = [ctypes.c_int]
    H.harness_rx_driver_writes(int(str(zero_copy).startswith("driver_writes")))
    H.harness_cnet_set(fib.h, fib6.h)
    assert H.harness_eth_rx_port(0, port) == 0
    ptrs = pool.ptrs(np.arange(n))
    assert H.harness_rx_load(port, ptrs, n) == 0
    try:
        assert H.harness_graph_create(5) == 0
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
        assert H.harness_walk_until(n) >= 0
        assert H.harness_rx_left(port) == 0 and H.harness_total() == n
        got = np.full(n, -1, np.int64)
        buf = (ctypes.c_void_p * n)()
        for k, name in enumerate(ETH_RX_EDGES):
            m = H.harness_take_edge(name, buf, n)
            idx = pool.index_of(np.array([x or 0 for x in buf[:m]], np.uint64))
            assert np.all(np.diff(idx) > 0), f"{name}: out of receive order"
            got[idx] = k
    finally:
        H.harness_rx_driver_writes(0)
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
        H.harness_graph_destroy()
        L.cndp_node_gpu_umem_reset()
    want_e = cnet_check(pool, orig, ref, t4, t6, port)
    want = np.array([_edge_of_queue_code(int(e)) for e in want_e])
    assert np.array_equal(got, want)
    assert set(np.unique(got).tolist()) >= {0, 3, 4, 6}   # drop, gtpu_input, ip4_forward, ip6_forward


@pytest.mark.gpu
@pytest.mark.parametrize("sel", [N.CNE_FIB_LOOKUP_DEFAULT, N.CNE_FIB_LOOKUP_GPU], ids=["host", "gpu"])
def test_cnet_node_with_sync_fib_callers(gpu, sel):
    """The link swap of INTEGRATION.md §3 as cnet runs it: the GPU eth_rx node
    is bound to this_cnet's rt4 FIB while, on other threads, an
    ip4_forward-style caller looks up 4 destinations per cne_fib_lookup_bulk
    call in that same FIB (ip4_forward.c:134-178) and an ARP-style caller one
    key per call in an arp-fib of /32 host entries (cnet_arp.c:77,195,
    ip4_output.c:118).  In either selection of cne_fib_select_lookup every
    synchronous answer equals brute-force LPM and every mbuf leaves the node
    by the oracle's edge."""
    import threading
    from cndp_amd.fib import Fib
    from helpers import CNET_DEF, cnet_fibs
    from oracle import oracle as O
    from test_gpu_mq import _bursts, _cnet_expect, cnet_check, cnet_pool
    H = _cnet_harness()
    H.harness_fib_caller.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32]
    L = N.lib()
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    assert fib.select_lookup(sel) == 0
    arp = Fib("arp-fib", N.CNE_FIB_DIR24_8, default_nh=CNET_DEF, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B,
              num_tbl8=256, lookup=sel)
    arp_routes = [((10 << 24) | (200 << 16) | i, 32, i) for i in range(1024)]
    for ip, d, nh in arp_routes:
        assert arp.add(ip, d, nh) == 0
    rng = np.random.default_rng(12)
    k4 = rng.integers(0, 2**32, size=8192, dtype=np.uint64).astype(np.uint32)
    k4[::2] = np.array([ip for ip, _, _ in routes], np.uint32)[rng.integers(0, len(routes), 4096)] | \
        rng.integers(0, 256, 4096).astype(np.uint32)
    ka = ((10 << 24) | (200 << 16) | rng.integers(0, 1100, size=4096)).astype(np.uint32)
    want4 = O.lpm4_bruteforce([(ip, d, nh) for ip, d, nh in v4vals], CNET_DEF, k4)
    wanta = O.lpm4_bruteforce(arp_routes, CNET_DEF, ka)
    out4 = np.zeros(k4.size, np.uint64)
    outa = np.zeros(ka.size, np.uint64)
    rcs = {}

    def caller(tag, f, keys, out, per_call):
        rcs[tag] = H.harness_fib_caller(f.h, keys.ctypes.data, out.ctypes.data, keys.size, per_call, 20)

    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    n, port = 24000, 3
    pool, orig = cnet_pool(n, routes, v6, True)
    ref = _cnet_expect(pool, np.arange(n), _bursts(n, 0, "full"), t4, t6, 0, port)
    L.cndp_node_gpu_umem_reset()
    L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes))
    H.harness_cnet_set(fib.h, fib6.h)
    assert H.harness_eth_rx_port(0, port) == 0
    assert H.harness_rx_load(port, pool.ptrs(np.arange(n)), n) == 0
    th = [threading.Thread(target=caller, args=("fwd4", fib, k4, out4, 4)),
          threading.Thread(target=caller, args=("arp1", arp, ka, outa, 1))]
    try:
        assert H.harness_graph_create(5) == 0
        for t in th:
            t.start()
        assert H.harness_walk_until(n) >= 0
        for t in th:
            t.join()
        assert H.harness_rx_left(port) == 0 and H.harness_total() == n
        got = np.full(n, -1, np.int64)
        buf = (ctypes.c_void_p * n)()
        for k, name in enumerate(ETH_RX_EDGES):
            m = H.harness_take_edge(name, buf, n)
            got[pool.index_of(np.array([x or 0 for x in buf[:m]], np.uint64))] = k
    finally:
        H.harness_graph_destroy()
        L.cndp_node_gpu_umem_reset()
    assert rcs == {"fwd4": 0, "arp1": 0}
    assert np.array_equal(out4, want4)
    assert np.array_equal(outa, wanta)
    want_e = cnet_check(pool, orig, ref, t4, t6, port)
    assert np.array_equal(got, np.array([_edge_of_queue_code(int(e)) for e in want_e]))


@pytest.mark.gpu
def test_cnet_node_stats(gpu):
    """With ptype, ip4_input and ip6_input in the graph (as cnet registers
    them), the GPU eth_rx node credits their walk stats
    (cne_graph_worker.h:156-160) with what they would have processed: ptype
    every mbuf, each input node the mbufs the ptype node routed to it."""
    from helpers import CNET_DEF, cnet_fibs
    from oracle import oracle as O
    from test_gpu_mq import _bursts, _cnet_expect, cnet_check, cnet_pool
    H = _cnet_harness()
    H.harness_node_stats.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(ctypes.c_uint64)]
    H.harness_register_input_nodes()
    L = N.lib()
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    n, port = 20000, 2
    pool, orig = cnet_pool(n, routes, v6, True)
    ref = _cnet_expect(pool, np.arange(n), _bursts(n, 0, "full"), t4, t6, 0, port)
    L.cndp_node_gpu_umem_reset()
    L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes))
    H.harness_cnet_set(fib.h, fib6.h)
    assert H.harness_eth_rx_port(0, port) == 0
    assert H.harness_rx_load(port, pool.ptrs(np.arange(n)), n) == 0
    stats = {}
    try:
        assert H.harness_graph_create(6) == 0
        assert H.harness_walk_until(n) >= 0
        for name in (b"ptype", b"ip4_input", b"ip6_input"):
            c, o = ctypes.c_uint64(), ctypes.c_uint64()
            assert H.harness_node_stats(name, ctypes.byref(c), ctypes.byref(o)) == 0
            stats[name] = (c.value, o.value)
    finally:
        H.harness_graph_destroy()
        L.cndp_node_gpu_umem_reset()
    want_e = np.asarray(cnet_check(pool, orig, ref, t4, t6, port), np.int64)
    node = want_e >> 8
    assert stats[b"ptype"][1] == n and stats[b"ptype"][0] >= 1
    assert stats[b"ip4_input"][1] == int((node == N.CNDP_MQ_NODE_IP4).sum()) > 0
    assert stats[b"ip6_input"][1] == int((node == N.CNDP_MQ_NODE_IP6).sum()) > 0


def test_cnet_node_edges_match_reference_names():
    """The GPU eth_rx node's edges are exactly the reference's next nodes of
    ptype (p_nxt edge ids -> ptype.c:213-230 names), ip4_input / ip6_input
    (their enums, ip{4,6}_input_priv.h) plus ptype, by the names in
    cnet_node_names.h; and cndp_node.h's input-edge ids and FIB next-index
    shift are the reference's (tests/golden/ptype_ref.json)."""
    import re
    from helpers import ptype_ref
    ref = ptype_ref()
    nm = ref["cnet_node_names"]
    assert ETH_RX_EDGES == [nm[k].encode() for k in (
        "PKT_DROP_NODE_NAME", "PUNT_KERNEL_NODE_NAME", "PUNT_ETHER_NODE_NAME", "GTPU_INPUT_NODE_NAME",
        "IP4_FORWARD_NODE_NAME", "IP4_PROTO_NODE_NAME", "IP6_FORWARD_NODE_NAME", "IP6_PROTO_NODE_NAME",
        "PTYPE_NODE_NAME")]
    hdr = open(os.path.join(HERE, "..", "include", "cndp_node.h")).read()
    val = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+(CNDP_\w+)\s+(\d+)", hdr)}
    inp = ref["input_next"]
    for fam in ("IP4", "IP6"):
        assert val["CNDP_INPUT_NEXT_PKT_DROP"] == inp[f"CNE_NODE_{fam}_INPUT_NEXT_PKT_DROP"]
        assert val["CNDP_INPUT_NEXT_FORWARD"] == inp[f"CNE_NODE_{fam}_INPUT_NEXT_FORWARD"]
        assert val["CNDP_INPUT_NEXT_PROTO"] == inp[f"CNE_NODE_{fam}_INPUT_NEXT_PROTO"]
    assert val["CNDP_RT_NEXT_INDEX_SHIFT"] == ref["next_index_shift"]["RT4_NEXT_INDEX_SHIFT"] \
        == ref["next_index_shift"]["RT6_NEXT_INDEX_SHIFT"]
    # the ptype edge ids the queue reports (eth_rx_gpu.c PT_NEXT_*) are ptype_priv.h's
    src = open(os.path.join(HERE, "..", "cndp_amd", "node", "eth_rx_gpu.c")).read()
    pt = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+PT_NEXT_(\w+)\s+(\d+)", src)}
    for k, v in pt.items():
        assert ref["ptype_next"]["PTYPE_NEXT_" + k] == v, k


@pytest.mark.gpu
def test_cnet_node_clones_per_port(gpu):
    """Two ports, one eth_rx clone each (cne_node_clone + the {port, nid}
    list, as pkt_ctrl.c:55-72 sets them up): every mbuf leaves by its edge
    with lport = its port, and each clone keeps its own ptype-node state
    (the oracle runs the two ports' burst streams separately)."""
    from helpers import CNET_DEF, cnet_fibs
    from oracle import oracle as O
    from test_gpu_mq import _bursts, _cnet_expect, cnet_check, cnet_pool
    H = _cnet_harness()
    H.harness_clone.restype = ctypes.c_uint32
    H.harness_clone.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L = N.lib()
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    n = 16000
    half = n // 2 + 100   # the ports' streams end on different burst boundaries
    pool, orig = cnet_pool(n, routes, v6, zero_copy=False)
    parts = ((3, np.arange(half)), (5, np.arange(half, n)))
    refs = [_cnet_expect(pool, idx, _bursts(len(idx), 0, "full"), t4, t6, 0, p) for p, idx in parts]
    ref = {k: np.concatenate([r[k] for r in refs]) for k in refs[0]}
    L.cndp_node_gpu_umem_reset()
    H.harness_cnet_set(fib.h, fib6.h)
    assert H.harness_eth_rx_port(0, 7) == 0   # the parent node (also in the graph here) on an idle port
    try:
        for p, idx in parts:
            nid = H.harness_clone(b"eth_rx", str(p).encode())
            assert nid != 0xFFFFFFFF
            assert H.harness_eth_rx_port(nid, p) == 0
            assert H.harness_rx_load(p, pool.ptrs(idx), len(idx)) == 0
        assert H.harness_graph_create(7) == 0
        assert H.harness_walk_until(n) >= 0
        assert H.harness_rx_left(3) == 0 and H.harness_rx_left(5) == 0 and H.harness_total() == n
        got = np.full(n, -1, np.int64)
        buf = (ctypes.c_void_p * n)()
        for k, name in enumerate(ETH_RX_EDGES):
            m = H.harness_take_edge(name, buf, n)
            got[pool.index_of(np.array([x or 0 for x in buf[:m]], np.uint64))] = k
    finally:
        H.harness_graph_destroy()
        H.harness_drop_clones()
    lport = np.concatenate([np.full(len(idx), p) for p, idx in parts])
    want_e = cnet_check(pool, orig, ref, t4, t6, lport)
    want = np.array([_edge_of_queue_code(int(e)) for e in want_e])
    assert np.array_equal(got, want)


# ---- the GPU ip4_rewrite node (cndp_amd/node/ip4_rewrite_gpu.c) -----------
def _rw_harness():
    H = _harness()
    H.cne_node_edge_update.restype = ctypes.c_uint16
    H.cne_node_edge_update.argtypes = [ctypes.c_uint32, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint16]
    H.cne_node_edge_count.restype = ctypes.c_uint16
    H.cne_node_edge_count.argtypes = [ctypes.c_uint32]
    H.harness_node_edges.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    H.harness_take_edge.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32]
    H.harness_take_edge.restype = ctypes.c_uint32
    return H


def _node_ids(H):
    name = ctypes.create_string_buffer(64)
    fl, ne = ctypes.c_uint64(), ctypes.c_int()
    e0, e1 = ctypes.c_char_p(), ctypes.c_char_p()
    n = H.harness_node_info(0, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
    ids = {}
    for i in range(n):
        H.harness_node_info(i, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
        ids[name.value.decode()] = i
    return ids


def _eth_config(H, L, ports):
    """cne_node_eth_config's part for ip4_rewrite (pktdev_ctrl.c:75-86): a
    "pktdev_tx-<port>" edge added to ip4_rewrite per port, then
    ip4_rewrite_set_next(port, its edge index)."""
    rw = _node_ids(H)["ip4_rewrite"]
    for p in ports:
        nm = ctypes.c_char_p(f"pktdev_tx-{p}".encode())
        assert H.cne_node_edge_update(rw, 0xFFFF, ctypes.byref(nm), 1) != 0xFFFF
        assert L.ip4_rewrite_set_next(p, H.cne_node_edge_count(rw) - 1) == 0


def _edges_of(H, i):
    names = (ctypes.c_char_p * 16)()
    k = H.harness_node_edges(i, names, 16)
    return list(names[:k])


def test_rewrite_node_registry():
    """ip4_rewrite registered as ip4_rewrite.c:314-326 (edge 0 pkt_drop),
    plus its drain source node; the tx edges cne_node_eth_config adds to
    ip4_rewrite show up on the drain node too (the ip4_rewrite_set_next hook),
    so the edge index a next hop's tx_node names is the same on both."""
    H = _rw_harness()
    L = N.lib()
    ids = _node_ids(H)
    name = ctypes.create_string_buffer(64)
    fl, ne = ctypes.c_uint64(), ctypes.c_int()
    e0, e1 = ctypes.c_char_p(), ctypes.c_char_p()
    H.harness_node_info(ids["ip4_rewrite"], name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0),
                        ctypes.byref(e1))
    assert (fl.value, ne.value, e0.value) == (0, 1, b"pkt_drop")
    H.harness_node_info(ids["ip4_rewrite_gpu_drain"], name, ctypes.byref(fl), ctypes.byref(ne),
                        ctypes.byref(e0), ctypes.byref(e1))
    assert (fl.value, ne.value, e0.value) == (1, 1, b"pkt_drop")
    L.cndp_node_ip4_rewrite_reset()
    try:
        _eth_config(H, L, (0, 3))
        want = [b"pkt_drop", b"pktdev_tx-0", b"pktdev_tx-3"]
        assert _edges_of(H, ids["ip4_rewrite"]) == want
        assert _edges_of(H, ids["ip4_rewrite_gpu_drain"]) == want
        # the table behind cne_node_ip4_rewrite_add takes the tx edge of the port
        data = (ctypes.c_uint8 * 12)(*range(12))
        assert L.cne_node_ip4_rewrite_add(5, data, 12, 3) == 0
        tx = ctypes.c_uint16()
        assert L.cndp_node_ip4_rewrite_get(5, None, None, ctypes.byref(tx), None) == 0 and tx.value == 2
        assert L.cne_node_ip4_rewrite_add(6, data, 12, 1) == -22   # port 1 has no tx edge
    finally:
        H.harness_edges_reset()
        L.cndp_node_ip4_rewrite_reset()


def test_rewrite_edge_mirrors_every_library():
    """Both harness libraries loaded in one process (five hooks on
    ip4_rewrite_set_next: each library's ip4_lookup and ip4_rewrite, the
    receive node): every hook runs, so in each library ip4_rewrite's drain
    node and ip4_lookup (and its drain node) carry ip4_rewrite's edges after
    their own -- the edge indices the queues return mean the same there."""
    Hn, Hr = _rw_harness(), _rx_harness()
    L = N.lib()
    L.cndp_node_ip4_rewrite_reset()
    try:
        for H in (Hn, Hr):
            _eth_config(H, L, (0, 3))
        want = [b"pkt_drop", b"pktdev_tx-0", b"pktdev_tx-3"]
        for H in (Hn, Hr):
            ids = _node_ids(H)
            assert _edges_of(H, ids["ip4_rewrite"]) == want
            assert _edges_of(H, ids["ip4_rewrite_gpu_drain"]) == want
            for nm in ("ip4_lookup", "ip4_lookup_gpu_drain"):
                assert _edges_of(H, ids[nm]) == [b"ip4_rewrite", b"pkt_drop"] + want
        assert _edges_of(Hr, _node_ids(Hr)["pktdev_rx"]) == PKTDEV_RX_EDGES + want
    finally:
        for H in (Hn, Hr):
            H.harness_edges_reset()
        L.cndp_node_ip4_rewrite_reset()


def _rw_table(L, seed, ports):
    """Next hops through cne_node_ip4_rewrite_add (the process-global table the
    GPU node follows) and the oracle's copy of it."""
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    tbl = np.zeros(64, dtype=O.REWRITE_NH)
    for nh in range(64):
        if nh % 9 == 8:
            continue
        ln = int(rng.choice([12, 12, 12, 0, 14, 22, 26, 30, 56]))
        data = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
        k = nh % len(ports)
        assert L.cne_node_ip4_rewrite_add(nh, ctypes.create_string_buffer(data, max(ln, 1)), ln, ports[k]) == 0
        tbl[nh]["rewrite_len"], tbl[nh]["tx_node"], tbl[nh]["enabled"] = ln, k + 1, 1
        tbl[nh]["rewrite_data"][:ln] = np.frombuffer(data, np.uint8)
    return tbl


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, "host_headers", False])
def test_rewrite_node_graph_walk(gpu, zero_copy):
    """Bursts into the GPU ip4_rewrite node's process(), graph walks drain it:
    every mbuf leaves by its next hop's pktdev_tx-<port> edge (or pkt_drop),
    in order per edge, and every frame equals the oracle node loop's over the
    same bursts (rewrite data, TTL - 1, the 4-wide / tail checksum rule of
    each burst).  Zero-copy with the node's default device headers and with
    the host reading them (CNDP_GPU_MQ_FLAGS=0)."""
    from cndp_amd import pktgen
    from cndp_amd.mbuf import MbufPool
    from oracle import oracle as O
    H = _rw_harness()
    L = N.lib()
    ports = (0, 2, 5)
    n = 12000
    gp, op = MbufPool(n), MbufPool(n)
    rng = np.random.default_rng(61)
    ck = rng.integers(0, 1 << 16, n, dtype=np.uint64)
    ck[::5] = 0xFFFF
    ck[2::5] = 0xFFFE
    priv = rng.integers(0, 70, n, dtype=np.uint64) | (rng.integers(0, 256, n, dtype=np.uint64) << 16) | (ck << 32)
    for p in (gp, op):
        p.fill(pktgen.packed_ipv4(n, routes=pktgen.l3fwd_routes(), seed=62))
        p.hdr["udata64"] = priv
    L.cndp_node_ip4_rewrite_reset()
    L.cndp_node_gpu_umem_reset()
    if zero_copy:
        assert L.cndp_node_gpu_umem_add(ctypes.c_void_p(gp.base), ctypes.c_uint64(gp.mem.nbytes)) == 0
    os.environ["CNDP_GPU_BATCH"] = "2048"
    if zero_copy == "host_headers":
        os.environ["CNDP_GPU_MQ_FLAGS"] = "0"
    bursts = []
    try:
        _eth_config(H, L, ports)
        tbl = _rw_table(L, 63, ports)
        assert H.harness_graph_create(11) == 0
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
        pos = 0
        while pos < n:
            b = int(min(n - pos, rng.choice([256, 256, 256, 97, 4, 3, 1])))
            bursts.append(b)
            assert H.harness_process(b"ip4_rewrite", gp.ptrs(np.arange(pos, pos + b)), b) == b
            H.harness_walk_sources()
            pos += b
        names = [b"pkt_drop"] + [f"pktdev_tx-{p}".encode() for p in ports]
        buf = (ctypes.c_void_p * n)()
        for _ in range(200000):
            if sum(H.harness_take_edge(nm, buf, n) for nm in names) == n:
                break
            H.harness_walk_sources()
        got = np.full(n, -1, np.int64)
        for k, nm in enumerate(names):
            m = H.harness_take_edge(nm, buf, n)
            idx = gp.index_of(np.array([x or 0 for x in buf[:m]], np.uint64))
            assert np.all(np.diff(idx) > 0), f"{nm}: out of order"
            got[idx] = k
    finally:
        H.harness_graph_destroy()
        H.harness_edges_reset()
        L.cndp_node_ip4_rewrite_reset()
        L.cndp_node_gpu_umem_reset()
        os.environ.pop("CNDP_GPU_BATCH", None)
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
    want = np.zeros(n, np.int64)
    pos = 0
    for b in bursts:
        want[pos:pos + b] = O.ip4_rewrite_node(op.ptrs(np.arange(pos, pos + b)), b, tbl)
        pos += b
    assert np.array_equal(got, want)
    bad = np.nonzero(np.any(gp.mem.reshape(n, -1)[:, 64:] != op.mem.reshape(n, -1)[:, 64:], axis=1))[0]
    assert bad.size == 0, f"{bad.size} frames differ, first {bad[:4]}"
    assert set(np.unique(got).tolist()) == {0, 1, 2, 3}


@pytest.mark.gpu
@pytest.mark.parametrize("fused,burst", [(True, 256), (True, 600), (False, 256)],
                         ids=["rewrite_in_lookup", "rewrite_in_lookup_600", "rewrite_node"])
def test_l3fwd_graph_chain(gpu, fused, burst):
    """The l3fwd-graph chain with both GPU nodes, walked as cne_graph_walk
    runs it (ip4_lookup's enqueues fill ip4_rewrite's stream, which runs in
    the same walk): every mbuf ends at pkt_drop or its next hop's tx edge with
    priv1 and the rewritten frame of the reference chain.  rewrite_in_lookup
    (the zero-copy default): ip4_lookup's queue runs ip4_rewrite itself
    (CNDP_MQ_F_REWRITE) and its mbufs leave on the mirrored pktdev_tx edges,
    byte for byte the reference pair per 256-mbuf walk (the 4-wide / tail
    checksum rule of the stream each call sends ip4_rewrite), in order per
    edge, with ip4_rewrite's stats credited.  rewrite_node
    (CNDP_GPU_LOOKUP_REWRITE=0): the GPU ip4_rewrite node gets the stream,
    checked where the two checksum rules agree (not 0xFFFE / 0xFFFF, whose
    rule depends on the stream split).  _600: 600-mbuf process() calls (a
    graph whose pkt_cls gathered several ports' bursts), whose rewrite rule
    applies per 256-mbuf piece of the call."""
    from cndp_amd import pktgen
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    from cndp_amd.mbuf import MbufPool
    from oracle import oracle as O
    H = _rw_harness()
    H.harness_chain.argtypes = [ctypes.c_int]
    L = N.lib()
    ports = (0, 1, 2, 3)
    n = 20000
    gp, op = MbufPool(n), MbufPool(n)
    for p in (gp, op):
        p.fill(pktgen.packed_ipv4(n, routes=pktgen.l3fwd_routes(), seed=71))
        # header checksums 0xFFFE / 0xFFFF, where the two rules differ
        d = p.data_pos().astype(np.int64)
        for sel, lo in ((np.arange(n) % 97 == 5, 0xFE), (np.arange(n) % 89 == 7, 0xFF)):
            p.mem[d[sel] + 24] = lo
            p.mem[d[sel] + 25] = 0xFF
    NodeFib.fini()
    L.cndp_node_ip4_rewrite_reset()
    L.cndp_node_gpu_umem_reset()
    assert L.cndp_node_gpu_umem_add(ctypes.c_void_p(gp.base), ctypes.c_uint64(gp.mem.nbytes)) == 0
    os.environ["CNDP_GPU_BATCH"] = "4096"
    if not fused:
        os.environ["CNDP_GPU_LOOKUP_REWRITE"] = "0"
    routes = pktgen.l3fwd_routes()
    H.harness_node_stats.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(ctypes.c_uint64)]
    calls, objs = ctypes.c_uint64(), ctypes.c_uint64()
    try:
        _eth_config(H, L, ports)
        tbl = _rw_table(L, 72, ports)
        H.harness_chain(1)
        assert H.harness_graph_create(12) == 0
        for ip, d, nh in routes:
            assert cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE) == 0
        assert H.harness_drive(b"ip4_lookup", gp.ptrs(np.arange(n)), n, burst, 1) >= 0
        names = [b"pkt_drop"] + [f"pktdev_tx-{p}".encode() for p in ports]
        buf = (ctypes.c_void_p * n)()
        got = np.full(n, -1, np.int64)
        for k, nm in enumerate(names):
            m = H.harness_take_edge(nm, buf, n)
            idx = gp.index_of(np.array([x or 0 for x in buf[:m]], np.uint64))
            if fused:
                assert np.all(np.diff(idx) > 0), f"{nm}: out of order"
            got[idx] = k
        assert H.harness_node_stats(b"ip4_rewrite", ctypes.byref(calls), ctypes.byref(objs)) == 0
    finally:
        H.harness_chain(0)
        H.harness_graph_destroy()
        H.harness_edges_reset()
        L.cndp_node_ip4_rewrite_reset()
        L.cndp_node_gpu_umem_reset()
        os.environ.pop("CNDP_GPU_BATCH", None)
        os.environ.pop("CNDP_GPU_LOOKUP_REWRITE", None)
    # the reference chain on the oracle's copy: ip4_lookup then ip4_rewrite
    t24, t8 = O.dir24_8_build(list(routes), N.IP4_LOOKUP_NEXT_PKT_DROP << 16, 256)
    d = op.data_pos().astype(np.int64)
    dip = np.zeros(n, np.uint32)
    for k in range(4):
        dip = (dip << 8) | op.mem[d + 30 + k].astype(np.uint32)
    val = O.dir24_8_lookup(t24, t8, dip).astype(np.uint64)
    ck = op.mem[d + 24].astype(np.uint64) | (op.mem[d + 25].astype(np.uint64) << 8)
    op.hdr["udata64"] = (val & 0xFFFF) | (op.mem[d + 22].astype(np.uint64) << 16) | (ck << 32)
    assert np.array_equal(gp.hdr["udata64"], op.hdr["udata64"])
    rw = np.nonzero((val >> 16) == 0)[0]
    want = np.zeros(n, np.int64)
    if fused:  # ip4_rewrite per walk: the stream each ip4_lookup call (256-mbuf piece) sends it
        for c in range(0, n, burst):
            for b in range(c, min(c + burst, n), 256):
                sel = rw[(rw >= b) & (rw < min(b + 256, c + burst))]
                want[sel] = O.ip4_rewrite_node(op.ptrs(sel), len(sel), tbl)
        ok = np.ones(n, bool)
        assert calls.value > 0 and objs.value == rw.size
    else:
        want[rw] = O.ip4_rewrite_node(op.ptrs(rw), len(rw), tbl)
        ok = (ck != 0xFFFE) & (ck != 0xFFFF)
    assert np.array_equal(got, want)
    diff = np.any(gp.mem.reshape(n, -1)[:, 64:] != op.mem.reshape(n, -1)[:, 64:], axis=1)  # buffers (buf_addr differs)
    assert not np.any(diff & ok), f"{int((diff & ok).sum())} frames differ"
    assert rw.size > n // 2 and (got == 0).sum() > 0
    NodeFib.fini()


@pytest.mark.gpu
def test_l3fwd_fused_unreachable_mbufs(gpu):
    """ip4_lookup with ip4_rewrite in its queue, mbufs of an unregistered pool
    mixed into its calls: those leave by pkt_drop untouched (header, priv1,
    frame), are not counted for ip4_rewrite, and do not shift the checksum
    rule of the others -- each call's reachable mbufs sent to ip4_rewrite are
    rewritten as ip4_rewrite would over that stream."""
    from cndp_amd import pktgen
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    from cndp_amd.mbuf import MbufPool
    from oracle import oracle as O
    H = _rw_harness()
    H.harness_chain.argtypes = [ctypes.c_int]
    L = N.lib()
    ports = (0, 1, 2, 3)
    n, m = 6000, 600
    gp, op, xp = MbufPool(n), MbufPool(n), MbufPool(m)
    for p in (gp, op):
        p.fill(pktgen.packed_ipv4(n, routes=pktgen.l3fwd_routes(), seed=73))
        p.hdr["udata64"] = 0x77
        d = p.data_pos().astype(np.int64)
        for sel, lo in ((np.arange(n) % 31 == 5, 0xFE), (np.arange(n) % 37 == 7, 0xFF)):
            p.mem[d[sel] + 24] = lo
            p.mem[d[sel] + 25] = 0xFF
    xp.fill(pktgen.packed_ipv4(m, routes=pktgen.l3fwd_routes(), seed=74))
    xp.hdr["udata64"] = 0x99
    x_before = xp.mem.copy()
    # the call stream: every 11th slot an outsider
    seq, gi, xi = [], 0, 0
    while gi < n:
        if len(seq) % 11 == 10 and xi < m:
            seq.append(("x", xi)); xi += 1
        else:
            seq.append(("g", gi)); gi += 1
    ptrs = (ctypes.c_void_p * len(seq))()
    for k, (w, i) in enumerate(seq):
        ptrs[k] = (gp if w == "g" else xp).addr(i)
    NodeFib.fini()
    L.cndp_node_ip4_rewrite_reset()
    L.cndp_node_gpu_umem_reset()
    assert L.cndp_node_gpu_umem_add(ctypes.c_void_p(gp.base), ctypes.c_uint64(gp.mem.nbytes)) == 0
    os.environ["CNDP_GPU_BATCH"] = "2048"
    routes = pktgen.l3fwd_routes()
    try:
        _eth_config(H, L, ports)
        tbl = _rw_table(L, 75, ports)
        H.harness_chain(1)
        assert H.harness_graph_create(14) == 0
        for ip, dd, nh in routes:
            assert cne_node_ip4_route_add(ip, dd, nh, N.IP4_LOOKUP_NEXT_REWRITE) == 0
        assert H.harness_drive(b"ip4_lookup", ptrs, len(seq), 256, 1) >= 0
        names = [b"pkt_drop"] + [f"pktdev_tx-{p}".encode() for p in ports]
        buf = (ctypes.c_void_p * len(seq))()
        got = {}
        for k, nm in enumerate(names):
            for a in buf[:H.harness_take_edge(nm, buf, len(seq))]:
                got[a] = k
    finally:
        H.harness_chain(0)
        H.harness_graph_destroy()
        H.harness_edges_reset()
        L.cndp_node_ip4_rewrite_reset()
        L.cndp_node_gpu_umem_reset()
        os.environ.pop("CNDP_GPU_BATCH", None)
    assert len(got) == len(seq)
    assert all(got[xp.addr(i)] == 0 for i in range(xi))
    assert np.array_equal(xp.mem, x_before)
    # the reference pair over each 256-slot call's reachable mbufs
    t24, t8 = O.dir24_8_build(list(routes), N.IP4_LOOKUP_NEXT_PKT_DROP << 16, 256)
    d = op.data_pos().astype(np.int64)
    dip = np.zeros(n, np.uint32)
    for k in range(4):
        dip = (dip << 8) | op.mem[d + 30 + k].astype(np.uint32)
    val = O.dir24_8_lookup(t24, t8, dip).astype(np.uint64)
    ck = op.mem[d + 24].astype(np.uint64) | (op.mem[d + 25].astype(np.uint64) << 8)
    op.hdr["udata64"] = (val & 0xFFFF) | (op.mem[d + 22].astype(np.uint64) << 16) | (ck << 32)
    assert np.array_equal(gp.hdr["udata64"], op.hdr["udata64"])
    want = np.zeros(n, np.int64)
    for c in range(0, len(seq), 256):
        mine = np.array([i for w, i in seq[c:c + 256] if w == "g"], np.int64)
        sel = mine[(val[mine] >> 16) == 0]
        want[sel] = O.ip4_rewrite_node(op.ptrs(sel), len(sel), tbl)
    assert np.array_equal(np.array([got[gp.addr(i)] for i in range(n)]), want)
    diff = np.any(gp.mem.reshape(n, -1)[:, 64:] != op.mem.reshape(n, -1)[:, 64:], axis=1)
    assert not np.any(diff), f"{int(diff.sum())} frames differ"
    NodeFib.fini()


# ---- the l3fwd-graph receive chain node (cndp_amd/node/pktdev_rx_gpu.c) ------
RX_HARNESS = os.path.join(HERE, "node_harness", "librx_harness.so")
PKTDEV_RX_EDGES = [b"ip4_lookup", b"pkt_cls", b"ip4_rewrite", b"pkt_drop"]


def _rx_harness():
    if not os.path.exists(RX_HARNESS):
        pytest.skip("rx node harness not built (build() makes it)")
    N.lib()
    H = ctypes.CDLL(RX_HARNESS)
    H.harness_node_info.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_char_p)]
    H.harness_node_edges.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    H.harness_take_edge.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32]
    H.harness_take_edge.restype = ctypes.c_uint32
    H.harness_rx_load.argtypes = [ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint32]
    H.harness_rx_left.restype = ctypes.c_uint32
    H.harness_pktdev_rx_port.argtypes = [ctypes.c_uint32, ctypes.c_uint16]
    H.harness_walk_until.argtypes = [ctypes.c_uint64]
    H.harness_walk_until.restype = ctypes.c_double
    H.harness_node_stats.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(ctypes.c_uint64)]
    H.harness_chain.argtypes = [ctypes.c_int]
    H.cne_node_edge_update.restype = ctypes.c_uint16
    H.cne_node_edge_update.argtypes = [ctypes.c_uint32, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint16]
    H.cne_node_edge_count.restype = ctypes.c_uint16
    H.cne_node_edge_count.argtypes = [ctypes.c_uint32]
    H.harness_register_cls_node()
    return H


def test_rx_node_registry():
    """The node replacing lib/usr/clib/nodes/pktdev_rx.c: registered as
    "pktdev_rx", a source node (pktdev_rx.c:186-199) that pktdev_ctrl.c clones
    per port; its first two edges are the reference's (ip4_lookup, pkt_cls,
    pktdev_rx_priv.h), then the two it sends on (ip4_rewrite, pkt_drop)."""
    H = _rx_harness()
    ids = _node_ids(H)
    i = ids["pktdev_rx"]
    name = ctypes.create_string_buffer(64)
    fl, ne = ctypes.c_uint64(), ctypes.c_int()
    e0, e1 = ctypes.c_char_p(), ctypes.c_char_p()
    H.harness_node_info(i, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
    assert name.value == b"pktdev_rx" and fl.value == 1 and ne.value == 4
    # (after its own four: ip4_rewrite's edges, once ip4_rewrite_set_next ran)
    assert _edges_of(H, i)[:4] == PKTDEV_RX_EDGES
    assert {"ip4_lookup", "ip4_rewrite", "pkt_cls"} <= set(ids)


def test_rx_node_init_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    H = _rx_harness()
    assert H.harness_graph_create(0) == -19   # -ENODEV: there is no CPU path behind the node


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, "host_headers", "host_writeback", "device_headers_host_writeback",
                                       "no_rewrite", False, "driver_writes", "driver_writes_host_headers"])
def test_rx_node_graph_walk(gpu, zero_copy):
    """Graph walks over the GPU pktdev_rx node: it pulls 256-mbuf bursts from
    its port and every mbuf ends where l3fwd-graph's pktdev_rx -> pkt_cls ->
    ip4_lookup -> ip4_rewrite walk sends it (pkt_drop, or its next hop's tx
    edge) with the soft parse's packet_type, ip4_lookup's priv1 (IPv4 only)
    and the rewritten frame of the oracle chain; pkt_cls, ip4_lookup (and
    ip4_rewrite) get the stats of the mbufs they stand for.  Zero-copy, the
    node runs ip4_rewrite itself (CNDP_MQ_F_REWRITE), per receive burst as
    ip4_rewrite gets it in one call, so every frame matches the oracle's
    per-burst chain byte for byte; "no_rewrite" (CNDP_GPU_RX_REWRITE=0) and
    staged frames go on to the GPU ip4_rewrite node, whose bursts are its
    queue's polls (checksums 0xFFFE / 0xFFFF, whose rule depends on that
    split, not compared).  Mixed frames: routed IPv4, IPv6, VLAN, ARP, fuzz.
    driver_writes*: the receive stub writes each mbuf's data_len / data_off
    as xskdev's receive does (xskdev.c:296-297), so the node gets header lines
    dirty in the host core's cache, as pktdev_rx.c:107-125 does in a real
    graph.  host_writeback (CNDP_GPU_MQ_FLAGS=CNDP_MQ_F_HOST_WRITEBACK, with or
    without CNDP_MQ_F_DEVICE_HEADERS): the frames read and rewritten in place,
    packet_type and priv1 written by the node's polls from the queue's records."""
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    from cndp_amd.mbuf import MbufPool
    from cndp_amd import pktgen
    from oracle import oracle as O
    from test_gpu_mq import _mixed_l3_frames
    H = _rx_harness()
    L = N.lib()
    ports, port = (0, 1, 2, 3), 2
    n = 20000
    gp, op = MbufPool(n), MbufPool(n)
    fr = _mixed_l3_frames(n, seed=81)
    for p in (gp, op):
        p.fill(fr)
        p.hdr["udata64"] = 0x5A5A5A5A
        # header checksums 0xFFFE / 0xFFFF, where the 4-wide and tail rules of
        # ip4_rewrite differ (ip4_rewrite.c:97-110 / :209-216)
        d = p.data_pos().astype(np.int64)
        for sel, lo in ((np.arange(n) % 97 == 5, 0xFE), (np.arange(n) % 89 == 7, 0xFF)):
            p.mem[d[sel] + 24] = lo
            p.mem[d[sel] + 25] = 0xFF
    # the header checksums before the rewrite (the rule-dependent ones)
    d = op.data_pos().astype(np.int64)
    ck = op.mem[d + 24].astype(np.uint64) | (op.mem[d + 25].astype(np.uint64) << 8)
    NodeFib.fini()
    L.cndp_node_ip4_rewrite_reset()
    L.cndp_node_gpu_umem_reset()
    if zero_copy:
        assert L.cndp_node_gpu_umem_add(ctypes.c_void_p(gp.base), ctypes.c_uint64(gp.mem.nbytes)) == 0
    os.environ["CNDP_GPU_BATCH"] = "4096"
    if zero_copy in ("host_headers", "driver_writes_host_headers"):
        os.environ["CNDP_GPU_MQ_FLAGS"] = "0"
    if zero_copy == "host_writeback":
        os.environ["CNDP_GPU_MQ_FLAGS"] = str(N.CNDP_MQ_F_HOST_WRITEBACK)
    if zero_copy == "device_headers_host_writeback":
        os.environ["CNDP_GPU_MQ_FLAGS"] = str(N.CNDP_MQ_F_HOST_WRITEBACK | N.CNDP_MQ_F_DEVICE_HEADERS)
    if zero_copy == "no_rewrite":
        os.environ["CNDP_GPU_RX_REWRITE"] = "0"
    fused = zero_copy in (True, "host_headers", "host_writeback", "device_headers_host_writeback", "driver_writes",
                          "driver_writes_host_headers")
    H.harness_rx_driver_writes.argtypes = [ctypes.c_int]
    H.harness_rx_driver_writes(int(str(zero_copy).startswith("driver_writes")))
    routes = pktgen.l3fwd_routes()
    ids = _node_ids(H)
    assert H.harness_pktdev_rx_port(ids["pktdev_rx"], port) == 0
    assert H.harness_rx_load(port, gp.ptrs(np.arange(n)), n) == 0
    try:
        _eth_config(H, L, ports)   # ip4_rewrite's tx edges; the hook copies them onto pktdev_rx
        assert _edges_of(H, ids["pktdev_rx"]) == PKTDEV_RX_EDGES + _edges_of(H, ids["ip4_rewrite"])
        tbl = _rw_table(L, 82, ports)
        H.harness_chain(1)
        assert H.harness_graph_create(13) == 0
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
        os.environ.pop("CNDP_GPU_RX_REWRITE", None)
        for ip, d, nh in routes:
            assert cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE) == 0
        assert H.harness_walk_until(n) >= 0
        assert H.harness_rx_left(port) == 0
        names = [b"pkt_drop"] + [f"pktdev_tx-{p}".encode() for p in ports]
        buf = (ctypes.c_void_p * n)()
        got = np.full(n, -1, np.int64)
        for k, nm in enumerate(names):
            m = H.harness_take_edge(nm, buf, n)
            idx = gp.index_of(np.array([x or 0 for x in buf[:m]], np.uint64))
            # pkt_drop takes drops from two nodes when ip4_rewrite runs as its
            # own node (rx node, then the rewrite node's polls), as the
            # reference's pkt_drop stream does (pkt_cls, ip4_lookup, ip4_rewrite)
            if fused or nm != b"pkt_drop":
                assert np.all(np.diff(idx) > 0), f"{nm}: out of receive order"
            got[idx] = k
        stats = {}
        for nm in (b"pkt_cls", b"ip4_lookup", b"ip4_rewrite"):
            c, o = ctypes.c_uint64(), ctypes.c_uint64()
            assert H.harness_node_stats(nm, ctypes.byref(c), ctypes.byref(o)) == 0
            stats[nm] = o.value
    finally:
        H.harness_rx_driver_writes(0)
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
        os.environ.pop("CNDP_GPU_RX_REWRITE", None)
        H.harness_chain(0)
        H.harness_graph_destroy()
        H.harness_edges_reset()
        L.cndp_node_ip4_rewrite_reset()
        L.cndp_node_gpu_umem_reset()
        os.environ.pop("CNDP_GPU_BATCH", None)
    # the reference chain on the oracle's copy: the receive chain per 256-mbuf
    # burst, then ip4_rewrite over each burst's mbufs ip4_lookup sent to it
    t24, t8 = O.dir24_8_build(list(routes), N.IP4_LOOKUP_NEXT_PKT_DROP << 16, 256)
    e = np.zeros(n, np.uint16)
    O.l3rx_chain_mbufs(op.ptrs(np.arange(n)), n, (t24, t8), edges=e)
    assert np.array_equal(gp.hdr["packet_type"], op.hdr["packet_type"])
    assert np.array_equal(gp.hdr["udata64"], op.hdr["udata64"])
    want = np.zeros(n, np.int64)
    for b0 in range(0, n, 256):
        ib = np.arange(b0, min(b0 + 256, n))
        rw = ib[e[ib] == 0]
        want[rw] = O.ip4_rewrite_node(op.ptrs(rw), len(rw), tbl)
    assert np.array_equal(got, want)
    ok = np.ones(n, bool) if fused else (ck != 0xFFFE) & (ck != 0xFFFF)
    diff = np.any(gp.mem.reshape(n, -1)[:, 64:] != op.mem.reshape(n, -1)[:, 64:], axis=1)
    assert not np.any(diff & ok)
    assert stats[b"pkt_cls"] == n and stats[b"ip4_lookup"] == int((e != 0xFFFE).sum())
    nrw = int((e == 0).sum())
    assert (e == 0xFFFE).sum() > 100 and nrw > n // 2 and (got == 0).sum() > 0
    if fused:
        assert stats[b"ip4_rewrite"] == nrw
        rw_all = np.nonzero(e == 0)[0]
        assert ((ck[rw_all] == 0xFFFE) | (ck[rw_all] == 0xFFFF)).sum() > 0   # the rule-dependent ones, compared
    NodeFib.fini()


@pytest.mark.gpu
@pytest.mark.parametrize("harness", ["rx", "cnet"])
def test_rx_nodes_idle_and_admin_down(gpu, harness):
    """The two GPU receive nodes on an idle port return 0 and enqueue nothing;
    on a port whose admin state is down they pass pktdev_rx_burst's
    PKTDEV_ADMIN_STATE_DOWN through (pktdev_rx.c:107-125, eth_rx.c:112-130)
    and enqueue nothing; a later burst on the same port still comes out."""
    from cndp_amd import pktgen
    from cndp_amd.mbuf import MbufPool
    L = N.lib()
    if harness == "rx":
        H = _rx_harness()
        nid = _node_ids(H)["pktdev_rx"]
        assert H.harness_pktdev_rx_port(nid, 5) == 0
        frames = pktgen.packed_ipv4(300, routes=pktgen.l3fwd_routes(), seed=91)
    else:
        from helpers import cnet_fibs
        H = _cnet_harness()
        fib, fib6, routes, v6, _, _ = cnet_fibs()
        H.harness_cnet_set(fib.h, fib6.h)
        nid = 0
        assert H.harness_eth_rx_port(nid, 5) == 0
        frames = pktgen.imix(300, v4routes=routes, v6routes=v6, seed=91)
    H.harness_process.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint16]
    H.harness_process.restype = ctypes.c_int
    H.harness_rx_down.argtypes = [ctypes.c_uint16, ctypes.c_int]
    pool = MbufPool(300)
    pool.fill(frames)
    L.cndp_node_gpu_umem_reset()
    assert L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes)) == 0
    name = b"pktdev_rx" if harness == "rx" else b"eth_rx"
    try:
        assert H.harness_graph_create(14) == 0
        assert H.harness_rx_load(5, None, 0) == 0
        H.harness_reset_counts()
        assert H.harness_process(name, None, 0) == 0 and H.harness_total() == 0
        assert H.harness_rx_load(5, pool.ptrs(np.arange(300)), 300) == 0
        H.harness_rx_down(5, 1)
        assert H.harness_process(name, None, 0) == 0xFFFF and H.harness_total() == 0
        assert H.harness_rx_left(5) == 300
        H.harness_rx_down(5, 0)
        assert H.harness_walk_until(300) >= 0
        assert H.harness_total() == 300 and H.harness_rx_left(5) == 0
    finally:
        H.harness_rx_down(5, 0)
        H.harness_graph_destroy()
        L.cndp_node_gpu_umem_reset()


def test_rewrite_hooks_unregistered_on_unload():
    """Each GPU node module hooks ip4_rewrite_set_next from its constructor and
    removes the hook from its destructor: a harness library loaded a second
    time (its own copy) and unloaded again leaves no hook behind, so a later
    ip4_rewrite_set_next neither calls into unmapped code nor edits that
    library's edges; a full hook table answers -ENOSPC, an unknown hook
    -ENOENT."""
    import shutil
    import _ctypes
    L = N.lib()
    _harness()   # the regular harness instance stays loaded throughout
    Hook = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint16, ctypes.c_uint16)
    L.cndp_node_ip4_rewrite_next_hook.argtypes = [Hook]
    L.cndp_node_ip4_rewrite_next_unhook.argtypes = [Hook]
    calls = []
    probe = Hook(lambda p, e: calls.append((p, e)) or 0)
    # count the free slots with a probe hook of our own
    fill = [Hook(lambda p, e: 0) for _ in range(20)]
    took = [f for f in fill if L.cndp_node_ip4_rewrite_next_hook(f) == 0]
    free_before = len(took)
    assert 0 < free_before < 20 and L.cndp_node_ip4_rewrite_next_hook(fill[-1]) == -28   # -ENOSPC
    for f in took:
        assert L.cndp_node_ip4_rewrite_next_unhook(f) == 0
    assert L.cndp_node_ip4_rewrite_next_unhook(fill[0]) == -2                            # -ENOENT
    # a second copy of the l3fwd harness: its two node modules hook on load
    cp = os.path.join(HERE, "node_harness", "libnode_harness_copy.so")
    shutil.copyfile(HARNESS, cp)
    try:
        h = ctypes.CDLL(cp)
        took = [f for f in fill if L.cndp_node_ip4_rewrite_next_hook(f) == 0]
        assert len(took) == free_before - 2     # ip4_lookup_gpu.c and ip4_rewrite_gpu.c of the copy
        for f in took:
            L.cndp_node_ip4_rewrite_next_unhook(f)
        _ctypes.dlclose(h._handle)
        del h
    finally:
        os.remove(cp)
    took = [f for f in fill if L.cndp_node_ip4_rewrite_next_hook(f) == 0]
    assert len(took) == free_before             # the copy's hooks went with it
    for f in took:
        L.cndp_node_ip4_rewrite_next_unhook(f)
    # and ip4_rewrite_set_next runs the remaining hooks only (none unmapped)
    assert L.cndp_node_ip4_rewrite_next_hook(probe) == 0
    try:
        L.cndp_node_ip4_rewrite_reset()
        assert L.ip4_rewrite_set_next(3, 1) == 0
        assert calls == [(3, 1)]
    finally:
        L.cndp_node_ip4_rewrite_next_unhook(probe)
        L.cndp_node_ip4_rewrite_reset()


# ---- one graph per worker lcore, all on one GPU ------------------------------
# l3fwd-graph creates a graph per worker lcore over the patterns "ip4*",
# "pktdev_tx-*", "pkt_drop", "pktdev_rx-<its ports>" and walks it on that
# lcore (examples/l3fwd-graph/fwd.c:128-139, :205-236); cnet-graph does the
# same with its eth_rx clones (examples/cnet-graph/cnet-graph.c:360).  Each
# graph's GPU nodes then hold a context and queue of their own on the shared
# GPU, and the walks run concurrently.
def _multi_graph_api(H):
    H.harness_clone.restype = ctypes.c_uint32
    H.harness_clone.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    H.harness_graph_new.restype = ctypes.c_void_p
    H.harness_graph_use.argtypes = [ctypes.c_void_p]
    H.harness_graph_free.argtypes = [ctypes.c_void_p]
    H.harness_graph_patterns.argtypes = [ctypes.c_void_p, ctypes.c_int]


def _run_lcores(H, pats_of, gids, want, between=None):
    """One thread per graph: use a graph of its own, create it over its
    patterns (every thread at once), then -- after `between` ran on the main
    thread (routes are added once the node FIB exists) -- walk it until
    want[k] objects were enqueued, and collect what each edge received.
    Returns per thread (seconds, {edge name: enqueued objects})."""
    import threading
    k_n = len(gids)
    graphs = [H.harness_graph_new() for _ in gids]
    created, go = threading.Barrier(k_n + 1), threading.Barrier(k_n + 1)
    res, errs = [None] * k_n, []

    def lcore(k):
        H.harness_graph_use(graphs[k])
        try:
            pats = [p.encode() for p in pats_of(k)]
            arr = (ctypes.c_char_p * len(pats))(*pats)
            assert H.harness_graph_patterns(arr, len(pats)) == 0
            rc = H.harness_graph_create(gids[k])
            created.wait(timeout=120)
            go.wait(timeout=120)
            assert rc == 0, f"graph {gids[k]} create: {rc}"
            t = H.harness_walk_until(want[k])
            assert t >= 0, f"graph {gids[k]} stalled"
            res[k] = t
        except BaseException as ex:  # reported below; the barriers must not wait forever
            errs.append(ex)
            created.abort()
            go.abort()

    th = [threading.Thread(target=lcore, args=(k,)) for k in range(k_n)]
    for t in th:
        t.start()
    try:
        created.wait(timeout=120)
        if between:
            between()
        go.wait(timeout=120)
    except threading.BrokenBarrierError:
        pass
    for t in th:
        t.join(timeout=180)
    return graphs, res, errs


def _edge_objs(H, graph, names, cap):
    H.harness_graph_use(graph)
    buf = (ctypes.c_void_p * cap)()
    out = {}
    for nm in names:
        m = H.harness_take_edge(nm, buf, cap)
        out[nm] = np.array([x or 0 for x in buf[:m]], np.uint64)
    H.harness_graph_use(None)
    return out


def _destroy_graphs(H, graphs):
    for g in graphs:
        H.harness_graph_use(g)
        H.harness_graph_destroy()
        H.harness_graph_use(None)
        H.harness_graph_free(g)


@pytest.mark.gpu
@pytest.mark.parametrize("threads,form", [(2, None), (4, None), (6, None), (4, "host_writeback"),
                                          (4, "device_headers_host_writeback")],
                         ids=["2", "4", "6", "4-host_writeback", "4-device_headers_host_writeback"])
def test_rx_node_graphs_per_lcore(gpu, threads, form):
    """`threads` worker lcores, each its own l3fwd-graph graph -- "ip4*",
    "pkt_cls" and its port's pktdev_rx clone (pktdev_ctrl.c:40-64) -- created
    and walked at the same time over disjoint UMEM pools: every mbuf of every
    pool leaves on the edge of the reference chain over that pool
    (pktdev_rx -> pkt_cls -> ip4_lookup -> ip4_rewrite per 256-mbuf burst),
    with its packet_type, priv1 and rewritten frame; each graph's pkt_cls /
    ip4_lookup / ip4_rewrite get the stats of their own pool.  form: the
    node's default for that many receive nodes (device headers at 2, host
    headers at 4, host writeback at 6), or the queues with
    CNDP_MQ_F_HOST_WRITEBACK (each lcore's polls write its mbufs)."""
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    from cndp_amd.mbuf import MbufPool
    from cndp_amd import pktgen
    from oracle import oracle as O
    from test_gpu_mq import _mixed_l3_frames
    H = _rx_harness()
    _multi_graph_api(H)
    L = N.lib()
    ports = tuple(range(threads))
    n = 12000
    pools = []
    NodeFib.fini()
    L.cndp_node_ip4_rewrite_reset()
    L.cndp_node_gpu_umem_reset()
    H.harness_edges_reset()
    H.harness_drop_clones()
    for k in ports:
        gp, op = MbufPool(n), MbufPool(n)
        fr = _mixed_l3_frames(n, seed=90 + k)
        for p in (gp, op):
            p.fill(fr)
            p.hdr["udata64"] = 0x5A5A5A5A
        pools.append((gp, op))
        assert L.cndp_node_gpu_umem_add(ctypes.c_void_p(gp.base), ctypes.c_uint64(gp.mem.nbytes)) == 0
        cid = H.harness_clone(b"pktdev_rx", str(k).encode())
        assert cid != 0xFFFFFFFF and H.harness_pktdev_rx_port(cid, k) == 0
        assert H.harness_rx_load(k, gp.ptrs(np.arange(n)), n) == 0
    os.environ["CNDP_GPU_BATCH"] = "4096"
    if form:
        os.environ["CNDP_GPU_MQ_FLAGS"] = str(N.CNDP_MQ_F_HOST_WRITEBACK |
                                              (N.CNDP_MQ_F_DEVICE_HEADERS if form.startswith("device") else 0))
    routes = pktgen.l3fwd_routes()
    names = [b"pkt_drop"] + [f"pktdev_tx-{p}".encode() for p in ports]
    graphs = []
    try:
        _eth_config(H, L, ports)   # ip4_rewrite's tx edges, mirrored onto every pktdev_rx clone
        tbl = _rw_table(L, 83, ports)
        H.harness_chain(1)

        def add_routes():
            for ip, d, nh in routes:
                assert cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE) == 0

        graphs, secs, errs = _run_lcores(H, lambda k: ["ip4*", "pkt_cls", f"pktdev_rx-{k}"],
                                         [120 + k for k in ports], [n] * threads, add_routes)
        assert not errs, errs
        got = [_edge_objs(H, g, names, n) for g in graphs]
        stats = []
        for g in graphs:
            H.harness_graph_use(g)
            st = {}
            for nm in (b"pkt_cls", b"ip4_lookup", b"ip4_rewrite"):
                c, o = ctypes.c_uint64(), ctypes.c_uint64()
                assert H.harness_node_stats(nm, ctypes.byref(c), ctypes.byref(o)) == 0
                st[nm] = o.value
            stats.append(st)
            H.harness_graph_use(None)
        assert all(H.harness_rx_left(k) == 0 for k in ports)
    finally:
        _destroy_graphs(H, graphs)
        os.environ.pop("CNDP_GPU_BATCH", None)
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
        H.harness_chain(0)
        H.harness_drop_clones()
        H.harness_pktdev_rx_ports_reset()
        H.harness_edges_reset()
        L.cndp_node_ip4_rewrite_reset()
        L.cndp_node_gpu_umem_reset()
    t24, t8 = O.dir24_8_build(list(routes), N.IP4_LOOKUP_NEXT_PKT_DROP << 16, 256)
    for k, (gp, op) in enumerate(pools):
        e = np.zeros(n, np.uint16)
        O.l3rx_chain_mbufs(op.ptrs(np.arange(n)), n, (t24, t8), edges=e)
        assert np.array_equal(gp.hdr["packet_type"], op.hdr["packet_type"]), k
        assert np.array_equal(gp.hdr["udata64"], op.hdr["udata64"]), k
        want = np.zeros(n, np.int64)
        for b0 in range(0, n, 256):
            ib = np.arange(b0, min(b0 + 256, n))
            rw = ib[e[ib] == 0]
            want[rw] = O.ip4_rewrite_node(op.ptrs(rw), len(rw), tbl)
        have = np.full(n, -1, np.int64)
        for j, nm in enumerate(names):
            idx = gp.index_of(got[k][nm])
            assert np.all(np.diff(idx) > 0), f"graph {k} {nm}: out of receive order"
            have[idx] = j
        assert np.array_equal(have, want), k
        assert not np.any(gp.mem.reshape(n, -1)[:, 64:] != op.mem.reshape(n, -1)[:, 64:]), k
        assert stats[k][b"pkt_cls"] == n and stats[k][b"ip4_lookup"] == int((e != 0xFFFE).sum())
        assert stats[k][b"ip4_rewrite"] == int((e == 0).sum())
    NodeFib.fini()


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [2, 4, 6])
def test_cnet_node_graphs_per_lcore(gpu, threads):
    """`threads` cnet-graph lcores, each with a graph over its port's eth_rx
    clone (pkt_ctrl.c:55-72), created and walked at the same time over
    disjoint UMEM pools of IMIX / fuzz / GTP frames: every mbuf of every pool
    gets the fields eth_rx and the input nodes write and leaves on the edge
    the reference's ptype / ip4_input / ip6_input send it to -- the ptype
    node's state is each graph's own, so each pool equals the oracle chain
    from state 0 over its own bursts.  At 6 the node's default result form is
    host writeback (beyond four receive nodes)."""
    from helpers import CNET_DEF, cnet_fibs
    from oracle import oracle as O
    from test_gpu_mq import _bursts, _cnet_expect, cnet_check, cnet_pool
    H = _cnet_harness()
    _multi_graph_api(H)
    L = N.lib()
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    n = 12000
    ports = tuple(range(threads))
    L.cndp_node_gpu_umem_reset()
    H.harness_drop_clones()
    H.harness_cnet_set(fib.h, fib6.h)
    pools = []
    for k in ports:
        pool, orig = cnet_pool(n, routes, v6, True)
        pools.append((pool, orig, _cnet_expect(pool, np.arange(n), _bursts(n, 0, "full"), t4, t6, 0, k)))
        assert L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes)) == 0
        cid = H.harness_clone(b"eth_rx", str(k).encode())
        assert cid != 0xFFFFFFFF and H.harness_eth_rx_port(cid, k) == 0
        assert H.harness_rx_load(k, pool.ptrs(np.arange(n)), n) == 0
    graphs = []
    try:
        graphs, secs, errs = _run_lcores(H, lambda k: [f"eth_rx-{k}", "ptype", "ip4_input", "ip6_input"],
                                         [140 + k for k in ports], [n] * threads)
        assert not errs, errs
        got = [_edge_objs(H, g, ETH_RX_EDGES, n) for g in graphs]
        assert all(H.harness_rx_left(k) == 0 for k in ports)
    finally:
        _destroy_graphs(H, graphs)
        H.harness_drop_clones()
        H.harness_eth_rx_ports_reset()
        L.cndp_node_gpu_umem_reset()
    for k, (pool, orig, ref) in enumerate(pools):
        have = np.full(n, -1, np.int64)
        for j, nm in enumerate(ETH_RX_EDGES):
            idx = pool.index_of(got[k][nm])
            assert np.all(np.diff(idx) > 0), f"graph {k} {nm}: out of receive order"
            have[idx] = j
        want_e = cnet_check(pool, orig, ref, t4, t6, k)
        want = np.array([_edge_of_queue_code(int(e)) for e in want_e])
        assert np.array_equal(have, want), k
        assert set(np.unique(have).tolist()) >= {0, 3, 4, 6}


def test_gpu_ip4_lookup_links_only_with_gpu_receive_node(tmp_path):
    """The supported build takes ip4_lookup_gpu.c only together with
    pktdev_rx_gpu.c: alone -- behind CNDP's own pktdev_rx,
    where one core beats it -- the node does not link (it references
    cndp_pktdev_rx_gpu_linked), so an unchanged l3fwd-graph always gets the
    fused GPU receive chain.  IP4_LOOKUP_GPU_STANDALONE (tests, bench) builds
    the node alone."""
    import subprocess
    root = os.path.dirname(HERE)
    nh = os.path.join(HERE, "node_harness")
    node = os.path.join(root, "cndp_amd", "node")
    base = ["gcc", "-O1", "-fPIC", "-shared", "-std=gnu11", "-Wall", "-Werror", f"-I{nh}",
            f"-I{os.path.join(root, 'include')}", "-Wl,--no-undefined", "-o", str(tmp_path / "x.so")]
    libs = [f"-L{os.path.join(root, 'cndp_amd', 'lib')}", "-lcndp_gpu", "-lpthread"]
    alone = subprocess.run(base + [os.path.join(node, "ip4_lookup_gpu.c"), os.path.join(nh, "harness.c")] + libs,
                           capture_output=True, text=True)
    assert alone.returncode != 0 and "cndp_pktdev_rx_gpu_linked" in alone.stderr
    ok = subprocess.run(base + ["-DIP4_LOOKUP_GPU_STANDALONE", os.path.join(node, "ip4_lookup_gpu.c"),
                                os.path.join(nh, "harness.c")] + libs, capture_output=True, text=True)
    assert ok.returncode == 0, ok.stderr[-2000:]
    with_rx = subprocess.run(base + [os.path.join(node, f) for f in ("pktdev_rx_gpu.c", "ip4_lookup_gpu.c")] +
                             [os.path.join(nh, f) for f in ("harness.c", "l3rx_stubs.c", "rx_stubs.c")] + libs,
                             capture_output=True, text=True)
    assert with_rx.returncode == 0, with_rx.stderr[-2000:]
