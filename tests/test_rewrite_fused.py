"""The l3fwd lookup + rewrite pass fused into the GPU ip4_lookup queue
(CNDP_MQ_F_REWRITE) and its host half in the GPU ip4_rewrite node
(cndp_node_ip4_rewrite_fused).

The host half is pure host code, so it runs here without a GPU: frames that
the lookup pass rewrote by the 4-wide loop's rule (ip4_rewrite.c:85-110) must
come out of any burst split exactly as ip4_rewrite_node_process leaves them
for that split (the tail loop's rule for the last nb % 4, :201-216), with the
same tx edges.  The fused device pass itself is checked on the GPU by
tests/test_node_graph.py::test_l3fwd_graph_chain[fused].
"""
import ctypes

import numpy as np
import pytest

from cndp_amd import native as N

PORTS = (0, 2, 5)


def _table(L, seed):
    """Next hops through cne_node_ip4_rewrite_add and the oracle's copy."""
    from oracle import oracle as O
    rng = np.random.default_rng(seed)
    tbl = np.zeros(64, dtype=O.REWRITE_NH)
    for k, p in enumerate(PORTS):
        assert L.ip4_rewrite_set_next(p, k + 1) == 0
    for nh in range(64):
        if nh % 9 == 8:
            continue
        ln = int(rng.choice([12, 12, 0, 14, 30, 56]))
        data = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
        k = nh % len(PORTS)
        assert L.cne_node_ip4_rewrite_add(nh, ctypes.create_string_buffer(data, max(ln, 1)), ln, PORTS[k]) == 0
        tbl[nh]["rewrite_len"], tbl[nh]["tx_node"], tbl[nh]["enabled"] = ln, k + 1, 1
        tbl[nh]["rewrite_data"][:ln] = np.frombuffer(data, np.uint8)
    return tbl


def _pools(n, seed):
    from cndp_amd import pktgen
    from cndp_amd.mbuf import MbufPool
    rng = np.random.default_rng(seed)
    gp, op = MbufPool(n), MbufPool(n)
    ck = rng.integers(0, 1 << 16, n, dtype=np.uint64)
    ck[::5] = 0xFFFF
    ck[2::5] = 0xFFFE
    priv = rng.integers(0, 70, n, dtype=np.uint64) | (rng.integers(0, 256, n, dtype=np.uint64) << 16) | (ck << 32)
    for p in (gp, op):
        p.fill(pktgen.packed_ipv4(n, routes=pktgen.l3fwd_routes(), seed=seed + 1))
        p.hdr["udata64"] = priv
    return gp, op, rng


def test_rewrite_fused_host_half():
    from oracle import oracle as O
    L = N.lib()
    n = 6000
    L.cndp_node_ip4_rewrite_reset()
    try:
        tbl = _table(L, 5)
        gp, op, rng = _pools(n, 6)
        # the lookup pass: every frame by the 4-wide rule (one burst, n % 4 == 0),
        # and the mark in ttl's high byte (ip4_rewrite stores ttl - 1 as a u8)
        assert n % 4 == 0
        O.ip4_rewrite_node(gp.ptrs(np.arange(n)), n, tbl)
        gp.hdr["udata64"] |= np.uint64(N.CNDP_PRIV1_REWRITTEN << 24)
        edges = (ctypes.c_uint16 * 1024)()
        pos = 0
        while pos < n:
            b = int(min(n - pos, rng.choice([256, 256, 97, 4, 3, 1, 6, 1024])))
            idx = np.arange(pos, pos + b)
            assert L.cndp_node_ip4_rewrite_fused(gp.ptrs(idx), b, edges) == b
            want = O.ip4_rewrite_node(op.ptrs(idx), b, tbl)
            assert np.array_equal(np.frombuffer(edges, np.uint16)[:b], want), f"burst at {pos}"
            pos += b
    finally:
        L.cndp_node_ip4_rewrite_reset()
    frames = lambda p: p.mem.reshape(n, -1)[:, 64:]  # noqa: E731 (buffers; headers differ by address)
    bad = np.nonzero(np.any(frames(gp) != frames(op), axis=1))[0]
    assert bad.size == 0, f"{bad.size} frames differ, first {bad[:4]}"


def test_rewrite_fused_needs_every_mark():
    """A burst with one unmarked mbuf is left alone (0): the node runs it
    through its queue, so the tail positions stay those of its own burst."""
    L = N.lib()
    n = 64
    L.cndp_node_ip4_rewrite_reset()
    try:
        _table(L, 7)
        gp, _, _ = _pools(n, 8)
        gp.hdr["udata64"] |= np.uint64(N.CNDP_PRIV1_REWRITTEN << 24)
        gp.hdr["udata64"][37] &= ~np.uint64(0xFF << 24)
        before = gp.mem.copy()
        edges = (ctypes.c_uint16 * n)()
        assert L.cndp_node_ip4_rewrite_fused(gp.ptrs(np.arange(n)), n, edges) == 0
        assert np.array_equal(gp.mem, before)
        assert L.cndp_node_ip4_rewrite_fused(gp.ptrs(np.arange(37)), 37, edges) == 37
        assert L.cndp_node_ip4_rewrite_fused(None, 1, edges) == -22
    finally:
        L.cndp_node_ip4_rewrite_reset()


def test_mq_rewrite_flag_declared():
    """The flag and the mark as the header declares them (the ctypes mirror
    and the node sources use the same values)."""
    assert N.CNDP_MQ_F_REWRITE == 8 and N.CNDP_PRIV1_REWRITTEN == 0x80
    hdr = open(N.os.path.join(N.os.path.dirname(N.HERE), "include", "cndp_gpu.h")).read()
    assert "#define CNDP_MQ_F_REWRITE (1u << 3)" in hdr
    assert "#define CNDP_PRIV1_REWRITTEN 0x80u" in hdr


@pytest.mark.gpu
def test_mq_rewrite_flag_refused_when_staged(gpu):
    """CNDP_MQ_F_REWRITE is for the ip4_lookup mode over registered UMEMs
    only (the pass writes frames in place): a staged queue and another mode
    refuse it at create (-EINVAL)."""
    from cndp_amd.classify import Classifier
    from cndp_amd.fib import Fib
    cl = Classifier(0)
    f4 = Fib("fz", N.CNE_FIB_DIR24_8, default_nh=1 << 16, max_routes=16, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=16)
    cl.set_fib(f4, None)
    conf = N.MqConf(mode=N.CNDP_MQ_IP4_LOOKUP, flags=N.CNDP_MQ_F_REWRITE)
    q = ctypes.c_void_p()
    assert N.lib().cndp_gpu_mq_create(cl.h, ctypes.byref(conf), ctypes.byref(q)) == -22
    conf = N.MqConf(mode=N.CNDP_MQ_MAC_SWAP, flags=N.CNDP_MQ_F_REWRITE, umem=1)
    assert N.lib().cndp_gpu_mq_create(cl.h, ctypes.byref(conf), ctypes.byref(q)) == -22
    cl.close()
