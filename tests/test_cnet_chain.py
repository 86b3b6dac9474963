"""The CPU baseline of the cnet chain (oracle/cnet_chain.c: eth_rx -> ptype ->
ip4_input / ip6_input per 256-mbuf burst over pktmbuf_t pointers, direct loads
and the reference nodes' prefetching) against the checker (orc_classify) on
the same frames: C4 IMIX, C5 1500-B frames with corrupted checksums, and the
fuzz frames that steer every cne_get_ptype branch.  Every mbuf field the chain
writes is compared: packet_type, tx_offload / ol_flags (the checker's rxmeta),
the flow hash, where the ptype and input nodes sent the mbuf and its FIB value,
data_off / data_len after the chain, and the input nodes' cnet_metadata."""
import numpy as np
import pytest

from cndp_amd import native as N
from cndp_amd import pktgen
from oracle import oracle as O

from helpers import CNET_DEF, cnet_fibs

NH_INVALID = 0xFFFFFFFF


def _tables():
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    return routes, v6, t4, t6


def _run_both(slab, offsets, lens, t4, t6, burst=256, state0=0):
    slab = np.concatenate([slab, np.zeros(4096, np.uint8)])  # the checker reads bytes past the end as 0
    n = len(offsets)
    st = np.array([state0], np.uint16)
    ref = O.classify(O.MODE_CNET, slab, n, offsets=offsets, tables4=t4, tables6=t6, spec_burst=burst,
                     spec_state=st)
    hdr, ptrs = O.slab_mbufs(slab, offsets, lens)
    st2 = np.array([state0], np.uint16)
    t = O.cnet_chain(ptrs, n, lens, 0, t4, t6, burst=burst, hash=True, state=st2)
    assert t >= 0
    return ref, hdr, st[0], st2[0], slab


def _compare(ref, hdr, slab, offsets):
    assert np.array_equal(hdr["packet_type"], ref["ptype"])
    rxmeta = (hdr["tx_offload"] & 0xFFFFFF).astype(np.uint32) | (hdr["ol_flags"] >> np.uint64(32)).astype(np.uint32)
    assert np.array_equal(rxmeta, ref["rxmeta"])
    assert np.array_equal(hdr["hash"], ref["hash"])
    nh = (hdr["udata64"] & 0xFFFFFFFF).astype(np.uint32)
    edge = (hdr["udata64"] >> np.uint64(32)).astype(np.uint32)
    assert np.array_equal(nh, ref["nh"])
    assert np.array_equal(edge.astype(np.uint8), ref["edge"])
    # the frames an input node took: data_len from their IP header, and
    # cnet_metadata {family, len, addr} of source and destination
    l2 = (hdr["tx_offload"] & 0x7F).astype(np.int64)
    assert np.array_equal(hdr["data_off"].astype(np.int64), l2)
    took4 = np.isin(edge, [0, 1, 2]) & (nh != NH_INVALID)
    for i in np.flatnonzero(took4)[:2000]:
        ip = int(offsets[i]) + int(l2[i])
        md = hdr["metadata"][i]
        if md[0] == 2:
            assert int(hdr["data_len"][i]) == int(slab[ip + 2]) << 8 | int(slab[ip + 3])
            assert bytes(md[4:8]) == bytes(slab[ip + 12:ip + 16]) and bytes(md[24:28]) == bytes(slab[ip + 16:ip + 20])
        else:
            assert md[0] == 10
            assert int(hdr["data_len"][i]) == int(slab[ip + 4]) << 8 | int(slab[ip + 5])
            assert bytes(md[24:40]) == bytes(slab[ip + 24:ip + 40])


def test_chain_c4_imix():
    routes, v6, t4, t6 = _tables()
    n = 40000
    fr = pktgen.imix(n, v4routes=routes, v6routes=v6, seed=31)
    slab = fr.slab.numpy()
    offs = fr.offsets.numpy().astype(np.uint64)
    lens = fr.lengths.numpy().astype(np.uint16)
    ref, hdr, s1, s2, slab = _run_both(slab, offs, lens, t4, t6)
    _compare(ref, hdr, slab, offs)
    assert s1 == s2
    assert set(np.unique(ref["edge"]).tolist()) >= {1}


def test_chain_c5_checksums():
    routes, v6, t4, t6 = _tables()
    n = 6000
    fr = pktgen.packed_ipv4(n, slot=1536, frame_len=1500, routes=routes, seed=32)
    pktgen.corrupt_cksum(fr, 64, 32)
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(1536))
    ref, hdr, s1, s2, slab = _run_both(fr.slab.numpy(), offs, np.full(n, 1500, np.uint16), t4, t6)
    _compare(ref, hdr, slab, offs)
    assert (ref["edge"] == 0).sum() > 0     # the corrupted checksums are dropped


@pytest.mark.parametrize("burst", [256, 64, 7])
def test_chain_gtp_speculation(burst):
    """GTP-U / GTP-C frames inside UDP runs: the ptype node's speculation
    re-routes frames, state carried across bursts and from a given start."""
    from test_gpu_parity import _gtp_mix  # noqa: F401  (same frame recipe on the CPU)
    routes, v6, t4, t6 = _tables()
    n = 256 * 40 + 13
    fr = _gtp_mix(n, routes, v6, "cpu", seed=33)
    offs = fr.offsets.numpy().astype(np.uint64)
    lens = (fr.lengths.numpy() if fr.lengths is not None else np.full(n, 512)).astype(np.uint16)
    ref, hdr, s1, s2, slab = _run_both(fr.slab.numpy(), offs, lens, t4, t6, burst=burst, state0=0x0211)
    _compare(ref, hdr, slab, offs)
    assert s1 == s2


def test_chain_fuzz_get_ptype():
    """Every cne_get_ptype branch (VLAN / QinQ / ARP / MPLS, IHL, fragments,
    IPv6 extension chains, tunnels, GTP): the direct-load restatement equals
    the checker's bounded one."""
    routes, v6, t4, t6 = _tables()
    n = 20000
    fr = pktgen.fuzz_frames(n, seed=34, slot=128)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(128)
    ref, hdr, s1, s2, slab = _run_both(fr.slab.numpy(), offs, np.full(n, 124, np.uint16), t4, t6)
    assert np.array_equal(hdr["packet_type"], ref["ptype"])
    rxmeta = (hdr["tx_offload"] & 0xFFFFFF).astype(np.uint32) | (hdr["ol_flags"] >> np.uint64(32)).astype(np.uint32)
    assert np.array_equal(rxmeta, ref["rxmeta"])
    assert np.array_equal(hdr["hash"], ref["hash"])
    assert len(np.unique(ref["ptype"])) > 40


def test_chain_threads_and_passes():
    """Several threads and passes (the bench's form): every pass starts from
    the received mbufs, so the results equal one single-threaded pass."""
    routes, v6, t4, t6 = _tables()
    n = 4096 * 4
    fr = pktgen.imix(n, v4routes=routes, v6routes=v6, seed=35)
    slab = np.concatenate([fr.slab.numpy(), np.zeros(4096, np.uint8)])
    offs = fr.offsets.numpy().astype(np.uint64)
    lens = fr.lengths.numpy().astype(np.uint16)
    h1, p1 = O.slab_mbufs(slab, offs, lens)
    O.cnet_chain(p1, n, lens, 0, t4, t6, hash=True)
    h4, p4 = O.slab_mbufs(slab, offs, lens)
    O.cnet_chain(p4, n, lens, 0, t4, t6, hash=True, nthreads=4, iters=3)
    for k in ("packet_type", "hash", "data_off", "data_len", "tx_offload", "ol_flags"):
        assert np.array_equal(h1[k], h4[k]), k
    # the speculation restarts per thread (one graph per lcore): only the
    # per-frame results of chunks whose entering state matches agree, which
    # for IMIX (universal groups in every burst) is all of them
    assert np.array_equal(h1["udata64"], h4["udata64"])
