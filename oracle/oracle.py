"""ctypes wrapper of oracle/liboracle.so (and oracle/_ref/libcndp_ref.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product (cndp_amd/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, Structure, c_double, c_int, c_uint8, c_uint16, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libcndp_ref.so")

MODE_L3FWD, MODE_CNET, MODE_HASH = 0, 1, 2


class Route4(Structure):
    _fields_ = [("ip", c_uint32), ("depth", c_uint8), ("nh", c_uint64)]


class Route6(Structure):
    _fields_ = [("ip", c_uint8 * 16), ("depth", c_uint8), ("nh", c_uint64)]


class HdrLens(Structure):
    _fields_ = [("l2_len", c_uint8), ("inner_l2_len", c_uint8), ("l3_len", c_uint16),
                ("inner_l3_len", c_uint16), ("tunnel_len", c_uint16), ("l4_len", c_uint8),
                ("inner_l4_len", c_uint8)]


class ClassifyArgs(Structure):
    _fields_ = [("mode", c_uint32), ("slab", c_void_p), ("slab_len", c_uint64), ("stride", c_uint64),
                ("offsets", c_void_p), ("data_off", c_uint32), ("n", c_uint32), ("buf_len", c_uint32),
                ("tbl24", c_void_p), ("tbl8", c_void_p), ("tbl24_6", c_void_p), ("tbl8_6", c_void_p),
                ("rss_key", c_void_p), ("reta", c_void_p), ("reta_size", c_uint32), ("n_bins", c_uint32),
                ("nh", c_void_p), ("hash", c_void_p), ("queue", c_void_p), ("edge", c_void_p),
                ("bins", c_void_p), ("ptype", c_void_p), ("rxmeta", c_void_p), ("spec_burst", c_uint32),
                ("spec_state", c_void_p), ("no_hash", c_uint32)]


_lib = None
_ref = None


class ChainArgs(Structure):
    """struct orc_cnet_chain_args (oracle.h)"""
    _fields_ = [("mbufs", c_void_p), ("n", c_uint32), ("burst", c_uint32), ("rx_len", c_void_p),
                ("rx_data_off", c_uint16), ("lport", c_uint16), ("flags", c_uint32),
                ("tbl24", c_void_p), ("tbl8", c_void_p), ("tbl24_6", c_void_p), ("tbl8_6", c_void_p),
                ("rss_key", c_void_p), ("reta", c_void_p), ("reta_size", c_uint32), ("state", c_void_p)]


CHAIN_HASH = 1
# a pktmbuf_t header (pktmbuf.h:102-204) + the 64-B cnet_metadata after it
CHAIN_MBUF = np.dtype([("pooldata", "<u8"), ("buf_addr", "<u8"), ("hash", "<u4"), ("meta_index", "<u4"),
                       ("data_off", "<u2"), ("lport", "<u2"), ("buf_len", "<u2"), ("data_len", "<u2"),
                       ("packet_type", "<u4"), ("refcnt", "<u2"), ("rsvd16", "<u2"), ("tx_offload", "<u8"),
                       ("ol_flags", "<u8"), ("udata64", "<u8"), ("metadata", "u1", (64,))])


def slab_mbufs(slab: np.ndarray, offsets, lens, buf_len: int = 1984):
    """pktmbuf_t headers for frames that lie in a slab (frame i at
    slab + offsets[i], lens[i] bytes): buf_addr = the frame, data_off 0.
    Returns (headers, pointer array); keep both alive while they are used."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    n = len(offsets)
    hdr = np.zeros(n, CHAIN_MBUF)
    hdr["buf_addr"] = np.uint64(slab.ctypes.data) + offsets
    hdr["buf_len"] = buf_len
    hdr["data_len"] = np.asarray(lens, dtype=np.uint16)
    hdr["refcnt"] = 1
    ptrs = np.uint64(hdr.ctypes.data) + np.arange(n, dtype=np.uint64) * np.uint64(CHAIN_MBUF.itemsize)
    return hdr, ptrs


def cnet_chain(ptrs, n, rx_len, rx_data_off, tables4, tables6, burst=256, hash=False, key=None, reta=None,
               state=None, nthreads=1, iters=1, cpus=None, lport=0) -> float:
    """oracle/cnet_chain.c over n pktmbuf_t pointers (numpy u64 array or a
    ctypes pointer array): seconds for iters passes on nthreads threads."""
    from cndp_amd.native import MS_RSS_KEY
    key = np.frombuffer(key or MS_RSS_KEY, dtype=np.uint8).copy()
    reta = np.ascontiguousarray(reta if reta is not None else (np.arange(128) % 16), dtype=np.uint16)
    rx_len = np.ascontiguousarray(rx_len, dtype=np.uint16)
    a = ChainArgs()
    a.mbufs = ptrs.ctypes.data if isinstance(ptrs, np.ndarray) else ctypes.addressof(ptrs)
    a.n, a.burst, a.rx_len, a.rx_data_off, a.lport = n, burst, _p(rx_len), rx_data_off, lport
    a.flags = CHAIN_HASH if hash else 0
    a.tbl24, a.tbl8 = _p(tables4[0]), _p(tables4[1])
    a.tbl24_6, a.tbl8_6 = _p(tables6[0]), _p(tables6[1])
    a.rss_key, a.reta, a.reta_size = _p(key), _p(reta), len(reta)
    if state is not None:   # np.uint16 array of 1, updated in place
        a.state = _p(state)
    cp = np.ascontiguousarray(cpus, dtype=np.int32) if cpus is not None else None
    t = lib().orc_cnet_chain(ctypes.byref(a), nthreads, iters, _p(cp))
    if t < 0:
        raise ValueError("orc_cnet_chain rejected its arguments")
    return t


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE, os.path.join(HERE, "liboracle.so")], check=True)
        L = ctypes.CDLL(LIB)
        L.orc_softrss.restype = c_uint32
        L.orc_softrss.argtypes = [c_void_p, c_uint32, c_void_p]
        L.orc_softrss_be.restype = c_uint32
        L.orc_softrss_be.argtypes = [c_void_p, c_uint32, c_void_p]
        L.orc_convert_rss_key.argtypes = [c_void_p, c_void_p, c_int]
        L.orc_ipv4_cksum.restype = c_uint16
        L.orc_ipv4_cksum.argtypes = [c_void_p]
        L.orc_lpm4_bruteforce.argtypes = [c_void_p, c_uint32, c_uint64, c_void_p, c_uint32, c_void_p]
        L.orc_lpm6_bruteforce.argtypes = [c_void_p, c_uint32, c_uint64, c_void_p, c_uint32, c_void_p]
        L.orc_dir24_8_build.restype = c_int
        L.orc_dir24_8_build.argtypes = [c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p]
        L.orc_dir24_8_lookup.argtypes = [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]
        L.orc_trie_build.restype = c_int
        L.orc_trie_build.argtypes = [c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p]
        L.orc_trie_lookup.argtypes = [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]
        L.orc_cnet_ptype_edge.restype = c_uint32
        L.orc_cnet_ptype_edge.argtypes = [c_uint32]
        L.orc_get_ptype.restype = c_uint32
        L.orc_get_ptype.argtypes = [c_void_p, c_uint64, POINTER(HdrLens), c_uint32]
        L.orc_classify.restype = c_int
        L.orc_classify.argtypes = [POINTER(ClassifyArgs)]
        L.orc_l3fwd_burst_bench.restype = c_double
        L.orc_l3fwd_burst_bench.argtypes = [POINTER(ClassifyArgs), c_int, c_int]
        L.orc_burst_bench.restype = c_double
        L.orc_burst_bench.argtypes = [POINTER(ClassifyArgs), c_int, c_int, c_void_p]
        L.orc_dir24_8_lookup_bulk_pf.argtypes = [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]
        L.orc_ip4_lookup_mbufs.restype = c_double
        L.orc_ip4_lookup_mbufs.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_int]
        L.orc_ip4_rewrite.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p, c_uint32, c_uint32, c_void_p,
                                      c_uint32, c_void_p, c_void_p]
        L.orc_mac_swap.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p, c_uint32, c_uint32]
        L.orc_ip4_rewrite_node.argtypes = [c_void_p, c_uint32, c_void_p, c_void_p]
        L.orc_rx_ip4_lookup_mbufs.restype = c_double
        L.orc_rx_ip4_lookup_mbufs.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_int]
        L.orc_l3rx_chain_mbufs.restype = c_double
        L.orc_l3rx_chain_mbufs.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_int, c_void_p,
                                           c_void_p]
        L.orc_cnet_chain.restype = c_double
        L.orc_cnet_chain.argtypes = [POINTER(ChainArgs), c_int, c_int, c_void_p]
        L.orc_l3fwd_nodes_mbufs.restype = c_double
        L.orc_l3fwd_nodes_mbufs.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_int]
        _lib = L
    return _lib


def ref():
    """The reference's own cne_softrss / cne_ipv4_cksum (None if not built)."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB):
        R = ctypes.CDLL(REF_LIB)
        R.ref_softrss.restype = c_uint32
        R.ref_softrss.argtypes = [c_void_p, c_uint32, c_void_p]
        R.ref_softrss_be.restype = c_uint32
        R.ref_softrss_be.argtypes = [c_void_p, c_uint32, c_void_p]
        R.ref_convert_rss_key.argtypes = [c_void_p, c_void_p, c_int]
        R.ref_ipv4_cksum.restype = c_uint16
        R.ref_ipv4_cksum.argtypes = [c_void_p]
        R.ref_thash_load_v6.argtypes = [c_void_p, c_void_p]
        _ref = R
    return _ref


def _p(a):
    return a.ctypes.data if a is not None else None


def softrss(tuple_dw, key: bytes) -> int:
    t = np.ascontiguousarray(tuple_dw, dtype=np.uint32)
    return lib().orc_softrss(_p(t), len(t), key)


def ipv4_cksum(hdr: bytes) -> int:
    b = np.frombuffer(bytes(hdr) + bytes(64), dtype=np.uint8)
    return lib().orc_ipv4_cksum(_p(b))


def _routes4(routes):
    arr = (Route4 * max(1, len(routes)))()
    for i, (ip, d, nh) in enumerate(routes):
        arr[i].ip, arr[i].depth, arr[i].nh = ip & 0xFFFFFFFF, d, nh
    return arr


def _routes6(routes):
    arr = (Route6 * max(1, len(routes)))()
    for i, (ip, d, nh) in enumerate(routes):
        b = ip.to_bytes(16, "big") if isinstance(ip, int) else bytes(ip)
        arr[i].ip[:] = list(b)
        arr[i].depth, arr[i].nh = d, nh
    return arr


def lpm4_bruteforce(routes, def_nh, ips) -> np.ndarray:
    ips = np.ascontiguousarray(ips, dtype=np.uint32)
    out = np.zeros(len(ips), np.uint64)
    lib().orc_lpm4_bruteforce(_routes4(routes), len(routes), def_nh, _p(ips), len(ips), _p(out))
    return out


def lpm6_bruteforce(routes, def_nh, ips) -> np.ndarray:
    ips = np.ascontiguousarray(ips, dtype=np.uint8).reshape(-1, 16)
    out = np.zeros(len(ips), np.uint64)
    lib().orc_lpm6_bruteforce(_routes6(routes), len(routes), def_nh, _p(ips), len(ips), _p(out))
    return out


def dir24_8_build(routes, def_nh, num_tbl8=1024):
    t24 = np.empty(1 << 24, np.uint32)
    t8 = np.zeros((num_tbl8 + 1) * 256, np.uint32)
    rc = lib().orc_dir24_8_build(_routes4(routes), len(routes), def_nh, num_tbl8, _p(t24), _p(t8))
    if rc < 0:
        raise OSError(-rc, "orc_dir24_8_build")
    return t24, t8


def dir24_8_lookup(t24, t8, ips) -> np.ndarray:
    ips = np.ascontiguousarray(ips, dtype=np.uint32)
    out = np.zeros(len(ips), np.uint64)
    lib().orc_dir24_8_lookup(_p(t24), _p(t8), _p(ips), len(ips), _p(out))
    return out


def trie_build(routes, def_nh, num_tbl8=1 << 15):
    t24 = np.empty(1 << 24, np.uint32)
    t8 = np.zeros((num_tbl8 + 1) * 256, np.uint32)
    rc = lib().orc_trie_build(_routes6(routes), len(routes), def_nh, num_tbl8, _p(t24), _p(t8))
    if rc < 0:
        raise OSError(-rc, "orc_trie_build")
    return t24, t8


def trie_lookup(t24, t8, ips) -> np.ndarray:
    ips = np.ascontiguousarray(ips, dtype=np.uint8).reshape(-1, 16)
    out = np.zeros(len(ips), np.uint64)
    lib().orc_trie_lookup(_p(t24), _p(t8), _p(ips), len(ips), _p(out))
    return out


def cnet_ptype_edge(pt: int) -> int:
    """The ptype node's p_nxt[pt & _PTYPE_MASK] (ptype.c:32-46)."""
    return int(lib().orc_cnet_ptype_edge(ctypes.c_uint32(pt & 0xFFFFFFFF)))


def get_ptype(pkt: bytes):
    b = np.frombuffer(bytes(pkt), dtype=np.uint8)
    hl = HdrLens()
    pt = lib().orc_get_ptype(_p(b), len(b), ctypes.byref(hl), 0x0FFFFFFF)
    return pt, hl


def make_args(mode, slab, n, stride=64, offsets=None, data_off=0, buf_len=1984, tables4=None,
              tables6=None, key=None, reta=None, n_bins=64, spec_burst=0, spec_state=None, no_hash=False):
    from cndp_amd.native import MS_RSS_KEY
    key = np.frombuffer(key or MS_RSS_KEY, dtype=np.uint8).copy()
    reta = np.ascontiguousarray(reta if reta is not None else (np.arange(128) % 16), dtype=np.uint16)
    out = {"nh": np.zeros(n, np.uint32), "hash": np.zeros(n, np.uint32), "queue": np.zeros(n, np.uint16),
           "edge": np.zeros(n, np.uint8), "bins": np.zeros(n_bins + 2, np.uint64),
           "ptype": np.zeros(n, np.uint32), "rxmeta": np.zeros(n, np.uint32)}
    slab = np.ascontiguousarray(slab, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64) if offsets is not None else None
    a = ClassifyArgs()
    a.mode, a.slab, a.slab_len, a.stride = mode, _p(slab), slab.nbytes, stride
    a.offsets, a.data_off, a.n, a.buf_len = _p(off), data_off, n, buf_len
    if tables4 is not None:
        a.tbl24, a.tbl8 = _p(tables4[0]), _p(tables4[1])
    if tables6 is not None:
        a.tbl24_6, a.tbl8_6 = _p(tables6[0]), _p(tables6[1])
    a.rss_key, a.reta, a.reta_size, a.n_bins = _p(key), _p(reta), len(reta), n_bins
    a.nh, a.hash, a.queue, a.edge, a.bins = (_p(out["nh"]), _p(out["hash"]), _p(out["queue"]),
                                            _p(out["edge"]), _p(out["bins"]))
    a.ptype, a.rxmeta = _p(out["ptype"]), _p(out["rxmeta"])
    a.spec_burst = spec_burst
    a.no_hash = 1 if no_hash else 0
    if spec_state is not None:   # np.uint16 array of 1, updated in place
        a.spec_state = _p(spec_state)
    keep = (slab, off, key, reta, tables4, tables6, spec_state)  # keep buffers alive with the struct
    return a, out, keep


def classify(mode, slab, n, **kw) -> dict:
    a, out, keep = make_args(mode, slab, n, **kw)
    rc = lib().orc_classify(ctypes.byref(a))
    if rc < 0:
        raise OSError(-rc, "orc_classify")
    del keep
    return out


def burst_bench(mode, slab, n, nthreads=1, iters=1, cpus=None, **kw) -> float:
    """Seconds for `iters` passes of the per-burst CPU chain over n packets on
    nthreads threads (thread t pinned to cpus[t] when given)."""
    a, out, keep = make_args(mode, slab, n, **kw)
    cp = np.ascontiguousarray(cpus, dtype=np.int32) if cpus is not None else None
    t = lib().orc_burst_bench(ctypes.byref(a), nthreads, iters, _p(cp))
    del keep, cp
    return t


def dir24_8_lookup_bulk_pf(t24, t8, ips) -> np.ndarray:
    ips = np.ascontiguousarray(ips, dtype=np.uint32)
    out = np.zeros(len(ips), np.uint64)
    lib().orc_dir24_8_lookup_bulk_pf(_p(t24), _p(t8), _p(ips), len(ips), _p(out))
    return out


def set_driver_writes(on: bool) -> None:
    """Receive-driver header writes (xskdev.c:296-297: data_len / data_off of
    every mbuf, values kept) before each burst of the l3fwd mbuf node loops
    below -- the header-cache state a real graph walk gives its nodes."""
    lib().orc_set_driver_writes(1 if on else 0)


def ip4_lookup_mbufs(ptrs, n, tables4, burst=256, iters=1) -> float:
    """The ip4_lookup node's CPU loop over pktmbuf_t pointers (one thread): seconds."""
    return lib().orc_ip4_lookup_mbufs(ptrs, n, burst, _p(tables4[0]), _p(tables4[1]), iters)


def rx_ip4_lookup_mbufs(ptrs, n, tables4, burst=256, iters=1) -> float:
    """pktdev_rx's soft parse then the ip4_lookup node loop per burst (one thread): seconds."""
    return lib().orc_rx_ip4_lookup_mbufs(ptrs, n, burst, _p(tables4[0]), _p(tables4[1]), iters)


def l3rx_chain_mbufs(ptrs, n, tables4, burst=256, iters=1, edges=None, rewrite=None) -> float:
    """l3fwd-graph's receive chain per burst on one thread (pktdev_rx's soft
    parse, pkt_cls, the ip4_lookup loop over the IPv4 mbufs; with rewrite, a
    REWRITE_NH table, the ip4_rewrite node over the ones sent to it): seconds;
    edges (uint16 array of n, optional) gets each mbuf's ip4_lookup edge --
    FIB value >> 16, or 0xFFFE where pkt_cls dropped it."""
    return lib().orc_l3rx_chain_mbufs(ptrs, n, burst, _p(tables4[0]), _p(tables4[1]), iters,
                                      None if edges is None else _p(edges), _p(rewrite))


def l3fwd_burst_bench(slab, n, stride, tables4, nthreads=1, iters=1, **kw) -> float:
    a, out, keep = make_args(MODE_L3FWD, slab, n, stride=stride, tables4=tables4, **kw)
    t = lib().orc_l3fwd_burst_bench(ctypes.byref(a), nthreads, iters)
    del keep
    return t


REWRITE_NH = np.dtype([("rewrite_len", "<u2"), ("tx_node", "<u2"), ("enabled", "<u2"), ("rsvd", "<u2"),
                       ("rewrite_data", "u1", (56,))])


def ip4_rewrite(slab: np.ndarray, n: int, nh: np.ndarray, table: np.ndarray, burst: int = 256,
                stride: int = 64, offsets=None, data_off: int = 0):
    """In-place ip4_rewrite restatement; returns tx_edge (u16)."""
    assert slab.dtype == np.uint8 and slab.flags.c_contiguous
    nh = np.ascontiguousarray(nh, dtype=np.uint32)
    table = np.ascontiguousarray(table, dtype=REWRITE_NH)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64) if offsets is not None else None
    tx = np.zeros(n, np.uint16)
    lib().orc_ip4_rewrite(slab.ctypes.data, slab.nbytes, stride, offs.ctypes.data if offs is not None else None,
                          data_off, n, nh.ctypes.data, burst, table.ctypes.data, tx.ctypes.data)
    return tx


def ip4_rewrite_node(ptrs, n: int, table: np.ndarray) -> np.ndarray:
    """ip4_rewrite_node_process over one burst of pktmbuf_t pointers (in place,
    host memory); returns the tx edge of each mbuf."""
    table = np.ascontiguousarray(table, dtype=REWRITE_NH)
    tx = np.zeros(max(n, 1), np.uint16)
    lib().orc_ip4_rewrite_node(ptrs, n, table.ctypes.data, tx.ctypes.data)
    return tx[:n]


def l3fwd_nodes_mbufs(ptrs, n: int, tables4, table: np.ndarray, burst: int = 256, iters: int = 1) -> float:
    """ip4_lookup + ip4_rewrite node loop over pktmbuf_t pointers, one thread: seconds."""
    table = np.ascontiguousarray(table, dtype=REWRITE_NH)
    return lib().orc_l3fwd_nodes_mbufs(ptrs, n, burst, _p(tables4[0]), _p(tables4[1]), table.ctypes.data, iters)


def mac_swap(slab: np.ndarray, n: int, stride: int = 64, offsets=None, data_off: int = 0):
    offs = np.ascontiguousarray(offsets, dtype=np.uint64) if offsets is not None else None
    lib().orc_mac_swap(slab.ctypes.data, slab.nbytes, stride, offs.ctypes.data if offs is not None else None,
                       data_off, n)
