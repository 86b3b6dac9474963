"""ctypes binding of libcndp_gpu.so (the C-ABI declared in include/cndp_fib.h,
include/cndp_node.h and include/cndp_gpu.h).

The library is built in-tree (cndp_amd/lib/libcndp_gpu.so, see build.py).
There is no fallback: if the shared object is missing, importing the
product API raises, so a test or bench can never silently run a CPU path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, Union, c_char_p, c_int, c_uint8, c_uint16,
                    c_uint32, c_uint64, c_void_p)

HERE = os.path.dirname(os.path.abspath(__file__))
# CNDP_GPU_LIB: an alternative build of the same library (A/B timing experiments)
LIB_PATH = os.environ.get("CNDP_GPU_LIB") or os.path.join(HERE, "lib", "libcndp_gpu.so")

# cne_fib.h:34-38, :53-58, :60, :63-73 (+ CNE_FIB_LOOKUP_GPU)
CNE_FIB_DUMMY, CNE_FIB_DIR24_8, CNE_FIB_TRIE = 0, 1, 2
CNE_FIB_DIR24_8_1B, CNE_FIB_DIR24_8_2B, CNE_FIB_DIR24_8_4B, CNE_FIB_DIR24_8_8B = 0, 1, 2, 3
CNE_FIB_TRIE_2B, CNE_FIB_TRIE_4B, CNE_FIB_TRIE_8B = 1, 2, 3
(CNE_FIB_LOOKUP_DEFAULT, CNE_FIB_LOOKUP_DIR24_8_SCALAR_MACRO, CNE_FIB_LOOKUP_DIR24_8_SCALAR_INLINE,
 CNE_FIB_LOOKUP_DIR24_8_SCALAR_UNI, CNE_FIB_LOOKUP_DIR24_8_VECTOR_AVX512, CNE_FIB_LOOKUP_TRIE_SCALAR,
 CNE_FIB_LOOKUP_TRIE_VECTOR_AVX512, CNE_FIB_LOOKUP_GPU) = range(8)
CNE_FIB_MAXDEPTH = 32
CNE_FIB6_MAXDEPTH = 128

# cndp_gpu.h
CNDP_MODE_L3FWD, CNDP_MODE_CNET, CNDP_MODE_HASH = 0, 1, 2
CNDP_NH_INVALID = 0xFFFFFFFF
CNDP_EDGE_CLS_DROP = 0xFF
CNDP_RSS_KEY_LEN = 40
CNDP_RETA_MAX = 512
CNDP_BINS_MAX = 1024
CNDP_FRAMES_CACHED = 1
CNDP_TUNE_NT, CNDP_TUNE_UNROLL, CNDP_TUNE_BLOCKS_PER_CU, CNDP_TUNE_TILE, CNDP_TUNE_DIR16 = 1, 2, 3, 4, 5
CNDP_TUNE_CNET_TILE = 6
CNDP_TUNE_HOST_CHUNK = 7
CNDP_TUNE_RW_WB = 8
CNDP_TUNE_CNET_SPEC = 9
CNDP_TUNE_LOAD_NT = 10
CNDP_TUNE_SPEC_SCAN = 11
CNDP_STAT_CNET_WORKLIST, CNDP_STAT_CNET_UNIFORM, CNDP_STAT_SPEC_ERR = 1, 2, 3
CNDP_TUNE_MBUF_HASH = 12
CNDP_TUNE_CNET_FOLD = 13
CNDP_TUNE_SPEC_GRID = 14
CNDP_TUNE_SPEC_LISTS = 15
CNDP_TUNE_SPEC_TYPES = 16
CNDP_TUNE_STREAM_BAL = 17
CNDP_TUNE_SPEC_WAIT = 18
CNDP_TUNE_HOST_WINDOW = 19
CNDP_MQ_IP4_LOOKUP, CNDP_MQ_CNET, CNDP_MQ_MAC_SWAP, CNDP_MQ_IP4_REWRITE = 0, 1, 2, 3
CNDP_MQ_F_HASH, CNDP_MQ_F_NO_METADATA, CNDP_MQ_F_DEVICE_HEADERS, CNDP_MQ_F_RX_PARSE = 1, 2, 4, 8
CNDP_MQ_F_REWRITE = 16
CNDP_MQ_F_HOST_WRITEBACK = 1 << 5
CNDP_MQ_EDGE_NONE = 0xFFFF
CNDP_MQ_EDGE_CLS_DROP = 0xFFFE
CNDP_MQ_EDGE_LOOKUP_DROP = 0xFFFD
CNDP_MQ_STAT_BATCHES, CNDP_MQ_STAT_MBUFS = 1, 2
CNDP_MQ_NODE_PTYPE, CNDP_MQ_NODE_IP4, CNDP_MQ_NODE_IP6 = 0, 1, 2
CNDP_MBUF_EDGE_CLS_DROP = 0xFFFF

# l3fwd edges (node_ip4_api.h:28-34) and cnet edges (ip4_input_priv.h:26-31)
IP4_LOOKUP_NEXT_REWRITE, IP4_LOOKUP_NEXT_PKT_DROP = 0, 1
IP4_INPUT_NEXT_PKT_DROP, IP4_INPUT_NEXT_FORWARD, IP4_INPUT_NEXT_PROTO = 0, 1, 2

MS_RSS_KEY = bytes.fromhex(
    "6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")


class _Dir24(Structure):
    _fields_ = [("nh_sz", c_int), ("num_tbl8", c_uint32)]


class _ConfU(Union):
    _fields_ = [("dir24_8", _Dir24), ("trie", _Dir24)]


class FibConf(Structure):
    """struct cne_fib_conf (cne_fib.h:76-91)."""
    _anonymous_ = ("u",)
    _fields_ = [("type", c_int), ("default_nh", c_uint64), ("max_routes", c_int), ("u", _ConfU)]


class FibImage(Structure):
    _fields_ = [("nh_sz", c_uint32), ("tbl8_groups", c_uint32), ("tbl24", c_void_p),
                ("tbl8", c_void_p), ("def_nh", c_uint64)]


class Batch(Structure):
    """struct cndp_batch (cndp_gpu.h)."""
    _fields_ = [("mode", c_uint32), ("n", c_uint32), ("slab", c_void_p), ("slab_len", c_uint64),
                ("stride", c_uint64), ("offsets", c_void_p), ("data_off", c_uint32),
                ("buf_len", c_uint32), ("nh", c_void_p), ("hash", c_void_p), ("queue", c_void_p),
                ("edge", c_void_p), ("bins", c_void_p), ("n_bins", c_uint32), ("ptype", c_void_p),
                ("rxmeta", c_void_p)]


class MqConf(Structure):
    """struct cndp_mq_conf (cndp_gpu.h)."""
    _fields_ = [("mode", c_uint32), ("flags", c_uint32), ("batch", c_uint32), ("depth", c_uint32),
                ("max_delay_us", c_uint32), ("stage_max", c_uint32), ("umem", c_void_p),
                ("lport", c_uint16), ("rsvd", c_uint16 * 3), ("metadata", c_void_p)]


class NativeLibraryMissing(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the native library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (no CPU fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        # cndp_fib.h
        "cne_fib_create": (c_void_p, [c_char_p, POINTER(FibConf)]),
        "cne_fib_free": (None, [c_void_p]),
        "cne_fib_add": (c_int, [c_void_p, c_uint32, c_uint8, c_uint64]),
        "cne_fib_delete": (c_int, [c_void_p, c_uint32, c_uint8]),
        "cne_fib_lookup_bulk": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
        "cne_fib_get_dp": (c_void_p, [c_void_p]),
        "cne_fib_get_rib": (c_void_p, [c_void_p]),
        "cne_fib_select_lookup": (c_int, [c_void_p, c_int]),
        "cne_fib6_create": (c_void_p, [c_char_p, POINTER(FibConf)]),
        "cne_fib6_free": (None, [c_void_p]),
        "cne_fib6_add": (c_int, [c_void_p, c_void_p, c_uint8, c_uint64]),
        "cne_fib6_delete": (c_int, [c_void_p, c_void_p, c_uint8]),
        "cne_fib6_lookup_bulk": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
        "cne_fib6_get_dp": (c_void_p, [c_void_p]),
        "cne_fib6_get_rib": (c_void_p, [c_void_p]),
        "cne_fib6_select_lookup": (c_int, [c_void_p, c_int]),
        "cndp_fib_image": (c_int, [c_void_p, POINTER(FibImage)]),
        "cndp_fib6_image": (c_int, [c_void_p, POINTER(FibImage)]),
        "cndp_fib_sync": (c_int, [c_void_p, c_void_p]),
        "cndp_fib6_sync": (c_int, [c_void_p, c_void_p]),
        "cndp_fib_lookup_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]),
        "cndp_fib6_lookup_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]),
        "cndp_fib_stats": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]),
        "cndp_fib6_stats": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]),
        "cndp_fib_sync_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
        "cndp_fib6_sync_stats": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_uint64)]),
        # cndp_node.h
        "cne_node_ip4_route_add": (c_int, [c_uint32, c_uint8, c_uint16, c_int]),
        "cne_node_ip4_rewrite_add": (c_int, [c_uint16, c_void_p, c_uint8, c_uint16]),
        "ip4_rewrite_set_next": (c_int, [c_uint16, c_uint16]),
        "cne_node_ip4_add_input": (c_int, [c_void_p, c_uint32, c_uint8, c_uint32]),
        "cne_node_ip6_add_input": (c_int, [c_void_p, c_void_p, c_uint8, c_uint32]),
        "cndp_node_ip4_lookup_init": (c_int, []),
        "cndp_node_ip4_lookup_fib": (c_void_p, []),
        "cndp_node_ip4_lookup_fini": (None, []),
        "cndp_node_ip4_rewrite_get": (c_int, [c_uint16, c_void_p, POINTER(c_uint16), POINTER(c_uint16),
                                              POINTER(c_uint16)]),
        "cndp_node_ip4_rewrite_reset": (None, []),
        "cndp_node_gpu_umem_add": (c_int, [c_void_p, c_uint64]),
        "cndp_node_gpu_umem_get": (c_int, [c_uint32, POINTER(c_void_p), POINTER(c_uint64)]),
        "cndp_node_gpu_umem_reset": (None, []),
        # cndp_gpu.h
        "cndp_gpu_init": (c_int, [c_int, POINTER(c_void_p)]),
        "cndp_gpu_fini": (None, [c_void_p]),
        "cndp_gpu_device": (c_int, [c_void_p]),
        "cndp_gpu_set_rss": (c_int, [c_void_p, c_char_p, c_uint32, c_void_p, c_uint32, c_uint32]),
        "cndp_gpu_set_fib": (c_int, [c_void_p, c_void_p, c_void_p]),
        "cndp_gpu_classify": (c_int, [c_void_p, POINTER(Batch), c_void_p]),
        "cndp_gpu_stream_release": (c_int, [c_void_p, c_void_p]),
        "cndp_gpu_classify_host": (c_int, [c_void_p, POINTER(Batch)]),
        "cndp_gpu_host_register": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_void_p)]),
        "cndp_gpu_host_unregister": (c_int, [c_void_p, c_void_p]),
        "cndp_gpu_frames_alloc": (c_int, [c_int, c_uint64, c_uint32, POINTER(c_void_p)]),
        "cndp_gpu_frames_free": (c_int, [c_void_p]),
        "cndp_gpu_l3fwd_mbufs": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p, c_void_p]),
        "cndp_gpu_ip4_rewrite_set_next": (c_int, [c_void_p, c_uint16, c_uint16]),
        "cndp_gpu_ip4_rewrite_add": (c_int, [c_void_p, c_uint16, c_void_p, c_uint8, c_uint16]),
        "cndp_gpu_ip4_rewrite": (c_int, [c_void_p, POINTER(Batch), c_uint32, c_void_p, c_void_p]),
        "cndp_gpu_mac_swap": (c_int, [c_void_p, POINTER(Batch), c_void_p]),
        "cndp_gpu_classify_rewrite": (c_int, [c_void_p, POINTER(Batch), c_uint32, c_void_p, c_void_p]),
        "cndp_gpu_bin_partition": (c_int, [c_void_p, c_void_p, c_uint32, c_uint32, c_void_p,
                                           c_void_p, c_void_p]),
        "cndp_gpu_bin_ids": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_uint32,
                                     c_uint32, c_void_p, c_void_p]),
        "cndp_gpu_set_tuning": (c_int, [c_void_p, c_int, c_int]),
        "cndp_gpu_mq_create": (c_int, [c_void_p, POINTER(MqConf), POINTER(c_void_p)]),
        "cndp_gpu_mq_free": (None, [c_void_p]),
        "cndp_gpu_mq_submit": (c_int, [c_void_p, c_void_p, c_uint32]),
        "cndp_gpu_mq_flush": (c_int, [c_void_p]),
        "cndp_gpu_mq_poll": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32]),
        "cndp_gpu_mq_wait": (c_int, [c_void_p]),
        "cndp_gpu_mq_pending": (c_uint32, [c_void_p]),
        "cndp_gpu_mq_stat": (ctypes.c_int64, [c_void_p, c_int]),
        "cndp_gpu_get_stat": (ctypes.c_int64, [c_void_p, c_int]),
        "cndp_gpu_version": (c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def exported_symbols():
    """Names the C-ABI headers declare (checked against the .so by tests)."""
    import re
    names = []
    inc = os.path.join(os.path.dirname(HERE), "include")
    for h in ("cndp_fib.h", "cndp_node.h", "cndp_gpu.h"):
        with open(os.path.join(inc, h)) as f:
            txt = f.read()
        names += re.findall(r"^[A-Za-z_][\w \*]*?\b((?:cne|cndp|ip4)_\w+)\s*\(", txt, re.M)
    return sorted(set(n for n in names if not n.endswith("_fn_t")))


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise OSError(-rc, f"{what} failed: {os.strerror(-rc)}")
    return rc
