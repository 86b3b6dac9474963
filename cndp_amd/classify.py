"""Python host API of the MI355X classify path (include/cndp_gpu.h).

    c = Classifier(device=0)
    c.set_rss(key=None, reta=None, nb_queues=16)
    c.set_fib(fib4, fib6)
    out = c.classify(frames, mode=CNDP_MODE_L3FWD)      # device-resident
    out = c.classify_host(np_slab, n, ...)              # host buffers (PCIe)

Frames carry torch tensors (the slab lives in HBM when they are on cuda);
outputs are allocated as torch tensors on the same device unless given.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native as N


class Classifier:
    def __init__(self, device: int = -1):
        self._L = N.lib()
        h = ctypes.c_void_p()
        N.check(self._L.cndp_gpu_init(device, ctypes.byref(h)), "cndp_gpu_init")
        self.h = h
        self.device = self._L.cndp_gpu_device(h)
        self.reta_size = 128
        self.fib4 = None
        self.fib6 = None

    def close(self):
        if self.h:
            self._L.cndp_gpu_fini(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_rss(self, key: bytes | None = None, reta=None, nb_queues: int = 16):
        rarr = None
        size = 0
        if reta is not None:
            rarr = np.ascontiguousarray(reta, dtype=np.uint16)
            size = len(rarr)
        N.check(self._L.cndp_gpu_set_rss(self.h, key, len(key) if key else 0,
                                         rarr.ctypes.data if rarr is not None else None, size,
                                         nb_queues), "cndp_gpu_set_rss")
        self.reta_size = size or 128

    def set_tuning(self, nt: int | None = None, unroll: int | None = None,
                   blocks_per_cu: int | None = None, tile: int | None = None,
                   dir16: int | None = None, cnet_tile: int | None = None,
                   host_chunk: int | None = None, rw_wb: int | None = None,
                   cnet_spec: int | None = None, load_nt: int | None = None,
                   spec_scan: int | None = None, mbuf_hash: int | None = None,
                   cnet_fold: int | None = None, spec_grid: int | None = None,
                   spec_lists: int | None = None, spec_types: int | None = None,
                   stream_bal: int | None = None, spec_wait: int | None = None,
                   host_window: int | None = None):
        """Kernel variant knobs (cndp_gpu_set_tuning); never change results
        (spec_wait, the speculation pass's wait bound in us, -1 = fault
        injection, turns an expired wait into -EIO, never into other edges)."""
        for key, v in ((N.CNDP_TUNE_CNET_FOLD, cnet_fold), (N.CNDP_TUNE_SPEC_GRID, spec_grid),
                       (N.CNDP_TUNE_SPEC_WAIT, spec_wait), (N.CNDP_TUNE_HOST_WINDOW, host_window),
                       (N.CNDP_TUNE_SPEC_LISTS, spec_lists), (N.CNDP_TUNE_SPEC_TYPES, spec_types),
                       (N.CNDP_TUNE_STREAM_BAL, stream_bal),
                       (N.CNDP_TUNE_NT, nt), (N.CNDP_TUNE_UNROLL, unroll),
                       (N.CNDP_TUNE_BLOCKS_PER_CU, blocks_per_cu), (N.CNDP_TUNE_TILE, tile),
                       (N.CNDP_TUNE_DIR16, dir16), (N.CNDP_TUNE_CNET_TILE, cnet_tile),
                       (N.CNDP_TUNE_HOST_CHUNK, host_chunk), (N.CNDP_TUNE_RW_WB, rw_wb),
                       (N.CNDP_TUNE_CNET_SPEC, cnet_spec), (N.CNDP_TUNE_LOAD_NT, load_nt),
                       (N.CNDP_TUNE_SPEC_SCAN, spec_scan), (N.CNDP_TUNE_MBUF_HASH, mbuf_hash)):
            if v is not None:
                N.check(self._L.cndp_gpu_set_tuning(self.h, key, int(v)), "cndp_gpu_set_tuning")

    def stat(self, key: int) -> int:
        """cndp_gpu_get_stat (CNDP_STAT_*)."""
        self._L.cndp_gpu_get_stat.restype = ctypes.c_int64
        return int(N.check(self._L.cndp_gpu_get_stat(self.h, key), "cndp_gpu_get_stat"))

    def set_fib(self, fib4=None, fib6=None):
        N.check(self._L.cndp_gpu_set_fib(self.h, fib4.h if fib4 else None, fib6.h if fib6 else None),
                "cndp_gpu_set_fib")
        self.fib4, self.fib6 = fib4, fib6

    def alloc_outputs(self, n: int, n_bins: int = 64, device=None, edge: bool = True, meta: bool = False):
        import torch
        dev = device if device is not None else f"cuda:{self.device}"
        out = {
            "nh": torch.empty(n, dtype=torch.int32, device=dev),
            "hash": torch.empty(n, dtype=torch.int32, device=dev),
            "queue": torch.empty(n, dtype=torch.int16, device=dev),
            "edge": torch.empty(n, dtype=torch.uint8, device=dev) if edge else None,
            "bins": torch.zeros(n_bins + 2, dtype=torch.int64, device=dev),
            "n_bins": n_bins,
        }
        if meta:
            out["ptype"] = torch.empty(n, dtype=torch.int32, device=dev)
            out["rxmeta"] = torch.empty(n, dtype=torch.int32, device=dev)
        return out

    @staticmethod
    def _ptr(t):
        return t.data_ptr() if t is not None else None

    def batch(self, frames, mode: int, out: dict, buf_len: int = 1984, offsets_t=None) -> "N.Batch":
        b = N.Batch()
        b.mode = mode
        b.n = frames.n
        b.slab = frames.slab.data_ptr()
        b.slab_len = frames.slab.numel()
        b.stride = frames.stride
        off = offsets_t if offsets_t is not None else frames.offsets
        b.offsets = off.data_ptr() if off is not None else None
        b.data_off = frames.data_off
        b.buf_len = buf_len
        b.nh = self._ptr(out.get("nh"))
        b.hash = self._ptr(out.get("hash"))
        b.queue = self._ptr(out.get("queue"))
        b.edge = self._ptr(out.get("edge"))
        b.bins = self._ptr(out.get("bins"))
        b.n_bins = out.get("n_bins", 64)
        b.ptype = self._ptr(out.get("ptype"))
        b.rxmeta = self._ptr(out.get("rxmeta"))
        return b

    def classify(self, frames, mode: int = N.CNDP_MODE_L3FWD, out: dict | None = None,
                 n_bins: int = 64, buf_len: int = 1984, stream: int | None = None) -> dict:
        """Enqueue one classify pass on `stream` (default: torch's current
        stream of the device).  Returns the output dict (torch tensors)."""
        import torch
        if out is None:
            out = self.alloc_outputs(frames.n, n_bins, device=frames.slab.device)
        if stream is None:
            stream = torch.cuda.current_stream(frames.slab.device).cuda_stream
        b = self.batch(frames, mode, out, buf_len)
        N.check(self._L.cndp_gpu_classify(self.h, ctypes.byref(b), stream or None), "cndp_gpu_classify")
        return out

    def stream_release(self, stream: int) -> None:
        """cndp_gpu_stream_release: call before destroying a HIP stream given to
        classify (torch's pooled streams are never destroyed)."""
        N.check(self._L.cndp_gpu_stream_release(self.h, stream or None), "cndp_gpu_stream_release")

    @staticmethod
    def _hptr(x):
        """Address of a host buffer (numpy array or CPU torch tensor)."""
        if x is None:
            return None
        if isinstance(x, np.ndarray):
            return x.ctypes.data
        return x.data_ptr()

    def classify_host(self, slab, n: int, mode: int, stride: int = 64, offsets=None,
                      data_off: int = 0, buf_len: int = 1984, n_bins: int = 64, out: dict | None = None,
                      slab_len: int | None = None) -> dict:
        """Host buffers in, host results out (streamed H2D / classify / D2H,
        PCIe-bound).  `slab`, `offsets` and the arrays of `out` may be numpy
        arrays or CPU torch tensors (pinned ones give full DMA rate)."""
        if isinstance(slab, np.ndarray):
            slab = np.ascontiguousarray(slab, dtype=np.uint8)
            nbytes = slab.nbytes
        else:
            nbytes = slab.numel() * slab.element_size()
        if out is None:
            out = {"nh": np.zeros(n, np.uint32), "hash": np.zeros(n, np.uint32),
                   "queue": np.zeros(n, np.uint16), "edge": np.zeros(n, np.uint8),
                   "bins": np.zeros(n_bins + 2, np.uint64)}
        if offsets is not None and isinstance(offsets, np.ndarray):
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        b = N.Batch()
        b.mode, b.n, b.slab = mode, n, self._hptr(slab)
        b.slab_len = nbytes if slab_len is None else slab_len
        b.stride, b.offsets, b.data_off, b.buf_len = stride, self._hptr(offsets), data_off, buf_len
        b.nh, b.hash, b.queue = self._hptr(out.get("nh")), self._hptr(out.get("hash")), self._hptr(out.get("queue"))
        b.edge, b.bins, b.n_bins = self._hptr(out.get("edge")), self._hptr(out.get("bins")), n_bins
        b.ptype, b.rxmeta = self._hptr(out.get("ptype")), self._hptr(out.get("rxmeta"))
        N.check(self._L.cndp_gpu_classify_host(self.h, ctypes.byref(b)), "cndp_gpu_classify_host")
        return out

    def host_register(self, buf) -> int:
        """Pin + map a host buffer; returns its device address (zero-copy)."""
        d = ctypes.c_void_p()
        size = buf.nbytes if isinstance(buf, np.ndarray) else buf.numel() * buf.element_size()
        N.check(self._L.cndp_gpu_host_register(self.h, self._hptr(buf), size, ctypes.byref(d)),
                "cndp_gpu_host_register")
        return d.value

    def host_unregister(self, buf):
        N.check(self._L.cndp_gpu_host_unregister(self.h, self._hptr(buf)), "cndp_gpu_host_unregister")

    def classify_ptrs(self, mode: int, n: int, slab: int, slab_len: int, out: dict, stride: int = 64,
                      data_off: int = 0, offsets: int | None = None, buf_len: int = 1984,
                      n_bins: int = 64, stream: int | None = None):
        """cndp_gpu_classify on raw device-visible addresses (e.g. a
        host_register'd UMEM): outputs are torch device tensors."""
        import torch
        b = N.Batch()
        b.mode, b.n, b.slab, b.slab_len = mode, n, slab, slab_len
        b.stride, b.offsets, b.data_off, b.buf_len = stride, offsets, data_off, buf_len
        b.nh, b.hash, b.queue = self._ptr(out.get("nh")), self._ptr(out.get("hash")), self._ptr(out.get("queue"))
        b.edge, b.bins, b.n_bins = self._ptr(out.get("edge")), self._ptr(out.get("bins")), n_bins
        b.ptype, b.rxmeta = self._ptr(out.get("ptype")), self._ptr(out.get("rxmeta"))
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        N.check(self._L.cndp_gpu_classify(self.h, ctypes.byref(b), stream or None), "cndp_gpu_classify")
        return out

    # -- ip4_rewrite / cndpfwd loopback (in place on the device slab) -------
    def rewrite_set_next(self, port_id: int, next_index: int):
        """ip4_rewrite_set_next (ip4_rewrite.c:252-263)."""
        N.check(self._L.cndp_gpu_ip4_rewrite_set_next(self.h, port_id, next_index), "ip4_rewrite_set_next")

    def rewrite_add(self, next_hop: int, rewrite_data: bytes, dst_port: int) -> int:
        """cne_node_ip4_rewrite_add (ip4_rewrite.c:265-295); returns its rc."""
        buf = ctypes.create_string_buffer(bytes(rewrite_data), max(1, len(rewrite_data)))
        return self._L.cndp_gpu_ip4_rewrite_add(self.h, next_hop, buf, len(rewrite_data), dst_port)

    def ip4_rewrite(self, frames, nh, burst: int = 256, tx_edge=None, stream: int | None = None):
        """Rewrite the frames routed to ip4_rewrite (l3fwd classify value
        `nh` with edge 0) in place; returns the tx edge per packet (u16 as
        int16 tensor, 0xFFFF = not rewritten)."""
        import torch
        if tx_edge is None:
            tx_edge = torch.empty(frames.n, dtype=torch.int16, device=frames.slab.device)
        b = N.Batch()
        b.mode, b.n, b.slab, b.slab_len = N.CNDP_MODE_L3FWD, frames.n, frames.slab.data_ptr(), frames.slab.numel()
        b.stride, b.data_off = frames.stride, frames.data_off
        b.offsets = frames.offsets.data_ptr() if frames.offsets is not None else None
        b.nh = nh.data_ptr()
        if stream is None:
            stream = torch.cuda.current_stream(frames.slab.device).cuda_stream
        N.check(self._L.cndp_gpu_ip4_rewrite(self.h, ctypes.byref(b), burst, tx_edge.data_ptr(), stream or None),
                "cndp_gpu_ip4_rewrite")
        return tx_edge

    def classify_rewrite(self, frames, out: dict | None = None, burst: int = 256, tx_edge=None,
                         stream: int | None = None):
        """l3fwd classify + ip4_rewrite (fused for packed 64-B slots, 256-bursts)."""
        import torch
        if out is None:
            out = self.alloc_outputs(frames.n, 64, device=frames.slab.device, edge=False)
        if tx_edge is None:
            tx_edge = torch.empty(frames.n, dtype=torch.int16, device=frames.slab.device)
        if stream is None:
            stream = torch.cuda.current_stream(frames.slab.device).cuda_stream
        b = self.batch(frames, N.CNDP_MODE_L3FWD, out)
        N.check(self._L.cndp_gpu_classify_rewrite(self.h, ctypes.byref(b), burst, tx_edge.data_ptr(),
                                                  stream or None), "cndp_gpu_classify_rewrite")
        return out, tx_edge

    def mac_swap(self, frames, stream: int | None = None):
        """cndpfwd loopback MAC swap on every frame (in place)."""
        import torch
        b = N.Batch()
        b.n, b.slab, b.slab_len = frames.n, frames.slab.data_ptr(), frames.slab.numel()
        b.stride, b.data_off = frames.stride, frames.data_off
        b.offsets = frames.offsets.data_ptr() if frames.offsets is not None else None
        if stream is None:
            stream = torch.cuda.current_stream(frames.slab.device).cuda_stream
        N.check(self._L.cndp_gpu_mac_swap(self.h, ctypes.byref(b), stream or None), "cndp_gpu_mac_swap")

    def bin_partition(self, bin_of, n_bins: int, stream: int | None = None):
        """Stable partition of packet indices by bin id (per-edge streams)."""
        import torch
        n = bin_of.numel()
        start = torch.empty(n_bins + 3, dtype=torch.int32, device=bin_of.device)
        order = torch.empty(max(n, 1), dtype=torch.int32, device=bin_of.device)
        if stream is None:
            stream = torch.cuda.current_stream(bin_of.device).cuda_stream
        N.check(self._L.cndp_gpu_bin_partition(self.h, bin_of.data_ptr(), n, n_bins, start.data_ptr(),
                                               order.data_ptr(), stream or None), "cndp_gpu_bin_partition")
        return start, order[:n]

    def bin_ids(self, mode: int, out: dict, n: int, n_bins: int, stream: int | None = None):
        import torch
        dev = out["queue"].device
        bins = torch.empty(n, dtype=torch.int16, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev).cuda_stream
        N.check(self._L.cndp_gpu_bin_ids(self.h, mode, self._ptr(out.get("nh")), self._ptr(out.get("edge")),
                                         self._ptr(out.get("queue")), n, n_bins, bins.data_ptr(),
                                         stream or None), "cndp_gpu_bin_ids")
        return bins
