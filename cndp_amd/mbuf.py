"""pktmbuf_t pools in host memory and the asynchronous node queue (cndp_gpu_mq_*).

MbufPool lays frames out the way CNDP's pktmbuf pool does inside an AF_XDP
UMEM (lib/core/pktmbuf/pktmbuf.h:102-204, pktmbuf.c:60-80): 2 KiB frames, the
64-byte pktmbuf_t header at the frame start, buf_addr = frame + 64,
buf_len = 1984, data_off = 192, so packet data starts at frame + 256.

MbufQueue wraps the C-ABI queue: submit bursts of mbuf pointers, poll the
finished ones (fields written back, next edges returned), in order.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native as N

# struct pktmbuf_s, 64 bytes (pktmbuf.h:102-204)
MBUF_DT = np.dtype([("pooldata", "<u8"), ("buf_addr", "<u8"), ("hash", "<u4"), ("meta_index", "<u4"),
                    ("data_off", "<u2"), ("lport", "<u2"), ("buf_len", "<u2"), ("data_len", "<u2"),
                    ("packet_type", "<u4"), ("refcnt", "<u2"), ("rsvd16", "<u2"), ("tx_offload", "<u8"),
                    ("ol_flags", "<u8"), ("udata64", "<u8")])
assert MBUF_DT.itemsize == 64

FRAME = 2048
HDR = 64
HEADROOM = 192          # data_off of a fresh mbuf: packet data at frame + 256
BUF_LEN = FRAME - HDR   # 1984


class MbufPool:
    """n mbufs in one page-aligned host buffer (optionally registered with a
    Classifier for zero-copy).  hugepages: an anonymous mapping advised for
    2 MiB transparent huge pages, 2 MiB-aligned, as a UMEM from CNDP's
    mmap_alloc(MMAP_HUGEPAGE_2MB) would be (lib/core/mmap/cne_mmap.h:29)."""

    def __init__(self, n: int, hugepages: bool = False):
        self.n = n
        if hugepages:
            import mmap
            self._mm = mmap.mmap(-1, n * FRAME + (2 << 20), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
            self._mm.madvise(mmap.MADV_HUGEPAGE)
            raw = np.frombuffer(self._mm, np.uint8)
            a = (-raw.ctypes.data) % (2 << 20)
        else:
            raw = np.zeros(n * FRAME + 4096, np.uint8)
            a = (-raw.ctypes.data) % 4096
        self._raw = raw
        self.mem = raw[a:a + n * FRAME]
        self.base = self.mem.ctypes.data
        rows = self.mem.reshape(n, FRAME)
        self.hdr = rows[:, :HDR].view(MBUF_DT)[:, 0]
        self.hdr["buf_addr"] = self.base + np.arange(n, dtype=np.uint64) * FRAME + HDR
        self.hdr["buf_len"] = BUF_LEN
        self.hdr["data_off"] = HEADROOM
        self.hdr["refcnt"] = 1

    def addr(self, i: int) -> int:
        return self.base + i * FRAME

    def data_pos(self) -> np.ndarray:
        """Byte offset of each mbuf's packet data inside self.mem."""
        return (np.arange(self.n, dtype=np.uint64) * FRAME + HDR + self.hdr["data_off"].astype(np.uint64))

    def fill(self, frames, lengths=None, max_bytes: int = BUF_LEN - HEADROOM):
        """Copy frame i of a pktgen.Frames batch into mbuf i; data_len = its
        length (frames.lengths, else the slot size), at most max_bytes."""
        slab = frames.slab.cpu().numpy() if hasattr(frames.slab, "cpu") else np.asarray(frames.slab)
        n = frames.n
        assert n <= self.n
        if frames.offsets is not None:
            offs = frames.offsets.cpu().numpy().astype(np.int64)
        else:
            offs = np.arange(n, dtype=np.int64) * frames.stride
        offs = offs + frames.data_off
        if lengths is None:
            if frames.lengths is not None:
                lengths = frames.lengths.cpu().numpy().astype(np.int64)
            else:
                lengths = np.full(n, frames.stride, np.int64)
        dpos = self.data_pos()
        if frames.offsets is None and frames.lengths is None and slab.size >= n * frames.stride \
                and np.all(self.hdr["data_off"][:n] == HEADROOM):
            ln = int(min(frames.stride, max_bytes))   # fixed-stride slab: one strided copy
            rows = self.mem.reshape(self.n, FRAME)[:n, HDR + HEADROOM:HDR + HEADROOM + ln]
            rows[:] = slab[:n * frames.stride].reshape(n, frames.stride)[:, frames.data_off:frames.data_off + ln]
            self.hdr["data_len"][:n] = lengths
            return
        for i in range(n):
            o = int(offs[i])
            ln = int(min(lengths[i], max_bytes, max(0, slab.size - o)))
            d = int(dpos[i])
            self.mem[d:d + ln] = slab[o:o + ln]
            self.hdr["data_len"][i] = lengths[i]

    def ptrs(self, idx) -> "ctypes.Array":
        idx = np.asarray(idx, dtype=np.int64)
        arr = (ctypes.c_void_p * len(idx))()
        addrs = (self.base + idx.astype(np.uint64) * FRAME).tolist()
        arr[:] = addrs
        return arr

    def index_of(self, addrs) -> np.ndarray:
        return ((np.asarray(addrs, dtype=np.uint64) - np.uint64(self.base)) // FRAME).astype(np.int64)


class MbufQueue:
    """cndp_gpu_mq_* over a Classifier's context."""

    METADATA_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p)

    def __init__(self, cl, mode: int, flags: int = 0, batch: int = 8192, depth: int = 4,
                 max_delay_us: int = 50, umem=None, lport: int = 0, stage_max: int = 0, metadata=None):
        """metadata: cnet's pktmbuf_metadata hook, a Python function of the mbuf
        address returning the metadata address (None: m + 64)."""
        self._L = N.lib()
        c = N.MqConf()
        c.mode, c.flags, c.batch, c.depth = mode, flags, batch, depth
        c.max_delay_us, c.stage_max, c.lport = max_delay_us, stage_max, lport
        c.umem = umem
        self._md_fn = self.METADATA_FN(metadata) if metadata else None  # kept alive with the queue
        if self._md_fn:
            c.metadata = ctypes.cast(self._md_fn, ctypes.c_void_p)
        h = ctypes.c_void_p()
        N.check(self._L.cndp_gpu_mq_create(cl.h, ctypes.byref(c), ctypes.byref(h)), "cndp_gpu_mq_create")
        self.h = h
        self.cl = cl

    def close(self):
        if self.h:
            self._L.cndp_gpu_mq_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def submit(self, ptrs, n: int | None = None) -> int:
        n = len(ptrs) if n is None else n
        return N.check(self._L.cndp_gpu_mq_submit(self.h, ptrs, n), "cndp_gpu_mq_submit")

    def flush(self):
        N.check(self._L.cndp_gpu_mq_flush(self.h), "cndp_gpu_mq_flush")

    def wait(self):
        N.check(self._L.cndp_gpu_mq_wait(self.h), "cndp_gpu_mq_wait")

    @property
    def pending(self) -> int:
        return self._L.cndp_gpu_mq_pending(self.h)

    def poll(self, max_n: int = 1 << 16):
        out = (ctypes.c_void_p * max_n)()
        edges = np.zeros(max_n, np.uint16)
        k = N.check(self._L.cndp_gpu_mq_poll(self.h, out, edges.ctypes.data, max_n), "cndp_gpu_mq_poll")
        return np.array([x or 0 for x in out[:k]], dtype=np.uint64), edges[:k].copy()

    def run(self, pool: MbufPool, idx, bursts):
        """Submit mbufs pool[idx] as graph bursts of the given sizes, polling
        as a node would (drain while the queue is full), until every mbuf has
        come back.  Returns (addresses, edges) in completion order."""
        idx = np.asarray(idx, dtype=np.int64)
        got_a, got_e = [], []
        pos = 0
        for b in bursts:
            ptrs = pool.ptrs(idx[pos:pos + b])
            done = 0
            while done < b:
                k = self.submit(ctypes.addressof(ptrs) + done * ctypes.sizeof(ctypes.c_void_p), b - done)
                done += k
                a, e = self.poll()
                got_a.append(a)
                got_e.append(e)
                if k == 0 and a.size == 0:
                    self.wait()
            pos += b
        for _ in range(1 << 20):
            if not self.pending:
                break
            self.flush()
            self.wait()
            a, e = self.poll()
            got_a.append(a)
            got_e.append(e)
        return np.concatenate(got_a) if got_a else np.zeros(0, np.uint64), \
            np.concatenate(got_e) if got_e else np.zeros(0, np.uint16)
