"""Deterministic synthetic packet / route generation for the BASELINE configs.

Every per-packet value is a counter-based hash of (seed, packet index,
field), computed with 32-bit integer arithmetic on torch tensors, so the
same frames come out on the CPU (tests, oracle) and directly in HBM on the
GPU (bench) without a host round trip.  Default seed 0x43444E50 ("CDNP").

Frames follow examples/cndpfwd/main.c:53-97 (setup_pkt_udp_ip_headers):
Ethernet II, IPv4 (IHL 5, TTL 64, valid header checksum), UDP.  Only the
first 64 bytes of a frame carry headers; payload bytes are zero.
"""
from __future__ import annotations

import torch

SEED = 0x43444E50
M32 = 0xFFFFFFFF


def _mul32(x: torch.Tensor, c: int) -> torch.Tensor:
    # (x * c) mod 2^32 for 0 <= x < 2^32 without int64 overflow
    lo = (x * (c & 0xFFFF)) & M32
    hi = ((x * (c >> 16)) & 0xFFFF) << 16
    return (lo + hi) & M32


def h32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 integer hash on int64 tensors holding u32 values."""
    x = x & M32
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    x = x ^ (x >> 16)
    return x


def _h32i(v: int) -> int:
    return int(h32(torch.tensor([v & M32], dtype=torch.int64))[0])


def rnd(seed: int, idx: torch.Tensor, field: int) -> torch.Tensor:
    """u32 pseudo-random value per index for a given field."""
    salt = _h32i(seed * 131 + field * 0x9E3779B9)
    return h32(h32((idx & M32) ^ salt) ^ (idx >> 32) ^ (field * 0x27D4EB2F & M32))


def put_be(hdr: torch.Tensor, off: int, val, nbytes: int) -> None:
    for k in range(nbytes):
        sh = 8 * (nbytes - 1 - k)
        if isinstance(val, int):
            hdr[:, off + k] = (val >> sh) & 0xFF
        else:
            hdr[:, off + k] = ((val >> sh) & 0xFF).to(torch.uint8)


def ipv4_cksum(words) -> torch.Tensor:
    s = sum(words)
    s = (s >> 16) + (s & 0xFFFF)
    s = (s >> 16) + (s & 0xFFFF)
    return (~s) & 0xFFFF


# ---------------------------------------------------------------------------
# route sets
# ---------------------------------------------------------------------------
def l3fwd_routes(n_routes: int = 1024, n_nh: int = 64):
    """C3: 896 x /24 in 10.0.0.0/14 + 128 x /25../32, one per /24 of
    10.4.0.0/16; next hop = index % 64.  Returns [(ip, depth, nh_id)]."""
    out = []
    n24 = n_routes * 7 // 8
    for i in range(n24):
        out.append(((10 << 24) + (i << 8), 24, i % n_nh))
    for k in range(n_routes - n24):
        depth = 25 + (k % 8)
        host = _h32i(0xC0FFEE + k) & 0xFF
        mask = (0xFF << (32 - depth)) & 0xFF
        ip = (10 << 24) | (4 << 16) | ((k & 0xFF) << 8) | (host & mask)
        out.append((ip, depth, (n24 + k) % n_nh))
    return out


def v6_routes(n_routes: int = 1024):
    """C4: prefixes /32../64 inside 2001:db8::/32 (one /32, the rest /33../64).
    Returns [(ip16 bytes, depth, index)]."""
    out = []
    for i in range(n_routes):
        depth = 32 if i == 0 else 33 + ((i - 1) % 32)
        w1 = _h32i(0xBEEF00 + i)
        bits = depth - 32
        w1 &= ((0xFFFFFFFF << (32 - bits)) & M32) if bits else 0
        ip = (0x20010DB8 << 96) | (w1 << 64)
        out.append((ip.to_bytes(16, "big"), depth, i))
    return out


def _route_tensors(routes, device):
    ip = torch.tensor([r[0] for r in routes], dtype=torch.int64, device=device)
    dp = torch.tensor([r[1] for r in routes], dtype=torch.int64, device=device)
    return ip, dp


# ---------------------------------------------------------------------------
# header builders: hdr is an [n, 64] uint8 tensor (first 64 bytes of frames)
# ---------------------------------------------------------------------------
def _eth(hdr, etype: int):
    put_be(hdr, 0, 0x020000000001, 6)
    put_be(hdr, 6, 0x020000000002, 6)
    put_be(hdr, 12, etype, 2)


def ipv4_udp_headers(idx: torch.Tensor, frame_len, seed: int = SEED, routes=None,
                     in_route_frac: float = 0.9, proto: int = 17) -> torch.Tensor:
    n = idx.numel()
    dev = idx.device
    hdr = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    _eth(hdr, 0x0800)
    if isinstance(frame_len, int):
        frame_len = torch.full((n,), frame_len, dtype=torch.int64, device=dev)
    tot = frame_len - 14
    ident = rnd(seed, idx, 2) & 0xFFFF
    src = rnd(seed, idx, 1)
    r5 = rnd(seed, idx, 5)
    if routes is not None and len(routes):
        rip, rdp = _route_tensors(routes, dev)
        ri = rnd(seed, idx, 4) % len(routes)
        depth = rdp[ri]
        hostmask = (M32 >> depth) & M32
        dst_in = (rip[ri] & ~hostmask & M32) | (r5 & hostmask)
        uniform = (rnd(seed, idx, 6) % 1000) >= int(round(in_route_frac * 1000))
        dst = torch.where(uniform, r5, dst_in)
    else:
        dst = r5
    ports = rnd(seed, idx, 3)
    ip = 14
    hdr[:, ip] = 0x45
    put_be(hdr, ip + 2, tot, 2)
    put_be(hdr, ip + 4, ident, 2)
    hdr[:, ip + 8] = 64
    hdr[:, ip + 9] = proto
    ck = ipv4_cksum([0x4500, tot, ident, 0, (64 << 8) | proto, src >> 16, src & 0xFFFF,
                     dst >> 16, dst & 0xFFFF])
    put_be(hdr, ip + 10, ck, 2)
    put_be(hdr, ip + 12, src, 4)
    put_be(hdr, ip + 16, dst, 4)
    put_be(hdr, 34, ports >> 16, 2)
    put_be(hdr, 36, ports & 0xFFFF, 2)
    put_be(hdr, 38, tot - 20, 2)
    return hdr


def ipv6_udp_headers(idx: torch.Tensor, frame_len, seed: int = SEED, routes=None,
                     in_route_frac: float = 0.9) -> torch.Tensor:
    n = idx.numel()
    dev = idx.device
    hdr = torch.zeros((n, 64), dtype=torch.uint8, device=dev)
    _eth(hdr, 0x86DD)
    if isinstance(frame_len, int):
        frame_len = torch.full((n,), frame_len, dtype=torch.int64, device=dev)
    ip = 14
    flow = rnd(seed, idx, 12) & 0xFFFFF
    put_be(hdr, ip, (6 << 28) | flow, 4)
    put_be(hdr, ip + 4, frame_len - 54, 2)
    hdr[:, ip + 6] = 17
    hdr[:, ip + 7] = 64
    for k in range(4):
        put_be(hdr, ip + 8 + 4 * k, rnd(seed, idx, 20 + k), 4)
    d = [rnd(seed, idx, 30 + k) for k in range(4)]
    if routes is not None and len(routes):
        rw0 = torch.tensor([int.from_bytes(r[0][0:4], "big") for r in routes], dtype=torch.int64, device=dev)
        rw1 = torch.tensor([int.from_bytes(r[0][4:8], "big") for r in routes], dtype=torch.int64, device=dev)
        rdp = torch.tensor([r[1] for r in routes], dtype=torch.int64, device=dev)
        ri = rnd(seed, idx, 34) % len(routes)
        bits = (rdp[ri] - 32).clamp(min=0, max=32)
        keep = (M32 << (32 - bits)) & M32
        w1 = (rw1[ri] & keep) | (d[1] & ~keep & M32)
        uniform = (rnd(seed, idx, 35) % 1000) >= int(round(in_route_frac * 1000))
        d[0] = torch.where(uniform, d[0], rw0[ri])
        d[1] = torch.where(uniform, d[1], w1)
    for k in range(4):
        put_be(hdr, ip + 24 + 4 * k, d[k], 4)
    ports = rnd(seed, idx, 36)
    put_be(hdr, 54, ports >> 16, 2)
    put_be(hdr, 56, ports & 0xFFFF, 2)
    put_be(hdr, 58, frame_len - 54, 2)
    return hdr


# ---------------------------------------------------------------------------
# batch layouts
# ---------------------------------------------------------------------------
class Frames:
    """A frame slab plus its layout (what struct cndp_batch describes)."""

    def __init__(self, slab, n, stride=0, offsets=None, data_off=0, lengths=None):
        self.slab = slab           # uint8 tensor
        self.n = n
        self.stride = stride
        self.offsets = offsets     # int64 tensor or None
        self.data_off = data_off
        self.lengths = lengths     # int64 tensor (frame bytes) or None

    @property
    def slab_len(self) -> int:
        return self.slab.numel()

    @property
    def header_bytes(self) -> int:
        return self.n * 64


class _FrameMemory:
    """cndp_gpu_frames_alloc memory (include/cndp_gpu.h) exposed to torch
    through __cuda_array_interface__; torch holds this object until the
    tensor's storage dies, and its finalizer frees the memory."""

    def __init__(self, nbytes: int, index: int, cached: bool):
        import ctypes
        from . import native as N
        self._L = N.lib()
        p = ctypes.c_void_p()
        N.check(self._L.cndp_gpu_frames_alloc(index, nbytes, N.CNDP_FRAMES_CACHED if cached else 0,
                                              ctypes.byref(p)), "cndp_gpu_frames_alloc")
        self.ptr = p.value
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 2, "strides": None}

    def __del__(self):
        if getattr(self, "ptr", None):
            self._L.cndp_gpu_frames_free(self.ptr)
            self.ptr = None


def frame_slab(nbytes: int, device="cpu", cached: bool = False) -> torch.Tensor:
    """A zeroed uint8 frame slab: on a GPU, device frame memory from
    cndp_gpu_frames_alloc (uncached unless `cached`: the receive-ring memory
    the classify kernels read windows from); on the CPU a
    plain tensor."""
    device = torch.device(device)
    if device.type != "cuda":
        return torch.zeros(nbytes, dtype=torch.uint8, device=device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = torch.as_tensor(_FrameMemory(nbytes, idx, cached), device=device)
    t.zero_()
    return t


def _slab(nbytes: int, device, frame_mem: str | None) -> torch.Tensor:
    # frame_mem: None = a torch tensor, "uncached" / "cached" = cndp_gpu_frames_alloc memory
    if frame_mem is None or torch.device(device).type != "cuda":
        return torch.zeros(nbytes, dtype=torch.uint8, device=device)
    return frame_slab(nbytes, device, cached=frame_mem == "cached")


def packed_ipv4(n: int, slot: int = 64, frame_len: int = 60, seed: int = SEED, routes=None,
                device="cpu", in_route_frac: float = 0.9, chunk: int = 1 << 22,
                frame_mem: str | None = None) -> Frames:
    """C2/C3 (slot 64) and C5 (slot 1536, frame 1500) fixed-stride slabs."""
    slab = _slab(n * slot, device, frame_mem)
    view = slab.view(n, slot)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        idx = torch.arange(s, e, dtype=torch.int64, device=device)
        view[s:e, :64] = ipv4_udp_headers(idx, frame_len, seed, routes, in_route_frac)
    return Frames(slab, n, stride=slot)


def umem_ipv4(n: int, seed: int = SEED, routes=None, device="cpu", frame_len: int = 60) -> Frames:
    """AF_XDP UMEM mirror: 2 KiB frames, 64-B pktmbuf header, data at +256
    (pktmbuf.h:102-204, pktmbuf.c:60-80)."""
    slab = torch.zeros(n * 2048, dtype=torch.uint8, device=device)
    view = slab.view(n, 2048)
    chunk = 1 << 20
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        idx = torch.arange(s, e, dtype=torch.int64, device=device)
        view[s:e, 256:320] = ipv4_udp_headers(idx, frame_len, seed, routes)
    return Frames(slab, n, stride=2048, data_off=256)


IMIX_SIZES = (64, 570, 1500)
IMIX_WEIGHTS = (7, 4, 1)


def imix(n: int, seed: int = SEED, v4routes=None, v6routes=None, device="cpu",
         v6_frac: float = 0.5, frame_mem: str | None = None, family_run: int = 0) -> Frames:
    """C4: IMIX 64/570/1500 at 7:4:1, IPv4/IPv6 mix, packed at roundup(len, 64).
    family_run > 0: the address family drawn once per run of that many frames
    (measurement of one-family wave tiles; C4 itself draws it per frame)."""
    idx = torch.arange(n, dtype=torch.int64, device=device)
    pick = rnd(seed, idx, 40) % 12
    size = torch.where(pick < 7, torch.full_like(pick, 64),
                       torch.where(pick < 11, torch.full_like(pick, 570), torch.full_like(pick, 1500)))
    slot = (size + 63) // 64 * 64
    offsets = torch.cumsum(slot, 0) - slot
    total = int(offsets[-1] + slot[-1]) if n else 0
    slab = _slab(max(total, 64), device, frame_mem)
    rows = slab.view(-1, 64)
    frame_len = size - 4
    is6 = (rnd(seed, idx // family_run if family_run > 0 else idx, 41) % 1000) < int(round(v6_frac * 1000))
    chunk = 1 << 21
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        sl = slice(s, e)
        h4 = ipv4_udp_headers(idx[sl], frame_len[sl], seed, v4routes)
        h6 = ipv6_udp_headers(idx[sl], frame_len[sl], seed, v6routes)
        hdr = torch.where(is6[sl, None], h6, h4)
        rows[offsets[sl] // 64] = hdr
    return Frames(slab, n, offsets=offsets, lengths=frame_len)


def corrupt_cksum(frames: Frames, every: int = 1024, seed: int = SEED) -> int:
    """C5: flip the IPv4 checksum of 1 in `every` packets; returns how many."""
    dev = frames.slab.device
    idx = torch.arange(frames.n, dtype=torch.int64, device=dev)
    bad = (rnd(seed, idx, 50) % every) == 0
    base = (frames.offsets if frames.offsets is not None else idx * frames.stride) + frames.data_off
    pos = base[bad] + 14 + 10
    frames.slab[pos] ^= 0x5A
    return int(bad.sum())


def fuzz_frames(n: int, seed: int = 1, slot: int = 128, device="cpu") -> Frames:
    """Random frames steered through every cne_get_ptype branch: ethertypes
    {IPv4, IPv6, VLAN, QinQ, ARP, MPLS, random}, IHL 0..15, IPv4 fragments,
    IPv6 extension chains, GRE / IPIP / IPv6-in-IP tunnels, GTP ports, and a
    ragged tail (the last frames run past the slab end)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    raw = torch.randint(0, 256, (n, slot), dtype=torch.uint8, generator=g)
    choice = torch.randint(0, 10, (n,), generator=g)
    ets = [0x0800, 0x0800, 0x0800, 0x86DD, 0x86DD, 0x8100, 0x88A8, 0x0806, 0x8847, -1]
    protos = torch.tensor([6, 17, 132, 47, 4, 41, 8, 129, 1, 0, 43, 44, 60, 59, 50])
    for ci, et in enumerate(ets):
        m = choice == ci
        k = int(m.sum())
        if k == 0 or et < 0:
            continue
        rows = raw[m]
        rows[:, 12] = et >> 8
        rows[:, 13] = et & 0xFF
        l3 = 14
        if et in (0x8100, 0x88A8):
            inner = torch.tensor([0x0800, 0x86DD, 0x0806])[torch.randint(0, 3, (k,), generator=g)]
            off = 16 if et == 0x8100 else 20
            rows[:, off] = (inner >> 8).to(torch.uint8)
            rows[:, off + 1] = (inner & 0xFF).to(torch.uint8)
            l3 = 18 if et == 0x8100 else 22
        # IPv4-looking header at l3 (harmless for IPv6 rows: overwritten below)
        ihl = torch.where(torch.rand(k, generator=g) < 0.7, torch.full((k,), 5),
                          torch.randint(0, 16, (k,), generator=g))
        rows[:, l3] = (0x40 | ihl).to(torch.uint8)
        fr = torch.rand(k, generator=g) < 0.85
        rows[fr, l3 + 6] = 0
        rows[fr, l3 + 7] = 0
        rows[:, l3 + 9] = protos[torch.randint(0, len(protos), (k,), generator=g)].to(torch.uint8)
        if et == 0x86DD:
            rows[:, l3] = 0x60
            rows[:, l3 + 6] = protos[torch.randint(0, len(protos), (k,), generator=g)].to(torch.uint8)
            rows[:, l3 + 4] = torch.randint(0, 8, (k,), generator=g).to(torch.uint8)
            # keep extension header lengths small so chains stay in the frame
            rows[:, l3 + 41] = torch.randint(0, 2, (k,), generator=g).to(torch.uint8)
        # GTP-U / GTP-C destination ports on some UDP rows
        gtp = torch.rand(k, generator=g) < 0.2
        port = torch.where(torch.rand(k, generator=g) < 0.5, torch.tensor(2152), torch.tensor(2123))
        l4 = l3 + 20
        rows[gtp, l4 + 2] = (port[gtp] >> 8).to(torch.uint8)
        rows[gtp, l4 + 3] = (port[gtp] & 0xFF).to(torch.uint8)
        raw[m] = rows
    # a few valid checksums so ip4_input sees both outcomes
    okm = torch.rand(n, generator=g) < 0.5
    rows = raw[okm]
    if rows.shape[0]:
        rows[:, 14] = 0x45
        rows[:, 24] = 0
        rows[:, 25] = 0
        w = rows[:, 14:34].to(torch.int64).view(-1, 10, 2)
        s = (w[:, :, 0] << 8 | w[:, :, 1]).sum(1)
        ck = ipv4_cksum([s])
        rows[:, 24] = (ck >> 8).to(torch.uint8)
        rows[:, 25] = (ck & 0xFF).to(torch.uint8)
        raw[okm] = rows
    slab = raw.reshape(-1)[: n * slot - 37].contiguous()  # ragged tail
    return Frames(slab.to(device), n, stride=slot)


def cndpfwd_udp(n: int, pkt_len: int = 60, src_mac: bytes = bytes.fromhex("020000000001")) -> Frames:
    """C1: the frame examples/cndpfwd builds (setup_pkt_udp_ip_headers,
    main.c:53-97): dst MAC ff:ff:ff:ff:ff:ff, the port's MAC as source (a
    synthetic locally administered one here), IPv4 IHL 5, TTL 64, UDP,
    198.18.0.1 -> 198.18.0.2, ports 9 -> 9, IPv4 and UDP checksums set,
    pkt_len bytes (60: a 64-B frame with its FCS).  Packed 64-B slots."""
    import struct
    f = bytearray(64)
    f[0:6] = b"\xff" * 6
    f[6:12] = src_mac
    f[12:14] = b"\x08\x00"
    ip_len = pkt_len - 14
    ip = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, ip_len, 0, 0, 64, 17, 0,
                               bytes([198, 18, 0, 1]), bytes([198, 18, 0, 2])))
    s = sum(struct.unpack(">10H", bytes(ip)))
    s = (s >> 16) + (s & 0xFFFF)
    s = (s >> 16) + (s & 0xFFFF)
    ip[10:12] = struct.pack(">H", (~s) & 0xFFFF)
    udp_len = pkt_len - 14 - 20
    udp = bytearray(struct.pack(">HHHH", 9, 9, udp_len, 0)) + bytes(udp_len - 8)
    # cne_ipv4_udptcp_cksum (cne_ip.h:311-325): pseudo header + UDP, 0 -> 0xffff
    ph = bytes([198, 18, 0, 1, 198, 18, 0, 2, 0, 17]) + struct.pack(">H", udp_len)
    data = ph + bytes(udp)
    if len(data) & 1:
        data += b"\x00"
    c = sum(struct.unpack(f">{len(data) // 2}H", data))
    while c >> 16:
        c = (c >> 16) + (c & 0xFFFF)
    c = (~c) & 0xFFFF
    udp[6:8] = struct.pack(">H", c or 0xFFFF)
    f[14:34] = ip
    f[34:34 + len(udp)] = udp[: 64 - 34]
    slab = torch.tensor(list(bytes(f)) * n, dtype=torch.uint8)
    return Frames(slab, n, stride=64, lengths=torch.full((n,), pkt_len, dtype=torch.int64))
