"""Python mirror of CNDP's FIB API (lib/usr/clib/fib/cne_fib.h, cne_fib6.h)
over libcndp_gpu.so.  Same operation names, argument meaning and return
codes (0 / negative errno).  lookup_bulk answers from the host table image
(CNE_FIB_LOOKUP_DEFAULT, as cne_fib.c:86 binds it) or, with
lookup=CNE_FIB_LOOKUP_GPU, from the HBM mirror; batch classify always reads
the mirror.

    Fib(name, type=CNE_FIB_DIR24_8, default_nh, max_routes, nh_sz, num_tbl8,
        lookup=None)    lookup: a cne_fib_lookup_type passed to select_lookup
        .add(ip, depth, nh) -> int        cne_fib_add      (cne_fib.h:129)
        .delete(ip, depth) -> int         cne_fib_delete   (cne_fib.h:143)
        .lookup_bulk(ips) -> ndarray u64  cne_fib_lookup_bulk (cne_fib.h:162)
        .lookup_dev(ips_t, out_t, stream) device tensors (extension)
    Fib6(...) likewise for IPv6 (cne_fib6.h:41-138).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native as N


def _conf(type_, default_nh, max_routes, nh_sz, num_tbl8):
    c = N.FibConf()
    c.type = type_
    c.default_nh = default_nh
    c.max_routes = max_routes
    c.dir24_8.nh_sz = nh_sz
    c.dir24_8.num_tbl8 = num_tbl8
    return c


class Fib:
    """IPv4 FIB (DIR-24-8 or DUMMY)."""

    def __init__(self, name="fib", type=N.CNE_FIB_DIR24_8, default_nh=0, max_routes=1024,
                 nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256, lookup=None):
        self._L = N.lib()
        conf = _conf(type, default_nh, max_routes, nh_sz, num_tbl8)
        self.h = self._L.cne_fib_create(name.encode() if name is not None else None,
                                        ctypes.byref(conf))
        if not self.h:
            raise ValueError("cne_fib_create rejected the configuration")
        self.type = type
        self.default_nh = default_nh
        if lookup is not None:
            N.check(self.select_lookup(lookup), "cne_fib_select_lookup")

    @staticmethod
    def create_raw(name, conf: "N.FibConf"):
        """cne_fib_create with arbitrary arguments; returns the handle (or None)."""
        return N.lib().cne_fib_create(name, ctypes.byref(conf) if conf is not None else None)

    def close(self):
        if self.h:
            self._L.cne_fib_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, ip: int, depth: int, nh: int) -> int:
        return self._L.cne_fib_add(self.h, ip & 0xFFFFFFFF, depth, nh)

    def delete(self, ip: int, depth: int) -> int:
        return self._L.cne_fib_delete(self.h, ip & 0xFFFFFFFF, depth)

    def lookup_bulk(self, ips) -> np.ndarray:
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        out = np.zeros(len(ips), dtype=np.uint64)
        N.check(self._L.cne_fib_lookup_bulk(self.h, ips.ctypes.data, out.ctypes.data, len(ips)),
                "cne_fib_lookup_bulk")
        return out

    def lookup_dev(self, ips_ptr: int, out_ptr: int, n: int, stream: int = 0) -> None:
        N.check(self._L.cndp_fib_lookup_dev(self.h, ips_ptr, out_ptr, n, stream or None),
                "cndp_fib_lookup_dev")

    def select_lookup(self, t: int) -> int:
        return self._L.cne_fib_select_lookup(self.h, t)

    def sync(self, stream: int = 0) -> None:
        N.check(self._L.cndp_fib_sync(self.h, stream or None), "cndp_fib_sync")

    def image(self):
        """(tbl24, tbl8) numpy views of the host table image."""
        im = N.FibImage()
        N.check(self._L.cndp_fib_image(self.h, ctypes.byref(im)), "cndp_fib_image")
        dt = {0: np.uint8, 1: np.uint16, 2: np.uint32, 3: np.uint64}[im.nh_sz]
        esz = 1 << im.nh_sz
        t24 = np.ctypeslib.as_array((ctypes.c_uint8 * ((1 << 24) * esz)).from_address(im.tbl24))
        t8 = np.ctypeslib.as_array((ctypes.c_uint8 * (im.tbl8_groups * 256 * esz)).from_address(im.tbl8))
        return t24.view(dt), t8.view(dt)

    def stats(self):
        r, u, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(self._L.cndp_fib_stats(self.h, ctypes.byref(r), ctypes.byref(u), ctypes.byref(s)),
                "cndp_fib_stats")
        return {"routes": r.value, "tbl8_used": u.value, "rsvd_tbl8s": s.value}


class Fib6:
    """IPv6 FIB (trie or DUMMY)."""

    def __init__(self, name="fib6", type=N.CNE_FIB_TRIE, default_nh=0, max_routes=1024,
                 nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15, lookup=None):
        self._L = N.lib()
        conf = _conf(type, default_nh, max_routes, nh_sz, num_tbl8)
        self.h = self._L.cne_fib6_create(name.encode() if name is not None else None,
                                         ctypes.byref(conf))
        if not self.h:
            raise ValueError("cne_fib6_create rejected the configuration")
        self.type = type
        self.default_nh = default_nh
        if lookup is not None:
            N.check(self.select_lookup(lookup), "cne_fib6_select_lookup")

    @staticmethod
    def create_raw(name, conf):
        return N.lib().cne_fib6_create(name, ctypes.byref(conf) if conf is not None else None)

    def close(self):
        if self.h:
            self._L.cne_fib6_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _ip(ip) -> bytes:
        if isinstance(ip, int):
            return ip.to_bytes(16, "big")
        b = bytes(ip)
        assert len(b) == 16
        return b

    def add(self, ip, depth: int, nh: int) -> int:
        return self._L.cne_fib6_add(self.h, self._ip(ip), depth, nh)

    def delete(self, ip, depth: int) -> int:
        return self._L.cne_fib6_delete(self.h, self._ip(ip), depth)

    def lookup_bulk(self, ips) -> np.ndarray:
        ips = np.ascontiguousarray(ips, dtype=np.uint8).reshape(-1, 16)
        out = np.zeros(len(ips), dtype=np.uint64)
        N.check(self._L.cne_fib6_lookup_bulk(self.h, ips.ctypes.data, out.ctypes.data, len(ips)),
                "cne_fib6_lookup_bulk")
        return out

    def lookup_dev(self, ips_ptr: int, out_ptr: int, n: int, stream: int = 0) -> None:
        N.check(self._L.cndp_fib6_lookup_dev(self.h, ips_ptr, out_ptr, n, stream or None),
                "cndp_fib6_lookup_dev")

    def select_lookup(self, t: int) -> int:
        return self._L.cne_fib6_select_lookup(self.h, t)

    def sync(self, stream: int = 0) -> None:
        N.check(self._L.cndp_fib6_sync(self.h, stream or None), "cndp_fib6_sync")

    def image(self):
        im = N.FibImage()
        N.check(self._L.cndp_fib6_image(self.h, ctypes.byref(im)), "cndp_fib6_image")
        dt = {1: np.uint16, 2: np.uint32, 3: np.uint64}[im.nh_sz]
        esz = 1 << im.nh_sz
        t24 = np.ctypeslib.as_array((ctypes.c_uint8 * ((1 << 24) * esz)).from_address(im.tbl24))
        t8 = np.ctypeslib.as_array((ctypes.c_uint8 * (im.tbl8_groups * 256 * esz)).from_address(im.tbl8))
        return t24.view(dt), t8.view(dt)

    def stats(self):
        r, u, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        N.check(self._L.cndp_fib6_stats(self.h, ctypes.byref(r), ctypes.byref(u), ctypes.byref(s)),
                "cndp_fib6_stats")
        return {"routes": r.value, "tbl8_used": u.value, "rsvd_tbl8s": s.value}


class NodeFib(Fib):
    """The l3fwd node FIB libcndp_gpu owns (ip4_lookup_nm, ip4_lookup.c:31-42),
    created by cndp_node_ip4_lookup_init (setup_fib, :292-311).  Routes go in
    through cne_node_ip4_route_add; this handle does not own the table."""

    def __init__(self):  # noqa: super().__init__ would create a second FIB
        self._L = N.lib()
        N.check(self._L.cndp_node_ip4_lookup_init(), "cndp_node_ip4_lookup_init")
        self.h = self._L.cndp_node_ip4_lookup_fib()
        self.type = N.CNE_FIB_DIR24_8
        self.default_nh = N.IP4_LOOKUP_NEXT_PKT_DROP << 16

    def close(self):
        self.h = None  # the library keeps the table (cndp_node_ip4_lookup_fini frees it)

    @staticmethod
    def fini():
        N.lib().cndp_node_ip4_lookup_fini()

    def route_add(self, ip: int, depth: int, next_hop: int, next_node: int) -> int:
        return N.lib().cne_node_ip4_route_add(ip & 0xFFFFFFFF, depth, next_hop, next_node)


def cne_node_ip4_route_add(ip: int, depth: int, next_hop: int, next_node: int) -> int:
    """The exported cne_node_ip4_route_add (ip4_lookup.c:259-289) on the node FIB."""
    return N.lib().cne_node_ip4_route_add(ip & 0xFFFFFFFF, depth, next_hop, next_node)


def node_ip4_route_add(fib: Fib, ip: int, depth: int, next_hop: int, next_node: int) -> int:
    """cne_node_ip4_route_add's arithmetic (ip4_lookup.c:272) applied to any FIB
    handle: val = (next_node << 16 | nh) & 0xFFFFFF.  For the node FIB itself use
    cne_node_ip4_route_add (the C export)."""
    val = ((next_node << 16) | next_hop) & ((1 << 24) - 1)
    return fib.add(ip, depth, val)


def node_ip4_add_input(fib: Fib, ip: int, depth: int, hop: int) -> int:
    """cne_node_ip4_add_input (lib/cnet/ipv4/ip4_input.c:263-272), the C export:
    nh = hop | (depth == 32 ? PROTO : FORWARD) << 24."""
    return N.lib().cne_node_ip4_add_input(fib.h, ip & 0xFFFFFFFF, depth, hop)


def node_ip6_add_input(fib6: Fib6, ip, depth: int, hop: int) -> int:
    """cne_node_ip6_add_input (lib/cnet/ipv6/ip6_input.c:263-274), the C export,
    including its `depth == 32` test (not 128) for the PROTO edge."""
    return N.lib().cne_node_ip6_add_input(fib6.h, Fib6._ip(ip), depth, hop)
