"""Shared setup for the parity tests: product FIBs (libcndp_gpu.so), oracle
tables (oracle/liboracle.so, independent painter), and output comparison."""
from __future__ import annotations

import numpy as np

from cndp_amd import native as N
from cndp_amd import pktgen
from oracle import oracle as O

L3FWD_DEF = N.IP4_LOOKUP_NEXT_PKT_DROP << 16
CNET_NR = 1024
CNET_DEF = (0 << 24) | (CNET_NR + 1)


def l3fwd_fib(routes=None):
    from cndp_amd.fib import Fib, node_ip4_route_add
    routes = routes if routes is not None else pktgen.l3fwd_routes()
    fib = Fib("rt4", N.CNE_FIB_DIR24_8, default_nh=L3FWD_DEF, max_routes=1024,
              nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
    for ip, d, nh in routes:
        assert node_ip4_route_add(fib, ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE) == 0
    vals = [(ip, d, (N.IP4_LOOKUP_NEXT_REWRITE << 16) | nh) for ip, d, nh in routes]
    return fib, vals


def l3fwd_oracle_tables(vals):
    return O.dir24_8_build(vals, L3FWD_DEF, 256)


def cnet_fibs():
    from cndp_amd.fib import Fib, Fib6, node_ip4_add_input, node_ip6_add_input
    routes = pktgen.l3fwd_routes()
    fib = Fib("rt4-fib", N.CNE_FIB_DIR24_8, default_nh=CNET_DEF, max_routes=CNET_NR,
              nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
    v4vals = []
    for i, (ip, d, _) in enumerate(routes):
        assert node_ip4_add_input(fib, ip, d, i) == 0
        v4vals.append((ip, d, i | ((2 if d == 32 else 1) << 24)))
    v6 = pktgen.v6_routes()
    fib6 = Fib6("rt6-fib", N.CNE_FIB_TRIE, default_nh=CNET_DEF, max_routes=CNET_NR,
                nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15)
    v6vals = []
    for ip, d, i in v6:
        assert node_ip6_add_input(fib6, ip, d, i) == 0
        v6vals.append((ip, d, i | ((2 if d == 32 else 1) << 24)))
    return fib, fib6, routes, v6, v4vals, v6vals


def oracle_classify(mode, frames, tables4=None, tables6=None, n_bins=64, reta=None, key=None,
                    buf_len=1984, spec_burst=None, spec_state=None):
    """The oracle over a Frames batch.  cnet mode models the ptype node's
    speculation over 256-packet bursts from state 0 (the library default
    after a reset) unless spec_burst says otherwise."""
    slab = frames.slab.cpu().numpy()
    offs = frames.offsets.cpu().numpy().astype(np.uint64) if frames.offsets is not None else None
    if spec_burst is None:
        spec_burst = 256 if mode == O.MODE_CNET else 0
    return O.classify(mode, slab, frames.n, stride=frames.stride, offsets=offs, data_off=frames.data_off,
                      tables4=tables4, tables6=tables6, n_bins=n_bins, reta=reta, key=key,
                      buf_len=buf_len, spec_burst=spec_burst, spec_state=spec_state)


DT = {"nh": np.uint32, "hash": np.uint32, "queue": np.uint16, "edge": np.uint8, "bins": np.uint64,
      "ptype": np.uint32, "rxmeta": np.uint32}


def assert_same(got: dict, ref: dict, keys=("nh", "hash", "queue", "edge", "bins")):
    for k in keys:
        g = got[k]
        if hasattr(g, "cpu"):
            g = g.cpu().numpy()
        g = g.view(DT[k]) if g.dtype.itemsize == np.dtype(DT[k]).itemsize else g.astype(DT[k])
        r = ref[k]
        if not np.array_equal(g, r):
            bad = np.nonzero(g != r)[0]
            i = int(bad[0])
            raise AssertionError(f"{k}: {len(bad)} mismatches, first at {i}: got {g[i]:#x} want {r[i]:#x}")


# ---- cne_get_ptype known answers from the reference's own tables ----------
# tests/golden/ptype_ref.json (tools/gen_ptype_golden.py) holds the CNE_PTYPE_*
# values, the ptype node's p_nxt table and cne_get_ptype's lookup tables,
# evaluated from the reference source text.  ptype_kat() builds one frame per
# table input, with the field of the packet type that input decides and the
# value the reference tables give it.
def ptype_ref():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ptype_ref.json")) as f:
        return json.load(f)


def ptype_kat(slot: int = 128):
    """[(frame bytes, field mask, expected field value, what)]"""
    ref = ptype_ref()
    C, T = ref["ptype_consts"], ref["get_ptype_tables"]
    eth = bytes(6) + bytes([2, 0, 0, 0, 0, 1])
    out = []

    def ip4(vihl=0x45, proto=17, frag=0):
        h = bytearray(20)
        h[0], h[2], h[3], h[8], h[9] = vihl, 0, 60, 64, proto
        h[6], h[7] = frag >> 8, frag & 0xFF
        h[12:16], h[16:20] = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
        return bytes(h)

    def pad(b):
        return (b + bytes(slot))[:slot]

    # IPv4 version / IHL byte -> the L3 field (pktmbuf_ptype.c:297-309)
    for v in range(256):
        f = eth + b"\x08\x00" + ip4(vihl=v) + bytes(8)
        out.append((pad(f), C["CNE_PTYPE_L3_MASK"], T["l3_ip_by_ihl"].get(str(v), 0), f"ipv4 vihl {v:#x}"))
    # IPv4 protocol -> the L4 field (:313-322)
    for p in range(256):
        f = eth + b"\x08\x00" + ip4(proto=p) + bytes(40)
        out.append((pad(f), C["CNE_PTYPE_L4_MASK"], T["l4_by_proto"].get(str(p), 0), f"ipv4 proto {p}"))
    # IPv4 fragment -> L4_FRAG whatever the protocol (:556-560)
    for fo in (0x2000, 0x0001, 0x1FFF, 0x4000):
        f = eth + b"\x08\x00" + ip4(proto=6, frag=fo) + bytes(40)
        want = C["CNE_PTYPE_L4_FRAG"] if fo & 0x3FFF else C["CNE_PTYPE_L4_TCP"]
        out.append((pad(f), C["CNE_PTYPE_L4_MASK"], want, f"ipv4 frag {fo:#x}"))
    # IPv6 next header -> the L3 field (:279-293)
    for n in range(256):
        h = bytearray(40)
        h[0], h[6], h[7] = 0x60, n, 64
        f = eth + b"\x86\xdd" + bytes(h) + bytes(48)
        want = C["CNE_PTYPE_L3_IPV6"] + T["ip6_ext_by_proto"].get(str(n), 0)
        out.append((pad(f), C["CNE_PTYPE_L3_MASK"], want, f"ipv6 nh {n}"))
    # GRE flags -> option length: the inner IPv4 header sits after it (:372-395)
    for fl in range(16):
        olen = T["gre_opt_len"].get(str(fl), 0)
        gre = bytes([fl << 4, 0, 0x08, 0x00]) + bytes(max(olen, 4) - 4)
        f = eth + b"\x08\x00" + ip4(proto=47) + gre + ip4(proto=17) + bytes(8)
        want = (C["CNE_PTYPE_TUNNEL_GRE"] | C["CNE_PTYPE_INNER_L3_IPV4"]) if olen else 0
        mask = C["CNE_PTYPE_TUNNEL_MASK"] | C["CNE_PTYPE_INNER_L3_MASK"]
        out.append((pad(f), mask, want, f"gre flags {fl:#x}"))
    # L2: ARP, VLAN, QinQ (:486-540)
    out.append((pad(eth + b"\x08\x06" + bytes(28)), 0xFFFFFFFF, C["CNE_PTYPE_L2_ETHER_ARP"], "arp"))
    f = eth + b"\x81\x00\x00\x05\x08\x00" + ip4() + bytes(8)
    out.append((pad(f), C["CNE_PTYPE_L2_MASK"] | C["CNE_PTYPE_L3_MASK"],
                C["CNE_PTYPE_L2_ETHER_VLAN"] | C["CNE_PTYPE_L3_IPV4"], "vlan"))
    f = eth + b"\x88\xa8\x00\x05\x81\x00\x00\x06\x08\x00" + ip4() + bytes(8)
    out.append((pad(f), C["CNE_PTYPE_L2_MASK"] | C["CNE_PTYPE_L3_MASK"],
                C["CNE_PTYPE_L2_ETHER_QINQ"] | C["CNE_PTYPE_L3_IPV4"], "qinq"))
    # UDP destination port -> GTP-U / GTP-C (:580-588)
    for port, name in ((2152, "CNE_PTYPE_TUNNEL_GTPU"), (2123, "CNE_PTYPE_TUNNEL_GTPC"), (2153, None)):
        f = eth + b"\x08\x00" + ip4() + bytes([0x30, 0x39, port >> 8, port & 0xFF, 0, 8, 0, 0])
        out.append((pad(f), C["CNE_PTYPE_TUNNEL_MASK"], C[name] if name else 0, f"udp dport {port}"))
    return out
