"""Pin the oracle (CPU restatement) against the reference's own outputs:
the committed golden fixtures (tests/golden/, made by tools/gen_golden.py
from the reference's cne_softrss / cne_ipv4_cksum / lpm6_data_test.h) and
the public Microsoft RSS KAT.  Also the reference fib_test.c / fib6_test.c
LPM ladders against the oracle's table painter.  CPU only."""
import json
import os
import socket
import struct

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kat():
    with open(os.path.join(GOLD, "rss_kat.json")) as f:
        return json.load(f)


def test_rss_kat_ipv4():
    k = _kat()
    key = bytes.fromhex(k["key"])
    for d, dp, s, sp, l3, l4 in k["ipv4"]:
        t = [struct.unpack(">I", socket.inet_aton(s))[0], struct.unpack(">I", socket.inet_aton(d))[0],
             (sp << 16) | dp]
        assert O.softrss(t[:2], key) == l3
        assert O.softrss(t, key) == l4


def test_rss_kat_ipv6():
    k = _kat()
    key = bytes.fromhex(k["key"])
    for d, dp, s, sp, l3, l4 in k["ipv6"]:
        sa, da = socket.inet_pton(socket.AF_INET6, s), socket.inet_pton(socket.AF_INET6, d)
        t = list(struct.unpack(">4I", sa)) + list(struct.unpack(">4I", da)) + [(sp << 16) | dp]
        assert O.softrss(t[:8], key) == l3
        assert O.softrss(t, key) == l4


def test_softrss_matches_reference_vectors():
    g = np.load(os.path.join(GOLD, "thash_ref.npz"))
    L = O.lib()
    for i in range(len(g["lens"])):
        t = np.ascontiguousarray(g["tuples"][i])
        key = np.ascontiguousarray(g["keys"][g["kidx"][i]])
        assert L.orc_softrss(t.ctypes.data, int(g["lens"][i]), key.ctypes.data) == g["expected"][i]
        kc = np.ascontiguousarray(g["keys_converted"][g["kidx"][i]])
        assert L.orc_softrss_be(t.ctypes.data, int(g["lens"][i]), kc.ctypes.data) == g["expected_be"][i]


def test_convert_key_matches_reference():
    g = np.load(os.path.join(GOLD, "thash_ref.npz"))
    for k in range(len(g["keys"])):
        src = np.ascontiguousarray(g["keys"][k])
        dst = np.zeros(40, np.uint8)
        O.lib().orc_convert_rss_key(src.ctypes.data, dst.ctypes.data, 40)
        assert np.array_equal(dst, g["keys_converted"][k])


def test_v6_tuple_loading_matches_reference():
    g = np.load(os.path.join(GOLD, "thash_ref.npz"))
    for h, exp in zip(g["v6_hdr"], g["v6_loaded"]):
        got = [int.from_bytes(bytes(h[8 + 4 * k: 12 + 4 * k]), "big") for k in range(8)]
        assert got == [int(x) for x in exp]


def test_ipv4_cksum_matches_reference():
    g = np.load(os.path.join(GOLD, "cksum_ref.npz"))
    for h, exp in zip(g["hdrs"], g["expected"]):
        assert O.ipv4_cksum(bytes(h)) == exp


def _ladder4(lookup, add, delete, def_nh=100):
    """test/testcne/fib_test.c:239-288 check_fib, expressed against callables."""
    ip_add = 128 << 24
    ip_arr = [(ip_add + (1 << i) - 1) & 0xFFFFFFFF for i in range(32)]
    missing = (127 << 24) | 0xFFFFFF

    def asc(n):
        got = lookup(ip_arr + [missing])
        exp = [n] * (32 - n + 1) + [n - 1 - k for k in range(n - 1)] + [def_nh]
        assert list(got) == exp, (n, list(got))

    def desc(n):
        got = lookup(ip_arr + [missing])
        exp = [32 - i for i in range(n)] + [def_nh] * (32 - n) + [def_nh]
        assert list(got) == exp, (n, list(got))

    desc(0)
    for i in range(1, 33):
        assert add(ip_add, i, i) == 0
        asc(i)
    for i in range(32, 1, -1):
        assert delete(ip_add, i) == 0
        asc(i - 1)
    assert delete(ip_add, 1) == 0
    desc(0)
    for i in range(32):
        assert add(ip_add, 32 - i, 32 - i) == 0
        desc(i + 1)
    for i in range(1, 33):
        assert delete(ip_add, i) == 0
        desc(32 - i)


def test_ladder4_oracle_painter():
    routes = {}

    def add(ip, d, nh):
        routes[(ip & (0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF, d)] = nh
        return 0

    def delete(ip, d):
        routes.pop((ip & (0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF, d))
        return 0

    def lookup(ips):
        rl = [(ip, d, nh) for (ip, d), nh in routes.items()]
        t24, t8 = O.dir24_8_build(rl, 100, 64)
        a = O.dir24_8_lookup(t24, t8, ips)
        b = O.lpm4_bruteforce(rl, 100, ips)
        assert np.array_equal(a, b)
        return a

    _ladder4(lookup, add, delete)


def test_lpm6_1000_rules_oracle():
    g = np.load(os.path.join(GOLD, "lpm6_1000.npz"))
    routes = [(bytes(ip), int(d), int(nh)) for ip, d, nh in zip(g["rule_ip"], g["rule_depth"], g["rule_nh"])]
    t24, t8 = O.trie_build(routes, 0, 1 << 16)
    got = O.trie_lookup(t24, t8, g["ip"])
    assert np.array_equal(got, g["nh"].astype(np.uint64))
    bf = O.lpm6_bruteforce(routes, 0, g["ip"][:2000])
    assert np.array_equal(bf, g["nh"][:2000].astype(np.uint64))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_dir24_8_painter_vs_bruteforce(seed):
    rng = np.random.default_rng(seed)
    routes = []
    for _ in range(300):
        d = int(rng.integers(0, 33))
        ip = int(rng.integers(0, 2**32)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF if d else 0)
        routes.append((ip, d, int(rng.integers(0, 2**31 - 1))))
    # concentrate some addresses inside the prefixes
    ips = rng.integers(0, 2**32, size=4096, dtype=np.uint64).astype(np.uint32)
    for i in range(0, 4096, 2):
        ip, d, _ = routes[i % len(routes)]
        ips[i] = (ip | (int(ips[i]) & ((1 << (32 - d)) - 1))) & 0xFFFFFFFF
    t24, t8 = O.dir24_8_build(routes, 7, 1024)
    assert np.array_equal(O.dir24_8_lookup(t24, t8, ips), O.lpm4_bruteforce(routes, 7, ips))


def test_trie_painter_vs_bruteforce():
    rng = np.random.default_rng(9)
    routes = []
    for _ in range(200):
        d = int(rng.integers(0, 129))
        ip = int.from_bytes(rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), "big")
        ip &= ((1 << 128) - 1) ^ ((1 << (128 - d)) - 1)
        routes.append((ip.to_bytes(16, "big"), d, int(rng.integers(0, 2**31 - 1))))
    ips = rng.integers(0, 256, size=(2048, 16), dtype=np.uint8)
    for i in range(0, 2048, 2):
        ip, d, _ = routes[i % len(routes)]
        v = int.from_bytes(ip, "big") | (int.from_bytes(ips[i].tobytes(), "big") & ((1 << (128 - d)) - 1))
        ips[i] = np.frombuffer(v.to_bytes(16, "big"), np.uint8)
    t24, t8 = O.trie_build(routes, 3, 1 << 14)
    assert np.array_equal(O.trie_lookup(t24, t8, ips), O.lpm6_bruteforce(routes, 3, ips))


def test_oracle_ip4_rewrite_known_answers():
    """ip4_rewrite restatement: TTL 64 -> 63 and checksum + 0x0100 (what the
    reference chain produced when run), the header still
    verifies, and the 4-wide / tail checksum rules at 0xFFFE / 0xFFFF."""
    import numpy as np
    from cndp_amd import pktgen
    fr = pktgen.packed_ipv4(8, routes=pktgen.l3fwd_routes())
    slab = fr.slab.numpy().copy()
    tbl = np.zeros(64, O.REWRITE_NH)
    tbl[:]["rewrite_len"] = 12
    tbl[:]["tx_node"] = 3
    nh = np.zeros(8, np.uint32)          # all to ip4_rewrite, next hop 0
    before = slab.reshape(8, 64).copy()
    tx = O.ip4_rewrite(slab, 8, nh, tbl, burst=8)
    after = slab.reshape(8, 64)
    assert (tx == 3).all()
    assert (before[:, 22] == 64).all() and (after[:, 22] == 63).all()
    ck0 = before[:, 24].astype(int) << 8 | before[:, 25]
    ck1 = after[:, 24].astype(int) << 8 | after[:, 25]
    assert ((ck0 + 0x100) & 0xFFFF == ck1).all()
    for r in after:
        assert O.ipv4_cksum(bytes(r[14:34])) == 0   # still a valid header
    # quirk table: raw little-endian checksum word -> result, per loop
    cases = {0xFFFE: (0xFFFF, 0x0000), 0xFFFF: (0x0001, 0x0000), 0x1234: (0x1235, 0x1235)}
    for raw, (vec, tail) in cases.items():
        s = np.zeros(64 * 5, np.uint8)
        s[24::64] = raw & 0xFF
        s[25::64] = raw >> 8
        O.ip4_rewrite(s, 5, np.zeros(5, np.uint32), tbl, burst=5)   # 4 in the 4-wide loop, 1 tail
        w = s[24::64].astype(int) | (s[25::64].astype(int) << 8)
        assert list(w) == [vec] * 4 + [tail], (hex(raw), [hex(x) for x in w])


def test_oracle_mac_swap():
    import numpy as np
    s = np.arange(128, dtype=np.uint8)
    O.mac_swap(s, 2, stride=64)
    assert list(s[:12]) == [6, 7, 8, 9, 10, 11, 0, 1, 2, 3, 4, 5]
    assert list(s[64:76]) == [70, 71, 72, 73, 74, 75, 64, 65, 66, 67, 68, 69]


def test_oracle_rxmeta_known_answers():
    """eth_rx mbuf_update fields for hand-built frames (eth_rx.c:35-63)."""
    import numpy as np
    def frame(et, ip=b"", dst=b"\x02" * 6):
        f = dst + b"\x02" * 6 + et.to_bytes(2, "big") + ip
        return np.frombuffer(f + bytes(128 - len(f)), np.uint8)
    v4 = bytes([0x45, 0, 0, 40, 0, 0, 0, 0, 64, 6]) + bytes(10)          # TCP
    tcp = bytes(12) + bytes([0x80]) + bytes(7)                         # data offset 8 words -> 32 B
    v6 = bytes([0x60, 0, 0, 0, 0, 8, 17, 64]) + bytes(32)                 # UDP
    frames = [frame(0x0800, v4 + tcp), frame(0x86DD, v6), frame(0x0806, dst=b"\xff" * 6),
              frame(0x0800, v4 + tcp, dst=b"\x01\x00\x5e\x00\x00\x01")]
    slab = np.concatenate(frames)
    r = O.classify(O.MODE_CNET, slab, 4, stride=128, tables4=O.dir24_8_build([], 0, 16),
                   tables6=O.trie_build([], 0, 16))
    m = r["rxmeta"]
    l2, l3, l4 = m & 0x7F, (m >> 7) & 0x1FF, (m >> 16) & 0xFF
    assert list(l2) == [14, 14, 14, 14]
    assert list(l3[:2]) == [20, 40] and l3[2] == 0
    assert list(l4) == [32, 8, 0, 32]
    assert [(x >> 29) & 7 for x in m] == [0, 4, 2, 1]      # IPv6, BCAST, MCAST bits
    assert list(r["ptype"][:3]) == [0x111, 0x241, 0x3]


def test_prefetching_bulk_lookup_matches():
    """dir24_8.h:118-148 restated with its prefetch schedule (the CPU
    baseline's lookup) == the plain lookup, for every n around the 15-ahead
    prefetch distance."""
    from cndp_amd import pktgen
    vals = [(ip, d, nh) for ip, d, nh in pktgen.l3fwd_routes()]
    t24, t8 = O.dir24_8_build(vals, 1 << 16, 256)
    rng = np.random.default_rng(4)
    for n in (0, 1, 4, 14, 15, 16, 31, 1000):
        ips = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        ips[::2] = (10 << 24) | (ips[::2] & 0x0004FFFF)
        assert np.array_equal(O.dir24_8_lookup_bulk_pf(t24, t8, ips), O.dir24_8_lookup(t24, t8, ips))


def test_burst_bench_runs_both_chains():
    """The CPU baselines (l3fwd node loop, cnet chain) run pinned on 2 threads."""
    from cndp_amd import pktgen
    import os as _os
    vals = [(ip, d, nh) for ip, d, nh in pktgen.l3fwd_routes()]
    t4 = O.dir24_8_build(vals, 1 << 16, 256)
    fr = pktgen.packed_ipv4(4096, routes=pktgen.l3fwd_routes())
    slab = fr.slab.numpy()
    cpus = sorted(_os.sched_getaffinity(0))[:2]
    assert O.burst_bench(O.MODE_L3FWD, slab, 4096, nthreads=len(cpus), cpus=cpus, stride=64, tables4=t4) > 0
    v6 = pktgen.v6_routes()
    t6 = O.trie_build([(ip, d, i | (1 << 24)) for ip, d, i in v6], 1025, 1 << 15)
    im = pktgen.imix(4096, v4routes=pktgen.l3fwd_routes(), v6routes=v6)
    t = O.burst_bench(O.MODE_CNET, im.slab.numpy(), 4096, nthreads=len(cpus), cpus=cpus,
                      offsets=im.offsets.numpy().astype(np.uint64), tables4=t4, tables6=t6)
    assert t > 0


def test_ptype_node_table_matches_reference():
    """The oracle's ptype-node edge, p_nxt[ptype & _PTYPE_MASK], against the
    table evaluated from lib/cnet/ptype/ptype.c:20-46 (tests/golden/ptype_ref.json)."""
    from helpers import ptype_ref
    ref = ptype_ref()
    assert ref["pnxt_mask"] == 0xFFFF
    want = {int(k, 16): v for k, v in ref["pnxt"].items()}
    rng = np.random.default_rng(3)
    high = rng.integers(0, 1 << 16, 64, dtype=np.uint64) << np.uint64(16)
    for pt in range(1 << 16):
        assert O.cnet_ptype_edge(pt) == want.get(pt, 0), hex(pt)
    for h in high.tolist():  # bits above the mask do not matter
        for pt in want:
            assert O.cnet_ptype_edge(pt | int(h)) == want[pt]


def test_get_ptype_tables_match_reference():
    """cne_get_ptype's lookup tables (IPv4 IHL, L4 protocol, IPv6 extension
    headers, GRE option lengths) and the L2 / GTP encodings, one frame per
    table input, against the values evaluated from pktmbuf_ptype.c / .h."""
    from helpers import ptype_kat
    bad = []
    for frame, mask, want, what in ptype_kat():
        pt, _ = O.get_ptype(frame)
        if (pt & mask) != want:
            bad.append((what, hex(pt), hex(want)))
    assert not bad, bad[:8]


def test_eth_rx_fields_match_reference_layout():
    """What eth_rx's mbuf_update writes (eth_rx.c:35-63), as the mbuf shim and
    the node queue store it (tx_offload = rxmeta & 0xFFFFFF, ol_flags = rxmeta
    >> 29 << 61): decoded with the reference's tx_offload bit-field layout and
    CNE_MBUF_TYPE_* bits (tests/golden/ptype_ref.json from pktmbuf_offload.h),
    the l2/l3/l4 lengths are cne_get_ptype's and the type bits follow the
    destination MAC and ethertype."""
    from helpers import CNET_DEF, cnet_fibs, ptype_kat, ptype_ref
    ref = ptype_ref()
    L, F = ref["tx_offload_layout"], ref["ol_flags_type"]
    frames = [k[0] for k in ptype_kat()]
    # destination MACs: unicast, broadcast, multicast, on IPv4 and IPv6 frames
    extra = []
    for f in frames[:3] + frames[512 + 4:512 + 7]:
        for dst in (bytes([0, 1, 2, 3, 4, 5]), b"\xff" * 6, bytes([1, 0, 0x5e, 0, 0, 1])):
            extra.append(dst + f[6:])
    frames = frames + extra
    n = len(frames)
    slab = np.frombuffer(b"".join(frames), np.uint8).copy()
    fib, fib6, routes, v6, v4vals, v6vals = cnet_fibs()
    t4 = O.dir24_8_build(v4vals, CNET_DEF, 256)
    t6 = O.trie_build(v6vals, CNET_DEF, 1 << 15)
    out = O.classify(O.MODE_CNET, slab, n, stride=128, tables4=t4, tables6=t6, spec_burst=0)
    rm = out["rxmeta"].astype(np.uint64)
    txo = rm & np.uint64(0xFFFFFF)
    olf = (rm >> np.uint64(29)) << np.uint64(61)

    def field(v, name):
        return (int(v) >> L[f"CNE_MBUF_{name}_LEN_OFS"]) & ((1 << L[f"CNE_MBUF_{name}_LEN_BITS"]) - 1)

    for i, f in enumerate(frames):
        _, hl = O.get_ptype(f)
        assert (field(txo[i], "L2"), field(txo[i], "L3"), field(txo[i], "L4")) == \
            (hl.l2_len & 0x7F, hl.l3_len & 0x1FF, hl.l4_len & 0xFF), i
        want = F["CNE_MBUF_TYPE_IPv6"] if f[12:14] == b"\x86\xdd" else 0
        if f[:6] == b"\xff" * 6:
            want |= F["CNE_MBUF_TYPE_BCAST"]
        elif f[0] & 1:
            want |= F["CNE_MBUF_TYPE_MCAST"]
        assert int(olf[i]) == want, (i, hex(int(olf[i])), hex(want))
