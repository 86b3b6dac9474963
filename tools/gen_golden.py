#!/usr/bin/env python3
"""Regenerate tests/golden/* from the REFERENCE's own code (run in the survey
container, where /root/reference exists and `make -C oracle` has built
oracle/_ref/).  The fixtures are data only: inputs plus the outputs the
reference's cne_softrss / cne_softrss_be / cne_thash_load_v6_addrs /
cne_ipv4_cksum and its lpm6_data_test.h get_next_hop produced for them.

    python tools/gen_golden.py
"""
from __future__ import annotations

import ctypes
import json
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
MS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")

# Microsoft RSS verification suite (public); every value below was also
# reproduced by the reference's cne_softrss before being written here.
KAT_V4 = [("161.142.100.80", 1766, "66.9.149.187", 2794, 0x323E8FC2, 0x51CCC178),
          ("65.69.140.83", 4739, "199.92.111.2", 14230, 0xD718262A, 0xC626B0EA),
          ("12.22.207.184", 38024, "24.19.198.95", 12898, 0xD2D0A5DE, 0x5C2B394A),
          ("209.142.163.6", 2217, "38.27.205.30", 48228, 0x82989176, 0xAFC7327F),
          ("202.188.127.2", 1303, "153.39.163.191", 44251, 0x5D1809C5, 0x10E828A2)]
KAT_V6 = [("3ffe:2501:200:3::1", 1766, "3ffe:2501:200:1fff::7", 2794, 0x2CC18CD5, 0x40207D3D),
          ("ff02::1", 4739, "3ffe:501:8::260:97ff:fe40:efab", 14230, 0x0F0C461C, 0xDDE51BBF),
          ("fe80::200:f8ff:fe21:67cf", 38024, "3ffe:1900:4545:3:200:f8ff:fe21:67cf", 44251,
           0x4B61E985, 0x02D1FEEF)]


def main():
    R = O.ref()
    if R is None:
        sys.exit("oracle/_ref/libcndp_ref.so missing: run `make -C oracle` where /root/reference exists")
    os.makedirs(GOLD, exist_ok=True)
    rng = np.random.default_rng(0x43444E50)

    # --- KAT, cross-checked against the reference --------------------------
    import socket
    for d, dp, s, sp, l3, l4 in KAT_V4:
        t = (ctypes.c_uint32 * 3)(struct.unpack(">I", socket.inet_aton(s))[0],
                                  struct.unpack(">I", socket.inet_aton(d))[0], (sp << 16) | dp)
        assert R.ref_softrss(t, 2, MS_KEY) == l3 and R.ref_softrss(t, 3, MS_KEY) == l4
    for d, dp, s, sp, l3, l4 in KAT_V6:
        hdr = bytearray(40)
        hdr[8:24] = socket.inet_pton(socket.AF_INET6, s)
        hdr[24:40] = socket.inet_pton(socket.AF_INET6, d)
        out = (ctypes.c_uint32 * 8)()
        R.ref_thash_load_v6(bytes(hdr), out)
        t = (ctypes.c_uint32 * 9)(*list(out), (sp << 16) | dp)
        assert R.ref_softrss(t, 8, MS_KEY) == l3 and R.ref_softrss(t, 9, MS_KEY) == l4
    with open(os.path.join(GOLD, "rss_kat.json"), "w") as f:
        json.dump({"key": MS_KEY.hex(), "source": "Microsoft RSS verification suite; "
                   "reproduced by reference cne_softrss (lib/core/hash/cne_thash.h:150-163)",
                   "ipv4": [list(k) for k in KAT_V4], "ipv6": [list(k) for k in KAT_V6]}, f, indent=1)

    # --- cne_softrss / cne_softrss_be on random tuples and keys -----------
    n = 4096
    tuples = rng.integers(0, 2**32, size=(n, 9), dtype=np.uint64).astype(np.uint32)
    lens = rng.choice([2, 3, 8, 9, 1, 4, 5], size=n).astype(np.uint32)
    keys = rng.integers(0, 256, size=(4, 40), dtype=np.uint8)
    keys[0] = np.frombuffer(MS_KEY, np.uint8)
    kidx = rng.integers(0, 4, size=n).astype(np.uint32)
    exp = np.zeros(n, np.uint32)
    exp_be = np.zeros(n, np.uint32)
    conv = np.zeros((4, 40), np.uint8)
    for k in range(4):
        R.ref_convert_rss_key(keys[k].ctypes.data, conv[k].ctypes.data, 40)
    for i in range(n):
        t = np.ascontiguousarray(tuples[i])
        exp[i] = R.ref_softrss(t.ctypes.data, int(lens[i]), keys[kidx[i]].ctypes.data)
        exp_be[i] = R.ref_softrss_be(t.ctypes.data, int(lens[i]), conv[kidx[i]].ctypes.data)
    # v6 address loading
    h6 = rng.integers(0, 256, size=(256, 40), dtype=np.uint8)
    load6 = np.zeros((256, 8), np.uint32)
    for i in range(256):
        R.ref_thash_load_v6(np.ascontiguousarray(h6[i]).ctypes.data, load6[i].ctypes.data)
    np.savez_compressed(os.path.join(GOLD, "thash_ref.npz"), tuples=tuples, lens=lens, keys=keys,
                        kidx=kidx, expected=exp, expected_be=exp_be, keys_converted=conv,
                        v6_hdr=h6, v6_loaded=load6)

    # --- cne_ipv4_cksum over every IHL, random bytes ------------------------
    m = 4096
    hdrs = rng.integers(0, 256, size=(m, 64), dtype=np.uint8)
    hdrs[:, 0] = 0x40 | (np.arange(m) % 16)
    # half of them with a correct checksum so both outcomes are covered
    ck = np.zeros(m, np.uint16)
    for i in range(m):
        if i % 2 == 0 and (hdrs[i, 0] & 0xF) >= 5:
            hdrs[i, 10:12] = 0
            c = R.ref_ipv4_cksum(np.ascontiguousarray(hdrs[i]).ctypes.data)
            hdrs[i, 10] = c & 0xFF  # cne_ipv4_cksum returns the LE-summed value
            hdrs[i, 11] = c >> 8
        ck[i] = R.ref_ipv4_cksum(np.ascontiguousarray(hdrs[i]).ctypes.data)
    np.savez_compressed(os.path.join(GOLD, "cksum_ref.npz"), hdrs=hdrs, expected=ck)

    # --- lpm6_data_test.h: 1000 rules + generated IPs + brute-force nh ------
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_lpm6")
    raw = subprocess.run([exe, str(0x43444E50)], check=True, capture_output=True).stdout
    nr = struct.unpack_from("<I", raw, 0)[0]
    rules = np.frombuffer(raw, dtype=np.uint8, count=nr * 18, offset=4).reshape(nr, 18)
    ni = struct.unpack_from("<I", raw, 4 + nr * 18)[0]
    ips = np.frombuffer(raw, dtype=np.uint8, count=ni * 17, offset=8 + nr * 18).reshape(ni, 17)
    sel = np.arange(0, ni, 5)
    np.savez_compressed(os.path.join(GOLD, "lpm6_1000.npz"), rule_ip=rules[:, :16].copy(),
                        rule_depth=rules[:, 16].copy(), rule_nh=rules[:, 17].copy(),
                        ip=ips[sel, :16].copy(), nh=ips[sel, 16].copy())
    for fn in sorted(os.listdir(GOLD)):
        print(fn, os.path.getsize(os.path.join(GOLD, fn)))


if __name__ == "__main__":
    main()
