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
