#!/usr/bin/env python3
"""Headline benchmark: device-resident parse + Toeplitz + LPM classify (Mpps).

python bench.py --gpus N --steps K --warmup W [--config c3|c2|c4|c5]

One step = one classify pass over one batch resident in HBM (default config
C3, the l3fwd-graph workload: 16M x 64-B IPv4/UDP frames per GPU, 1024-prefix
DIR-24-8 LPM + 5-tuple Toeplitz + RSS queue + next-hop bin counters).  For
N > 1 (torchrun) every rank classifies its own batch (weak scaling, no data
collective); after the K timed steps the per-bin counters are all-reduced
once over RCCL (the "final per-output-port count reduce").  Rank 0 prints one
JSON line.  Inputs are generated in HBM (synthetic, seeded) before timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "Mpps device-resident parse+hash+LPM, 64B & IMIX, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    # name: (description, packets per GPU, algorithmic bytes per packet)
    "c2": ("C2 64B IPv4/UDP parse + 5-tuple Toeplitz + RSS queue, 16M pkts/GPU device-resident",
           1 << 24, 64 + 4 + 2),
    "c3": ("C3 l3fwd-graph: 64B IPv4/UDP, 1024-prefix DIR-24-8 LPM + Toeplitz + RSS queue, "
           "16M pkts/GPU device-resident", 1 << 24, 64 + 4 + 4 + 2),
    # the full l3fwd-graph chain: C3's classify then ip4_rewrite in place
    # (read nh 4 + frame bytes 0..27, write 28 + tx edge 2 on top of C3's 74)
    "c3rw": ("C3 + ip4_rewrite: l3fwd-graph classify then MAC rewrite / TTL / checksum in place, "
             "16M pkts/GPU device-resident", 1 << 24, 74 + 4 + 28 + 28 + 2),
    "c4": ("C4 IMIX 64/570/1500 (7:4:1) IPv4+IPv6 cnet parse + DIR-24-8/trie LPM + Toeplitz, "
           "16M pkts/GPU device-resident", 1 << 24, 64 + 4 + 4 + 2),
    "c5": ("C5 1500B IPv4/UDP cnet parse + IPv4 checksum verify + LPM, 32M pkts/GPU "
           "(256M over 8 GPUs) device-resident", 1 << 25, 64 + 4),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def setup_dist():
    from cndp_amd import dist as D
    world, rank, local = D.init_from_env("nccl")
    torch.cuda.set_device(local)
    return world, rank, local


def build_state(cfg: str, dev, rank: int, n_override: int | None, in_route_frac: float = 0.9,
                ring: int = 0):
    from cndp_amd import native as N
    from cndp_amd import pktgen
    from cndp_amd.classify import Classifier
    from cndp_amd.fib import Fib, Fib6, node_ip4_add_input, node_ip4_route_add, node_ip6_add_input

    desc, n, algo = CONFIGS[cfg]
    if n_override:
        n = n_override
    seed = pktgen.SEED + rank
    cl = Classifier(dev.index)
    routes = pktgen.l3fwd_routes()
    state = {"desc": desc, "n": n, "algo": algo, "cl": cl, "routes": routes}
    if cfg in ("c2", "c3", "c3rw"):
        fib = Fib("rt4", N.CNE_FIB_DIR24_8, default_nh=N.IP4_LOOKUP_NEXT_PKT_DROP << 16, max_routes=1024,
                  nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
        for ip, d, nh in routes:
            assert node_ip4_route_add(fib, ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE) == 0
        cl.set_fib(fib)
        state["fib"] = fib
        state["mode"] = N.CNDP_MODE_HASH if cfg == "c2" else N.CNDP_MODE_L3FWD
        state["frames"] = pktgen.packed_ipv4(n, routes=routes, seed=seed, device=dev,
                                             in_route_frac=in_route_frac)
    else:
        nr = 1024
        fib = Fib("rt4-fib", N.CNE_FIB_DIR24_8, default_nh=(0 << 24) | (nr + 1), max_routes=nr,
                  nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
        for i, (ip, d, _) in enumerate(routes):
            assert node_ip4_add_input(fib, ip, d, i) == 0
        v6 = pktgen.v6_routes()
        fib6 = Fib6("rt6-fib", N.CNE_FIB_TRIE, default_nh=(0 << 24) | (nr + 1), max_routes=nr,
                    nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15)
        for ip, d, i in v6:
            assert node_ip6_add_input(fib6, ip, d, i) == 0
        cl.set_fib(fib, fib6)
        state.update(fib=fib, fib6=fib6, v6routes=v6, mode=N.CNDP_MODE_CNET)
        if cfg == "c4":
            state["frames"] = pktgen.imix(n, seed=seed, v4routes=routes, v6routes=v6, device=dev)
        else:
            fr = pktgen.packed_ipv4(n, slot=1536, frame_len=1500, routes=routes, seed=seed, device=dev)
            pktgen.corrupt_cksum(fr, 1024, seed)
            state["frames"] = fr
    # l3fwd / hash: the graph edge is nh >> 16 (no separate edge stream);
    # cnet keeps the edge output (its drop/forward/proto edge is not in nh
    # for packets the ptype node sends elsewhere)
    state["out"] = cl.alloc_outputs(n, 64, device=dev, edge=cfg in ("c4", "c5"))
    # Ring of batches: step k classifies batch k % R, as a NIC ring hands over
    # fresh buffers.  R is sized so that the ring's frames and results are
    # several times the 256 MiB Infinity Cache: no step is served results or
    # frames a previous step left on-die.  The bin counters are shared.
    fr0 = state["frames"]
    batch_bytes = fr0.slab.numel() + sum(t.numel() * t.element_size() for t in state["out"].values()
                                         if isinstance(t, torch.Tensor))
    R = ring if ring > 0 else max(1, min(4, -(-(4 << 30) // batch_bytes)))
    state["ring"] = [(fr0, state["out"])]
    for r in range(1, R):
        if cfg in ("c2", "c3", "c3rw"):
            fr = pktgen.packed_ipv4(n, routes=routes, seed=seed + 1000 * r, device=dev,
                                    in_route_frac=in_route_frac)
        elif cfg == "c4":
            fr = pktgen.imix(n, seed=seed + 1000 * r, v4routes=routes, v6routes=state["v6routes"], device=dev)
        else:
            fr = pktgen.packed_ipv4(n, slot=1536, frame_len=1500, routes=routes, seed=seed + 1000 * r, device=dev)
            pktgen.corrupt_cksum(fr, 1024, seed + 1000 * r)
        o = cl.alloc_outputs(n, 64, device=dev, edge=cfg in ("c4", "c5"))
        o["bins"] = state["out"]["bins"]
        state["ring"].append((fr, o))
    if cfg == "c3rw":
        import random
        rnd_ = random.Random(7)
        for p in range(4):
            cl.rewrite_set_next(p, p + 1)
        for nh in range(64):  # 12-B dst/src MAC rewrite per next hop (l3fwd-graph main.c)
            assert cl.rewrite_add(nh, bytes(rnd_.randrange(256) for _ in range(12)), nh % 4) == 0
        state["tx"] = torch.empty(n, dtype=torch.int16, device=dev)
    return state


def run_step(st, stream=None, k: int = 0):
    """One step of the configured workload (what the timed loop repeats):
    batch k % R of the ring."""
    cl, mode = st["cl"], st["mode"]
    fr, out = st["ring"][k % len(st["ring"])]
    sid = stream.cuda_stream if stream is not None else None
    if "tx" in st:
        cl.classify_rewrite(fr, out=out, burst=256, tx_edge=st["tx"], stream=sid)
    else:
        cl.classify(fr, mode, out=out, stream=sid)


def parity_sample(state, k: int = 1 << 16) -> bool:
    """Cheap spot check of the first k packets against the oracle (untimed)."""
    from cndp_amd import native as N
    from oracle import oracle as O
    fr = state["frames"]
    k = min(k, fr.n)
    cl = state["cl"]
    t24, t8 = (x.copy() for x in state["fib"].image())
    kw = dict(tables4=(t24, t8))
    if state["mode"] == N.CNDP_MODE_CNET:
        kw["tables6"] = tuple(x.copy() for x in state["fib6"].image())
        # the ptype-node model is stateful: restart it (last_type = 0), redo
        # one pass, and compare with the node loop from the same state
        kw["spec_burst"] = 256
        cl.set_tuning(cnet_spec=256)
        cl.classify(fr, state["mode"], out=state["out"])
    if fr.offsets is not None:
        offs = fr.offsets[:k].cpu().numpy().astype(np.uint64)
        end = int(offs[-1]) + 2048
        slab = fr.slab[:min(end, fr.slab.numel())].cpu().numpy()
        ref = O.classify(state["mode"], slab, k, offsets=offs, **kw)
    else:
        slab = fr.slab[:k * fr.stride].cpu().numpy()
        ref = O.classify(state["mode"], slab, k, stride=fr.stride, data_off=fr.data_off, **kw)
    out = state["out"]
    torch.cuda.synchronize()
    ok = True
    for key, dt in (("nh", np.uint32), ("hash", np.uint32), ("queue", np.uint16), ("edge", np.uint8)):
        if out.get(key) is None:
            continue
        g = out[key][:k].cpu().numpy().view(dt)
        ok &= bool(np.array_equal(g, ref[key]))
    return ok


def cpu_baseline(state, budget_s: float = 10.0):
    """The oracle's per-burst l3fwd loop on this host's cores (rank 0, N=1)."""
    from oracle import oracle as O
    fr = state["frames"]
    n = min(fr.n, 1 << 22)
    slab = np.concatenate([fr.slab[: n * fr.stride].cpu().numpy(), np.zeros(256, np.uint8)])
    t24, t8 = (x.copy() for x in state["fib"].image())
    threads = max(1, min(16, os.cpu_count() or 1))
    t1 = O.l3fwd_burst_bench(slab, n, fr.stride, (t24, t8), nthreads=1, iters=1)
    single = n / t1 / 1e6
    tt = O.l3fwd_burst_bench(slab, n, fr.stride, (t24, t8), nthreads=threads, iters=1)
    iters = max(1, int(budget_s / max(tt, 1e-6)))
    tt = O.l3fwd_burst_bench(slab, n, fr.stride, (t24, t8), nthreads=threads, iters=iters)
    multi = n * iters / tt / 1e6
    return {"value": round(multi, 2), "unit": "Mpps", "cores": threads, "kind": "port",
            "sample": (f"oracle/oracle.c per-256-burst l3fwd loop (ethertype parse, 4-wide DIR-24-8 "
                       f"lookup, cne_softrss restatement, RETA) over {n} of the same 64-B frames x "
                       f"{iters} passes on {threads} host threads ({tt:.1f} s); 1 thread: "
                       f"{single:.1f} Mpps")}


def sweep(st, stream, cfg):
    """Kernel-variant sweep (performance only; every variant is parity-tested)."""
    from cndp_amd import native as N
    cl, fr, out, mode = st["cl"], st["frames"], st["out"], st["mode"]
    rows = []
    variants = [dict(tile=0, nt=0, unroll=1, blocks_per_cu=4), dict(tile=0, nt=1, unroll=1, blocks_per_cu=4),
                dict(tile=0, nt=0, unroll=2, blocks_per_cu=4)]
    variants += [dict(tile=t, nt=nt, unroll=1, blocks_per_cu=b) for t in (1, 4) for nt in (0, 1) for b in (2, 4, 8)]
    variants += [dict(tile=2, nt=1, unroll=1, blocks_per_cu=4), dict(tile=3, nt=0, unroll=1, blocks_per_cu=4)]
    variants = [dict(v, dir16=1, load_nt=0) for v in variants] + [dict(tile=4, nt=1, unroll=1, blocks_per_cu=4,
                                                                      dir16=0, load_nt=0)]
    variants += [dict(tile=4, nt=nt, unroll=1, blocks_per_cu=b, dir16=1, load_nt=1) for nt in (1, 0)
                 for b in (2, 3, 4, 6)]
    variants += [dict(tile=5, nt=1, unroll=1, blocks_per_cu=b, dir16=d, load_nt=l) for l in (1, 0)
                 for b in (1, 2, 3, 4) for d in (1, 0)]
    if mode == N.CNDP_MODE_CNET:
        variants = [dict(cnet_tile=ct, dir16=d, cnet_spec=sp, load_nt=l) for sp in (256, 0) for ct in (3, 2, 1, 0)
                    for d in (1, 0) for l in (1, 0) if (sp == 256 or d == 1) and (ct >= 1 or l == 1)]
    if "tx" in st:
        variants = [dict(rw_wb=w, nt=nt, tile=4, load_nt=l, blocks_per_cu=b) for w in (0, 1, 2) for nt in (1, 0)
                    for l in (1, 0) for b in (2, 4)] + [dict(tile=1, rw_wb=0)]
    for v in variants:
        cl.set_tuning(**v)
        for k in range(3):
            run_step(st, stream, k)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for k in range(20):
            run_step(st, stream, k)
        b.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        gbs = st["algo"] * st["n"] / (ms * 1e-3) / 1e9
        rows.append(dict(v, kernel_ms=ms, algo_GBs=gbs, Mpps=st["n"] / ms / 1e3))
        log(f"[sweep {cfg}] {v}: {ms:.4f} ms {gbs:7.1f} GB/s {st['n'] / ms / 1e3:9.1f} Mpps")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"sweep_{cfg}.json"), "w") as f:
        json.dump(rows, f, indent=1)
    cl.set_tuning(tile=5, nt=1, unroll=1, blocks_per_cu=0, dir16=1, cnet_tile=3, rw_wb=2, cnet_spec=256,
                  load_nt=1)


def e2e_host(st, reps: int = 5):
    """Host-memory rates (rank 0, N=1): the frames start in host memory and
    the results end there (SURVEY §8(d) 'End to end').  Two paths, same
    kernel, same batch:
      pinned_stream : pinned host slab -> cndp_gpu_classify_host (64 MiB
                      H2D segments overlapped with classify and D2H of the
                      results, three streams) -> pinned host results;
      zero_copy     : the slab registered in place (cndp_gpu_host_register,
                      as an AF_XDP UMEM would be) and read by the kernel over
                      PCIe; results to HBM."""
    import mmap
    fr, cl, mode, n = st["frames"], st["cl"], st["mode"], st["n"]
    res = {}
    host = fr.slab.cpu().pin_memory()
    offs = fr.offsets.cpu().pin_memory() if fr.offsets is not None else None
    out = {k: torch.zeros(n, dtype=d).pin_memory() for k, d in
           (("nh", torch.int32), ("hash", torch.int32), ("queue", torch.int16))}
    if mode == 1:
        out["edge"] = torch.zeros(n, dtype=torch.uint8).pin_memory()
    out["bins"] = torch.zeros(66, dtype=torch.int64).pin_memory()
    kw = dict(stride=fr.stride, offsets=offs, data_off=fr.data_off, out=out)
    cl.classify_host(host, n, mode, **kw)
    t = time.perf_counter()
    for _ in range(reps):
        cl.classify_host(host, n, mode, **kw)
    dt = (time.perf_counter() - t) / reps
    in_bytes = host.numel() + (n * 8 if offs is not None else 0)
    res["pinned_stream"] = {"Mpps": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 3),
                            "h2d_bytes": in_bytes, "h2d_GBs": round(in_bytes / dt / 1e9, 1)}
    del host, offs, out
    # zero-copy from a registered, page-aligned buffer
    buf = mmap.mmap(-1, fr.slab.numel())
    arr = np.frombuffer(buf, dtype=np.uint8)
    arr[:] = fr.slab.cpu().numpy()
    dptr = cl.host_register(arr)
    try:
        dout = cl.alloc_outputs(n, 64, device=fr.slab.device, edge=mode == 1)
        offs_d = fr.offsets.data_ptr() if fr.offsets is not None else None
        args = (mode, n, dptr, arr.nbytes, dout)
        kw = dict(stride=fr.stride, data_off=fr.data_off, offsets=offs_d)
        cl.classify_ptrs(*args, **kw)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            cl.classify_ptrs(*args, **kw)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
        res["zero_copy"] = {"Mpps": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 3)}
    finally:
        cl.host_unregister(arr)
        del arr
        buf.close()
    return res


def imix_line(dev, rank: int, world: int, steps: int, warmup: int, parity: bool):
    """Secondary line for the IMIX half of the metric (config C4, cnet chain),
    measured the same way as the headline: ring of batches, one event pair
    around `steps` back-to-back launches, max over ranks."""
    from cndp_amd import dist as D
    st = build_state("c4", dev, rank, None)
    stream = torch.cuda.current_stream(dev)
    for k in range(warmup):
        run_step(st, stream, k)
    torch.cuda.synchronize()
    ok = parity_sample(st) if parity and rank == 0 else None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(steps):
        run_step(st, stream, k)
    ev1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps
    elapsed, kern_ms = D.max_over_ranks([elapsed, kern_ms], dev)
    n = st["n"]
    achieved = st["algo"] * n / (kern_ms * 1e-3) / 1e9
    res = {"config": "c4", "workload": st["desc"], "value": round(n * world * steps / elapsed / 1e6, 2),
           "unit": "Mpps", "ms_per_step": round(elapsed / steps * 1e3, 4), "kernel_ms": round(kern_ms, 5),
           "achieved_GBs": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
           "algorithmic_bytes_per_pkt": st["algo"], "ring_batches": len(st["ring"]),
           "parity_sample_vs_oracle": ok}
    del st
    torch.cuda.empty_cache()
    return res


def load_traffic(cfg: str):
    path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=0, help="override packets per GPU")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe) rates")
    ap.add_argument("--sweep", action="store_true", help="time every kernel variant (stderr + gpurun_out)")
    ap.add_argument("--no-imix", action="store_true", help="skip the secondary IMIX (C4) line")
    ap.add_argument("--in-route-frac", type=float, default=0.9,
                    help="share of DIPs inside the route set (SURVEY §8(d): 0.9)")
    ap.add_argument("--ring", type=int, default=0,
                    help="batches in the ring (0 = auto: >= 4 GiB of frames + results, at most 4)")
    ap.add_argument("--load-nt", type=int, default=None)
    ap.add_argument("--cnet-tile", type=int, default=None)
    ap.add_argument("--cnet-spec", type=int, default=None)
    ap.add_argument("--spec-scan", type=int, default=None)
    ap.add_argument("--tile", type=int, default=None)
    ap.add_argument("--dir16", type=int, default=None)
    ap.add_argument("--nt", type=int, default=None)
    ap.add_argument("--unroll", type=int, default=None)
    ap.add_argument("--bpc", type=int, default=None)
    args = ap.parse_args()

    from cndp_amd import dist as D
    world, rank, local = setup_dist()
    dev = torch.device(f"cuda:{local}")
    t0 = time.time()
    st = build_state(args.config, dev, rank, args.packets or None, args.in_route_frac, args.ring)
    torch.cuda.synchronize()
    if rank == 0:
        log(f"[bench] setup {time.time() - t0:.1f}s: {st['desc']}")
    cl, fr, out, mode = st["cl"], st["frames"], st["out"], st["mode"]
    stream = torch.cuda.current_stream(dev)
    cl.set_tuning(nt=args.nt, unroll=args.unroll, blocks_per_cu=args.bpc, tile=args.tile, dir16=args.dir16,
                  load_nt=args.load_nt, cnet_tile=args.cnet_tile, cnet_spec=args.cnet_spec,
                  spec_scan=args.spec_scan)
    if args.sweep and rank == 0:
        sweep(st, stream, args.config)

    for k in range(args.warmup):
        run_step(st, None, k)
    torch.cuda.synchronize()
    parity = None
    if rank == 0 and not args.no_parity:
        parity = parity_sample(st)
        log(f"[bench] parity sample vs oracle: {parity}")
    out["bins"].zero_()

    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    # One HIP event pair on the launch stream brackets the K back-to-back
    # launches: kern_ms = their average duration including the kernel
    # boundary (an event pair per launch adds ~10 us of marker overhead per
    # step on ROCm and would understate the kernel).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for s in range(args.steps):
        run_step(st, stream, s)
    ev1.record(stream)
    D.final_count_reduce(out["bins"])  # the one RCCL collective: per-bin counts
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kern_ms = ev0.elapsed_time(ev1) / args.steps

    elapsed, kern_ms = D.max_over_ranks([elapsed, kern_ms], dev)

    n = st["n"]
    total_pkts = n * world * args.steps
    value = total_pkts / elapsed / 1e6
    achieved = st["algo"] * n / (kern_ms * 1e-3) / 1e9
    bins = out["bins"].cpu().numpy()
    layout = ("packed 64-B slots" if fr.offsets is None and fr.stride == 64
              else ("IMIX packed at roundup(len,64)" if fr.offsets is not None else f"{fr.stride}-B slots"))
    ring_len = len(st["ring"])
    cpu = e2e = None
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline and args.config in ("c2", "c3"):
            cpu = cpu_baseline(st, args.cpu_budget)
        if world == 1 and not args.no_e2e and args.config != "c3rw":
            try:
                e2e = e2e_host(st)
                log(f"[bench] host-memory rates: {e2e}")
            except Exception as ex:  # reported, never fatal for the headline line
                e2e = {"error": repr(ex)}
    imix = None
    if args.config in ("c2", "c3") and not args.no_imix:  # every rank (max over ranks inside)
        del st["ring"], fr, out
        st.pop("frames", None)
        torch.cuda.empty_cache()
        try:
            imix = imix_line(dev, rank, world, max(5, args.steps // 2), args.warmup, not args.no_parity)
            if rank == 0:
                log(f"[bench] IMIX (C4) line: {imix}")
        except Exception as ex:  # reported, never fatal for the headline line
            imix = {"error": repr(ex)}
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded counter-hash frames generated in HBM)",
            "config": {"workload": st["desc"], "config": args.config, "packets_per_gpu": n,
                       "frame_layout": layout,
                       "ring_batches": ring_len,
                       "routes": len(st["routes"]), "parallelism": f"dp{world} (replicated FIB, sharded batches)",
                       "parity_sample_vs_oracle": parity,
                       "bins_total": int(bins.sum())},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(args.config),
                         "kernel_ms": round(kern_ms, 5),
                         "algorithmic_bytes_per_pkt": st["algo"]},
            "cpu_baseline": cpu,
            "host_memory_e2e": e2e,
            "imix": imix,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
