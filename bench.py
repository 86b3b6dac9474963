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

The same line carries, besides the headline:
  configs        every other BASELINE config measured the same way (C2, C4,
                 C5), each with its roofline object and its CPU baseline;
  node_boundary  the graph-node boundary over pktmbuf_t bursts of 256 (the
                 GPU ip4_lookup node, the cnet queue) next to one CPU core
                 running the same nodes;
  host_memory_e2e  frames starting and ending in host memory (packed slab and
                 the AF_XDP UMEM layout), never `value`.
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


def rank_launch_cmd(n: int, argv: list[str], port: int) -> list[str]:
    """The torchrun command that runs this script as n ranks on one node (the
    driver's own form: --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def check_rank_line(line: str, n: int) -> dict:
    """Rank 0's JSON line from an n-rank run: n_gpus must be n and the all-reduced
    bin counters must count every packet of every rank's timed steps."""
    res = json.loads(line)
    cfg = res.get("config", {})
    want = n * int(cfg.get("packets_per_gpu", -1)) * int(res.get("steps", -1))
    if res.get("n_gpus") != n:
        raise ValueError(f"rank line reports n_gpus {res.get('n_gpus')}, launched {n}")
    if cfg.get("bins_total") != want:
        raise ValueError(f"bins_total {cfg.get('bins_total')} != {n} ranks x packets x steps = {want}")
    return res


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` (N > 1) started without torchrun's environment: run
    the N ranks as a child torchrun (no exec: this process never touches the
    GPU; torch.cuda.device_count() does not initialise it on this image), pass
    their other output through to stderr, and print rank 0's JSON line -- the
    one line on stdout -- once it checks out (check_rank_line).  Returns the
    exit status."""
    import socket
    import subprocess
    backend = os.environ.get("CNDP_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend != "gloo" and ndev < n:
        log(f"[bench] --gpus {n}: {ndev} device(s) visible (CNDP_DIST_BACKEND=gloo lets ranks share one)")
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = rank_launch_cmd(n, argv, port)
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in proc.stdout:  # stdout keeps one line, rank 0's JSON; the rest (gloo / RCCL banners) to stderr
        if ln.startswith("{"):
            line = ln.strip()
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        log(f"[bench] ranks exited with status {rc}")
        return rc
    if line is None:
        log("[bench] no JSON line from rank 0")
        return 1
    try:
        check_rank_line(line, n)
    except ValueError as ex:
        log(f"[bench] {ex}")
        return 1
    print(line, flush=True)
    return 0


def setup_dist():
    """One process per GPU (torchrun), RCCL ("nccl") for the one collective.
    CNDP_DIST_BACKEND=gloo rehearses the same multi-rank path on a box with
    fewer GPUs than ranks (ranks then share devices: local_rank % devices)."""
    from cndp_amd import dist as D
    backend = os.environ.get("CNDP_DIST_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    local = int(os.environ.get("LOCAL_RANK", "0")) % ndev
    torch.cuda.set_device(local)
    world, rank, _ = D.init_from_env(backend)
    return world, rank, local


FRAME_MEM = {"c2": None, "c3": None, "c3rw": None, "c4": None, "c5": None}


def frame_mem_name(cfg: str) -> str:
    m = FRAME_MEM.get(cfg)
    return "torch tensor (hipMalloc)" if m is None else f"cndp_gpu_frames_alloc ({m})"


def build_state(cfg: str, dev, rank: int, n_override: int | None, in_route_frac: float = 0.9,
                ring: int = 0, frame_mem: str | None = "default"):
    from cndp_amd import native as N
    from cndp_amd import pktgen
    from cndp_amd.classify import Classifier
    from cndp_amd.fib import Fib, Fib6, node_ip4_add_input, node_ip4_route_add, node_ip6_add_input

    desc, n, algo = CONFIGS[cfg]
    # where the frames live: a torch (hipMalloc) tensor, or device frame memory
    # from cndp_gpu_frames_alloc ("uncached", the receive-ring memory a NIC's
    # peer DMA fills; "cached")
    fm = FRAME_MEM.get(cfg) if frame_mem == "default" else (None if frame_mem == "torch" else frame_mem)
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
                                             in_route_frac=in_route_frac, frame_mem=fm)
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
            state["frames"] = pktgen.imix(n, seed=seed, v4routes=routes, v6routes=v6, device=dev, frame_mem=fm,
                                          family_run=family_run())
        else:
            fr = pktgen.packed_ipv4(n, slot=1536, frame_len=1500, routes=routes, seed=seed, device=dev,
                                    frame_mem=fm)
            pktgen.corrupt_cksum(fr, 1024, seed)
            state["frames"] = fr
    # no config stores the edge stream: l3fwd's edge is nh >> 16, and SURVEY
    # §8(d) counts no edge bytes for cnet either (a cnet frame's edge still
    # shows in its nh -- a FIB value, or invalid when the ptype node sent it
    # elsewhere -- and in the bin counters the parity checks compare; the GPU
    # tests compare the edge stream itself);
    # the per-packet outputs each config's workload asks for, as SURVEY §8(d)
    # counts them: C2 hash + queue (hash mode's nh is a constant), C3 / C4 nh +
    # hash + queue, C5 the verdict / next hop alone (parse + checksum verify +
    # LPM: no flow hash)
    state["out"] = cl.alloc_outputs(n, 64, device=dev, edge=False)
    trim_outputs(cfg, state["out"])
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
                                    in_route_frac=in_route_frac, frame_mem=fm)
        elif cfg == "c4":
            fr = pktgen.imix(n, seed=seed + 1000 * r, v4routes=routes, v6routes=state["v6routes"], device=dev,
                             frame_mem=fm, family_run=family_run())
        else:
            fr = pktgen.packed_ipv4(n, slot=1536, frame_len=1500, routes=routes, seed=seed + 1000 * r, device=dev,
                                    frame_mem=fm)
            pktgen.corrupt_cksum(fr, 1024, seed + 1000 * r)
        o = cl.alloc_outputs(n, 64, device=dev, edge=False)
        o["bins"] = state["out"]["bins"]
        trim_outputs(cfg, o)
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


def family_run() -> int:
    """Measurement of the one-family wave regroup's ceiling (0 unless
    CNDP_BENCH_FAMILY_RUN=R): C4's IMIX with the address family drawn once per
    run of R frames instead of per frame, so every 64-frame wave tile holds
    one family (R = 64) at no regroup cost, in the frames' own memory order.
    A valid batch (the full-batch parity check runs on it); only the timing
    says what a regroup could gain at most."""
    return int(os.environ.get("CNDP_BENCH_FAMILY_RUN", "0"))


OUTPUTS = {"c2": ("hash", "queue"), "c3": ("nh", "hash", "queue"), "c3rw": ("nh", "hash", "queue"),
           "c4": ("nh", "hash", "queue"), "c5": ("nh",)}


def trim_outputs(cfg: str, out: dict) -> None:
    """Drop the per-packet outputs config cfg does not ask for (OUTPUTS)."""
    for k in ("nh", "hash", "queue", "edge"):
        if k not in OUTPUTS[cfg]:
            out[k] = None


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
    """Cheap spot check against the oracle (untimed): k packets at the start of
    the batch, in its middle and at its end.  Every output at the start; in the
    other two windows the stateless ones -- all of them for l3fwd / hash, the
    flow hash for cnet, whose edges and next hops depend on the ptype node's
    state carried from the batch's start."""
    from cndp_amd import native as N
    from oracle import oracle as O
    fr = state["frames"]
    k = min(k, fr.n)
    cl = state["cl"]
    t24, t8 = (x.copy() for x in state["fib"].image())
    kw = dict(tables4=(t24, t8))
    cnet = state["mode"] == N.CNDP_MODE_CNET
    if cnet:
        kw["tables6"] = tuple(x.copy() for x in state["fib6"].image())
        # the ptype-node model is stateful: restart it (last_type = 0), redo
        # one pass, and compare with the node loop from the same state
        kw["spec_burst"] = 256
        cl.set_tuning(cnet_spec=256)
        cl.classify(fr, state["mode"], out=state["out"])
    out = state["out"]
    torch.cuda.synchronize()
    ok = True
    starts = sorted({0, (fr.n // 2) // 256 * 256, (fr.n - k) // 256 * 256})
    for w, i0 in enumerate(starts):
        if fr.offsets is not None:
            offs = fr.offsets[i0:i0 + k].cpu().numpy().astype(np.uint64)
            lo = int(offs.min())
            end = int(offs.max()) + 2048
            slab = fr.slab[lo:min(end, fr.slab.numel())].cpu().numpy()
            ref = O.classify(state["mode"], slab, k, offsets=offs - np.uint64(lo), **kw)
        else:
            slab = fr.slab[i0 * fr.stride:(i0 + k) * fr.stride].cpu().numpy()
            ref = O.classify(state["mode"], slab, k, stride=fr.stride, data_off=fr.data_off, **kw)
        keys = ("nh", "hash", "queue", "edge") if (i0 == 0 or not cnet) else ("hash",)
        for key, dt in (("nh", np.uint32), ("hash", np.uint32), ("queue", np.uint16), ("edge", np.uint8)):
            if key not in keys or out.get(key) is None:
                continue
            g = out[key][i0:i0 + k].cpu().numpy().view(dt)
            ok &= bool(np.array_equal(g, ref[key]))
    return ok


def parity_full(state, max_slab_bytes: int = 8 << 30):
    """The whole batch against the oracle (untimed): every per-packet output
    (nh, hash, queue, edge) and the bin counters of one classify call, cnet
    from the ptype node's initial state like the oracle's node loop -- when the
    slab fits the host comfortably (C2, C3, C4), or in 1M-frame pieces for a
    strided slab that does not (C5's 48 GiB shard).  None when skipped."""
    from cndp_amd import native as N
    from oracle import oracle as O
    fr = state["frames"]
    chunked = fr.slab.numel() > max_slab_bytes
    if chunked and fr.offsets is not None:
        return None
    t0 = time.perf_counter()
    cl, out = state["cl"], state["out"]
    kw = dict(tables4=tuple(x.copy() for x in state["fib"].image()))
    cnet = state["mode"] == N.CNDP_MODE_CNET
    if cnet:
        kw["tables6"] = tuple(x.copy() for x in state["fib6"].image())
        kw["spec_burst"] = 256
        cl.set_tuning(cnet_spec=256)  # the node state back to 0, as the oracle starts
    o = dict(out)
    o["bins"] = torch.zeros_like(out["bins"])
    cl.classify(fr, state["mode"], out=o)
    torch.cuda.synchronize()
    keys = [(k, dt) for k, dt in (("nh", np.uint32), ("hash", np.uint32), ("queue", np.uint16), ("edge", np.uint8))
            if o.get(k) is not None]
    diff = {k: 0 for k, _ in keys}
    if not chunked:
        slab = fr.slab.cpu().numpy()
        if fr.offsets is not None:
            ref = O.classify(state["mode"], slab, fr.n, offsets=fr.offsets.cpu().numpy().astype(np.uint64),
                             data_off=fr.data_off, **kw)
        else:
            ref = O.classify(state["mode"], slab, fr.n, stride=fr.stride, data_off=fr.data_off, **kw)
        del slab
        for key, dt in keys:
            diff[key] = int(np.sum(o[key].cpu().numpy().view(dt) != ref[key]))
        ref_bins = ref["bins"]
    else:
        # C5: the shard in 1M-frame pieces (1.5 GiB of slab each), the ptype
        # node's state carried from piece to piece as the node carries it
        # across bursts -- the same walk as one call
        state16 = np.zeros(1, np.uint16)
        ref_bins = None
        step = 1 << 20
        for c0 in range(0, fr.n, step):
            c1 = min(fr.n, c0 + step)
            slab = fr.slab[c0 * fr.stride:c1 * fr.stride].cpu().numpy()
            ref = O.classify(state["mode"], slab, c1 - c0, stride=fr.stride, data_off=fr.data_off,
                             spec_state=state16 if cnet else None, **kw)
            del slab
            for key, dt in keys:
                diff[key] += int(np.sum(o[key][c0:c1].cpu().numpy().view(dt) != ref[key]))
            ref_bins = ref["bins"] if ref_bins is None else ref_bins + ref["bins"]
    diff["bins"] = int(np.sum(o["bins"].cpu().numpy().view(np.uint64) != ref_bins))
    return {"frames": fr.n, "equal": all(v == 0 for v in diff.values()), "mismatches": diff,
            "pieces": -(-fr.n // (1 << 20)) if chunked else 1, "seconds": round(time.perf_counter() - t0, 1)}


def host_cpus():
    """CPUs this process may run on, the CPU model, and the cgroup CPU quota."""
    cpus = sorted(os.sched_getaffinity(0))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return cpus, model, quota


def spread_cpus(cpus: list[int], k: int) -> list[int]:
    """k of the allowed CPUs for k pinned worker threads, as a packet-processing
    deployment places its lcores: one physical core each (no SMT sibling of a
    core already taken) and spread round-robin over the L3 domains (CCDs), so
    no two threads share an L3 while another is free; the GPU's NUMA node
    first.  Falls back to the first k CPUs where sysfs has no topology."""
    def rd(path):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return None
    node = rd("/sys/class/drm/card0/device/numa_node") or rd("/sys/class/drm/card1/device/numa_node")
    groups: dict = {}
    for c in cpus:
        l3 = rd(f"/sys/devices/system/cpu/cpu{c}/cache/index3/id")
        if l3 is None:
            return cpus[:k]
        nd = next((n for n in range(8) if os.path.exists(f"/sys/devices/system/cpu/cpu{c}/node{n}")), 0)
        groups.setdefault((0 if node is None or str(nd) == node else 1, nd, int(l3)), []).append(c)
    order = [groups[g] for g in sorted(groups)]
    taken, siblings = [], set()
    while len(taken) < k and any(order):
        for g in order:
            while g and g[0] in siblings:
                g.pop(0)
            if g and len(taken) < k:
                c = g.pop(0)
                taken.append(c)
                sib = rd(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") or str(c)
                for part in sib.split(","):
                    lo, _, hi = part.partition("-")
                    siblings.update(range(int(lo), int(hi or lo) + 1))
    return taken if len(taken) == k else cpus[:k]


def cpu_baseline(state, budget_s: float = 10.0):
    """The reference chain on this host's cores (rank 0, N=1), one pinned
    thread per CPU of the process's affinity set, and 1 thread, over a bounded
    sample of the same frames repeated to ~budget_s:
      C2 / C3: the l3fwd node loop per 256-packet burst (oracle/oracle.c);
      C4 / C5: the cnet chain as a graph walk runs it (oracle/cnet_chain.c:
        eth_rx -> ptype -> ip4_input / ip6_input over pktmbuf_t pointers,
        direct loads, the nodes' prefetching), with the reference's
        cne_softrss as the flow hash the GPU line computes; no_hash_Mpps is
        the same chain without it (CNDP's cnet nodes hash nothing), and
        checker_Mpps the per-frame checker loop earlier rounds reported."""
    from cndp_amd import native as N
    from oracle import oracle as O
    fr, mode = state["frames"], state["mode"]
    cnet = mode == N.CNDP_MODE_CNET
    n = min(fr.n, (1 << 20) if cnet else (1 << 22))
    kw = {"tables4": tuple(x.copy() for x in state["fib"].image())}
    if cnet:
        kw["tables6"] = tuple(x.copy() for x in state["fib6"].image())
    if fr.offsets is not None:
        offs = fr.offsets[:n].cpu().numpy().astype(np.uint64)
        slab = fr.slab[: int(offs[-1]) + 2048].cpu().numpy()
        kw["offsets"] = offs
    else:
        slab = np.concatenate([fr.slab[: n * fr.stride].cpu().numpy(), np.zeros(2048, np.uint8)])
        kw.update(stride=fr.stride, data_off=fr.data_off)
        offs = np.arange(n, dtype=np.uint64) * np.uint64(fr.stride) + np.uint64(fr.data_off)
    cpus, model, quota = host_cpus()
    aff = len(cpus)
    # one pinned thread per CPU of the quota (a quota below the affinity set),
    # on distinct physical cores spread over the L3 domains (spread_cpus)
    cpus = spread_cpus(cpus, min(len(cpus), max(1, int(-(-quota // 1)))) if quota else len(cpus))
    extra = {}
    if cnet:
        lens = (fr.lengths[:n].cpu().numpy() if fr.lengths is not None
                else np.full(n, min(fr.stride, 1500) if fr.stride else 1500)).astype(np.uint16)
        hdr, ptrs = O.slab_mbufs(slab, offs, lens)
        tabs = (kw["tables4"], kw["tables6"])

        def run(threads, iters, h):
            return O.cnet_chain(ptrs, n, lens, 0, *tabs, hash=h, nthreads=threads, iters=iters,
                                cpus=cpus[:threads])
        # the flow hash on the CPU too when the GPU line outputs it (C4), not
        # when it does not (C5: parse + checksum verify + LPM)
        wh = state["out"].get("hash") is not None
        t1 = run(1, 1, wh)
        single = n / t1 / 1e6
        tt = run(len(cpus), 1, wh)
        iters = max(1, int(budget_s / max(tt, 1e-6)))
        tt = run(len(cpus), iters, wh)
        multi = n * iters / tt / 1e6
        if wh:
            th = run(len(cpus), iters, False)
            extra["no_hash_Mpps"] = round(n * iters / th / 1e6, 2)
            extra["no_hash_single_core_Mpps"] = round(n / run(1, 1, False) / 1e6, 2)
            extra["no_hash_note"] = ("the same chain without the flow hash, which CNDP's cnet nodes never "
                                     "compute (the reference chain's own work)")
        tc = O.burst_bench(mode, slab, n, nthreads=len(cpus), iters=1, cpus=cpus, **kw)
        extra["checker_Mpps"] = round(n / tc / 1e6, 2)
        extra["checker_note"] = ("oracle/oracle.c's per-frame checker loop (bounds-checked byte reads, "
                                 "no prefetching), the figure earlier rounds reported")
        chain = ("cnet chain per 256-mbuf graph walk over pktmbuf_t pointers (oracle/cnet_chain.c: eth_rx "
                 "mbuf_update with cne_get_ptype, ptype-node speculation, ip4/ip6_input length + checksum + "
                 "metadata + 4-wide DIR-24-8 / trie lookups, the nodes' prefetching" +
                 ("; plus the reference's cne_softrss flow hash the GPU line computes -- no_hash_Mpps drops it)"
                  if wh else ")"))
        del hdr
    else:
        t1 = O.burst_bench(mode, slab, n, nthreads=1, iters=1, cpus=cpus[:1], **kw)
        single = n / t1 / 1e6
        tt = O.burst_bench(mode, slab, n, nthreads=len(cpus), iters=1, cpus=cpus, **kw)
        iters = max(1, int(budget_s / max(tt, 1e-6)))
        tt = O.burst_bench(mode, slab, n, nthreads=len(cpus), iters=iters, cpus=cpus, **kw)
        multi = n * iters / tt / 1e6
        chain = ("l3fwd node loop per 256-burst (ethertype parse, pkt_cls, ip4_lookup's 4-wide "
                 "cne_fib_lookup_bulk with dir24_8.h's prefetching lookup" +
                 (", skipped in C2" if mode == N.CNDP_MODE_HASH else "") + ", cne_softrss restatement, RETA)")
    return {"value": round(multi, 2), "unit": "Mpps", "cores": len(cpus), "kind": "port",
            "cpu_model": model, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "single_core_Mpps": round(single, 2), **extra,
            "sample": (f"{chain} over {n} of the same frames x {iters} passes on "
                       f"{len(cpus)} pinned threads ({tt:.1f} s); 1 thread: {single:.2f} Mpps")}


def sweep(st, stream, cfg):
    """Kernel-variant sweep (performance only; every variant is parity-tested)."""
    from cndp_amd import native as N
    cl, fr, out, mode = st["cl"], st["frames"], st["out"], st["mode"]
    rows = []
    variants = [dict(tile=0, nt=nt, blocks_per_cu=b) for nt in (0, 1) for b in (2, 4)]
    variants += [dict(tile=1, nt=nt, blocks_per_cu=b, dir16=d, load_nt=l) for nt in (1, 0) for l in (1, 0)
                 for b in (1, 2, 3, 4) for d in (1, 0)]
    if mode == N.CNDP_MODE_CNET:
        variants = [dict(cnet_tile=ct, dir16=d, cnet_spec=sp, load_nt=l) for sp in (256, 0) for ct in (1, 0)
                    for d in (1, 0) for l in (1, 0) if (sp == 256 or d == 1) and (ct >= 1 or l == 1)]
    if "tx" in st:
        variants = [dict(rw_wb=w, nt=nt, load_nt=l, blocks_per_cu=b) for w in (0, 1, 2) for nt in (1, 0)
                    for l in (1, 0) for b in (2, 4)]
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
    cl.set_tuning(tile=1, nt=1, unroll=1, blocks_per_cu=0, dir16=1, cnet_tile=1, rw_wb=2, cnet_spec=256,
                  load_nt=1)


def e2e_host(st, reps: int = 5, frames=None):
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
    fr, cl, mode = frames or st["frames"], st["cl"], st["mode"]
    n = fr.n
    res = {}
    host = fr.slab.cpu().pin_memory()
    offs = fr.offsets.cpu().pin_memory() if fr.offsets is not None else None
    out = {k: torch.zeros(n, dtype=d).pin_memory() for k, d in
           (("nh", torch.int32), ("hash", torch.int32), ("queue", torch.int16))}
    if mode == 1:
        out["edge"] = torch.zeros(n, dtype=torch.uint8).pin_memory()
    out["bins"] = torch.zeros(66, dtype=torch.int64).pin_memory()
    kw = dict(stride=fr.stride, offsets=offs, data_off=fr.data_off, out=out)
    # frames at a stride wider than their 64-B window (the AF_XDP UMEM layout):
    # the windows alone cross PCIe (CNDP_TUNE_HOST_WINDOW, the default), and,
    # beside it, the whole slab mirrored as before
    strided = offs is None and fr.stride > 64
    for key, window in (("pinned_stream", 1),) + ((("pinned_stream_whole_frames", 0),) if strided else ()):
        cl.set_tuning(host_window=window)
        cl.classify_host(host, n, mode, **kw)
        t = time.perf_counter()
        for _ in range(reps):
            cl.classify_host(host, n, mode, **kw)
        dt = (time.perf_counter() - t) / reps
        in_bytes = (n * 64 if strided and window else host.numel()) + (n * 8 if offs is not None else 0)
        res[key] = {"Mpps": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 3),
                    "h2d_bytes": in_bytes, "h2d_GBs": round(in_bytes / dt / 1e9, 1)}
        if strided and window:
            res[key]["copy"] = "64-B windows, one strided 2-D H2D copy per 1M-frame chunk (hipMemcpy2DAsync)"
    cl.set_tuning(host_window=1)
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


def probe_ceiling(st, stream, steps: int, kern_ms: float) -> dict:
    """The same-box ceiling of this config's memory traffic (untimed for the
    line, measured right after the kernel's timed windows): the access-shape
    probes of cndp_amd/csrc/roofline_probe.hip move the kernel's frame reads
    and result stores over the same ring of batches and outputs, and nothing
    else.  A few launch shapes are tried; the fastest is the ceiling.
    kernel_over_probe = kernel_ms / probe_ms tells this box's HBM apart from
    the kernel.  For C4 / C5 a second probe stores only the 4-B next hop
    SURVEY §8(d) counts, pricing the extra result bytes the kernel writes."""
    import ctypes
    P = ctypes.CDLL(os.path.join(ROOT, "cndp_amd", "lib", "libcndp_probe.so"))
    P.cndp_probe_slots.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 3 + \
        [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    P.cndp_probe_slots_bal.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 4
    P.cndp_probe_windows.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_uint64] + [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.c_void_p]
    ring = st["ring"]
    sid = stream.cuda_stream
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    fr0 = ring[0][0]
    cnet = fr0.offsets is not None or fr0.stride != 64
    t16 = torch.empty(fr0.n, dtype=torch.int16, device=fr0.slab.device) if cnet else None

    def timed(launch):
        for k in range(3):
            assert launch(k) == 0
        best = None
        for _ in range(2):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for k in range(steps):
                launch(k)
            b.record(stream)
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / steps
            best = ms if best is None else min(best, ms)
        return best

    rows = {}
    if not cnet:
        for pf in (1, 2):
            for bpc in (2, 4):
                def launch(k, pf=pf, bpc=bpc):
                    fr, o = ring[k % len(ring)]
                    return P.cndp_probe_slots(fr.slab.data_ptr(), fr.n, ptr(o.get("nh")), ptr(o.get("hash")),
                                              ptr(o.get("queue")), pf, bpc, sid)
                rows[f"slots_pf{pf}_bpc{bpc}"] = timed(launch)

        def blaunch(k):
            fr, o = ring[k % len(ring)]
            return P.cndp_probe_slots_bal(fr.slab.data_ptr(), fr.n, ptr(o.get("nh")), ptr(o.get("hash")),
                                          ptr(o.get("queue")), sid)
        rows["slots_balanced_512x1"] = timed(blaunch)
        shape = ("packed 64-B slots: 4 x 1 KiB nt loads per 64-frame wave tile through the LDS tile, the "
                 "kernel's result stores (nh / hash / queue as allocated), nothing else; static schedules "
                 "(1-2 tiles in flight, 2-4 blocks a CU) and the kernel's balanced one (one 512-thread block "
                 "a CU, tiles shared through an LDS counter)")
    else:
        def wlaunch(bpc, algo_only):
            def launch(k):
                fr, o = ring[k % len(ring)]
                offs = fr.offsets.data_ptr() if fr.offsets is not None else None
                if algo_only:
                    outs = (ptr(o.get("nh")), None, None, None, None)
                else:
                    outs = (ptr(o.get("nh")), ptr(o.get("hash")), ptr(o.get("queue")), ptr(o.get("edge")), ptr(t16))
                return P.cndp_probe_windows(fr.slab.data_ptr(), fr.stride, offs, fr.data_off, fr.n, *outs, bpc, sid)
            return launch
        for bpc in (4, 8):
            rows[f"windows_bpc{bpc}"] = timed(wlaunch(bpc, False))
        rows["windows_balanced_1024x1"] = timed(wlaunch(0, False))
        shape = ("the first 64 B of each frame (4 lanes a frame, 16 frames a load instruction, nt loads"
                 + (", u64 offsets read coalesced" if fr0.offsets is not None else f", {fr0.stride}-B stride")
                 + "), the kernel's result stores (nh / hash / queue / edge + the 2-B packet type of the "
                 "speculation model), nothing else; static schedules (4 / 8 blocks a CU) and k_cnet_defer's "
                 "balanced one (one 1024-thread block a CU, tiles shared through an LDS counter)")
    best = min(rows, key=rows.get)
    res = {"probe_ms": round(rows[best], 5), "kernel_over_probe": round(kern_ms / rows[best], 4),
           "probe_variant": best, "probe_variants_ms": {k: round(v, 5) for k, v in rows.items()},
           "probe_shape": shape}
    if cnet:
        bpc = int(best.rsplit("bpc", 1)[1]) if "bpc" in best else 0  # 0: the balanced probe
        res["probe_nh_only_ms"] = round(timed(wlaunch(bpc, True)), 5)
        res["probe_nh_only_note"] = ("the same windows with only the 4-B next hop stored (SURVEY §8(d)'s "
                                     "algorithmic bytes): probe_ms - this = the cost of the other result bytes")
    del t16
    return res


def config_line(cfg: str, dev, rank: int, world: int, steps: int, warmup: int, parity: bool,
                cpu: bool, cpu_budget: float, probe: bool = True):
    """One more BASELINE config measured like the headline: ring of batches,
    one event pair around `steps` back-to-back launches, max over ranks, with
    its roofline object (traffic from profiles/pmc_<cfg>.json) and, on rank 0
    at N=1, its CPU baseline."""
    from cndp_amd import dist as D
    st = build_state(cfg, dev, rank, None)
    stream = torch.cuda.current_stream(dev)
    for k in range(warmup):
        run_step(st, stream, k)
    torch.cuda.synchronize()
    ok = parity_sample(st) if parity and rank == 0 else None
    full = parity_full(st) if parity and rank == 0 else None
    # the parity checks restart the cnet node model (state 0): one call
    # settles it again, as the warmup did, before the timed windows
    for k in range(max(1, warmup)):
        run_step(st, stream, k)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # three timed windows of `steps` launches, the median one reported: a
    # window is ~10-25 ms here, so one host hiccup (seen once: +5.8 ms on C4)
    # would otherwise be a third of the line
    wins = []
    for _ in range(3):
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for k in range(steps):
            run_step(st, stream, k)
        ev1.record(stream)
        torch.cuda.synchronize()
        wins.append((time.perf_counter() - t0, ev0.elapsed_time(ev1) / steps))
    elapsed, kern_ms = sorted(wins)[1]
    elapsed, kern_ms = D.max_over_ranks([elapsed, kern_ms], dev)
    n = st["n"]
    achieved = st["algo"] * n / (kern_ms * 1e-3) / 1e9
    value = n * world * steps / elapsed / 1e6
    res = {"config": cfg, "workload": st["desc"], "value": round(value, 2),
           "unit": "Mpps", "ms_per_step": round(elapsed / steps * 1e3, 4), "packets_per_gpu": n,
           "ring_batches": len(st["ring"]), "frame_memory": frame_mem_name(cfg), "parity_sample_vs_oracle": ok,
           "parity_full_batch_vs_oracle": full,
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(cfg),
                        "kernel_ms": round(kern_ms, 5), "algorithmic_bytes_per_pkt": st["algo"]}}
    if probe and rank == 0:
        try:
            res["roofline"].update(probe_ceiling(st, stream, steps, kern_ms))
        except Exception as ex:  # reported, never fatal
            res["roofline"]["probe_error"] = repr(ex)
    if cfg == "c5":  # the 1500-B point also as wire-equivalent bandwidth
        pps = value * 1e6
        res["wire_Gbps"] = {"l2_1500B": round(pps * 1500 * 8 / 1e9, 1),
                            "line_1500B_plus_20B_preamble_ifg": round(pps * 1520 * 8 / 1e9, 1)}
    if cpu and rank == 0 and world == 1:
        try:
            res["cpu_baseline"] = cpu_baseline(st, cpu_budget)
        except Exception as ex:  # reported, never fatal
            res["cpu_baseline"] = {"error": repr(ex)}
    del st
    torch.cuda.empty_cache()
    return res


def fib_update(reps: int = 15) -> dict:
    """Route churn between batches: K route adds at
    scattered prefixes, then the first GPU-selection lookup, which syncs the
    HBM mirror -- the device painter of the changed ranges against the
    bounding-range copy (CNDP_FIB_PAINT=0).  Medians of `reps`: the call's
    µs (a 4-key lookup alone is ~10 µs) and the bytes the sync moved."""
    import ctypes
    import numpy as np
    from cndp_amd import native as N
    from cndp_amd.fib import Fib

    def stats(f):
        b, c = ctypes.c_uint64(), ctypes.c_uint64()
        N.lib().cndp_fib_sync_stats(f.h, ctypes.byref(b), ctypes.byref(c))
        return b.value, c.value

    res = {"what": "K scattered route adds (/16../32) then one 4-key GPU-selection lookup (mirror sync + lookup)"}
    old = os.environ.get("CNDP_FIB_PAINT")
    try:
        for mode, env in (("device_paint", "1"), ("bounding_copy", "0")):
            os.environ["CNDP_FIB_PAINT"] = env
            rng = np.random.default_rng(3)
            f = Fib(f"upd_{mode}", N.CNE_FIB_DIR24_8, default_nh=1 << 16, max_routes=1 << 16,
                    nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=4096, lookup=N.CNE_FIB_LOOKUP_GPU)
            keys = rng.integers(0, 2**32, size=4, dtype=np.uint64).astype(np.uint32)
            f.lookup_bulk(keys)
            for k in (8, 64):
                rows = []
                for _ in range(reps):
                    for _ in range(k):
                        d = int(rng.choice([16, 24, 24, 24, 28, 32]))
                        ip = int(rng.integers(0, 2**32)) & ((0xFFFFFFFF << (32 - d)) & 0xFFFFFFFF)
                        f.add(ip, d, int(rng.integers(0, 1 << 15)))
                    b0, _ = stats(f)
                    t = time.perf_counter()
                    f.lookup_bulk(keys)
                    dt = time.perf_counter() - t
                    rows.append((dt * 1e6, stats(f)[0] - b0))
                a = np.array(rows)
                res.setdefault(mode, {})[f"changes_{k}"] = {"median_us": round(float(np.median(a[:, 0])), 1),
                                                            "median_bytes": int(np.median(a[:, 1]))}
            del f
    finally:
        if old is None:
            os.environ.pop("CNDP_FIB_PAINT", None)
        else:
            os.environ["CNDP_FIB_PAINT"] = old
    return res


HEADER_STATE_NOTE = (
    "primary keys: every burst's mbuf headers were written on the host core just before the node saw them, as "
    "a real receive leaves them (xskdev.c:296-297 data_len / data_off; for the l3fwd nodes behind pktdev_rx also "
    "its soft parse's packet_type) -- on the GPU legs by the test harness's receive stub / driver, on the CPU "
    "legs by the oracle loops -- so header lines are dirty in that core's cache; cold_*: no such writes, the "
    "lines in whatever state the previous pass left them")


def node_boundary(dev, n: int = 1 << 20, burst: int = 256, passes: int = 3):
    """The graph-node boundary over pktmbuf_t bursts (rank 0, N=1).  One host
    thread drives, as one lcore's graph walk would:
      l3fwd : the GPU ip4_lookup node (cndp_amd/node/ip4_lookup_gpu.c, through
              the test-only graph stand-in) -- process() per burst, the drain
              source node per walk -- mbufs in a UMEM-layout pool, read in
              place (zero-copy) or staged; beside it the ip4_lookup node's CPU
              loop over the same mbufs on one core;
      cnet  : the cnet queue (eth_rx + ptype + ip4/ip6_input) driven per burst
              from C, zero-copy and staged; beside it the cnet chain on one core.
    Rates are mbufs in -> mbufs out with every field written back."""
    import ctypes
    from cndp_amd import native as N
    from cndp_amd import pktgen
    from cndp_amd.classify import Classifier
    from cndp_amd.fib import Fib, Fib6, NodeFib, cne_node_ip4_route_add, node_ip4_add_input, node_ip6_add_input
    from cndp_amd.mbuf import MbufPool, MbufQueue
    from oracle import oracle as O
    hp = os.path.join(ROOT, "tests", "node_harness", "libnode_harness.so")
    L = N.lib()
    H = ctypes.CDLL(hp)
    H.harness_drive.restype = ctypes.c_double
    H.harness_drive.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int]
    H.harness_mq_drive.restype = ctypes.c_double
    H.harness_mq_drive.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int]
    res = {"burst": burst, "mbufs": n, "host_threads": 1, "batch": 8192, "depth": 4,
           "pool": "2 KiB frames, pktmbuf_t at +0, data at +256 (pktmbuf.c:60-80)"}
    routes = pktgen.l3fwd_routes()
    # ---- l3fwd: the ip4_lookup node
    pool = MbufPool(n)
    pool.fill(pktgen.packed_ipv4(n, routes=routes, seed=99))
    ptrs = pool.ptrs(np.arange(n))
    l3 = {"header_state": HEADER_STATE_NOTE}
    NodeFib.fini()
    H.harness_rx_parse.argtypes = [ctypes.c_int]
    H.harness_driver_writes.argtypes = [ctypes.c_int]
    # Interleaved A/B, two rounds, medians.  Primary form: each burst's mbuf
    # headers written first as a graph on this lcore leaves them -- the
    # receive driver's data_len / data_off stores (xskdev.c:296-297) and
    # pktdev_rx's soft parse (pktdev_rx.c:36-101) -- then the GPU ip4_lookup
    # node with the kernel reading each header itself (CNDP_MQ_F_DEVICE_HEADERS,
    # the node's default) or the host resolving the frame addresses, or staged.
    # cold_*: the same without the header writes (the lines as the previous
    # pass left them).
    D = N.CNDP_MQ_F_DEVICE_HEADERS  # the node's default
    variants = [("gpu_zero_copy", True, D, 1), ("gpu_zero_copy_host_headers", True, 0, 1), ("gpu_staged", False, 0, 1),
                ("cold_gpu_zero_copy", True, D, 0), ("cold_gpu_zero_copy_host_headers", True, 0, 0),
                ("cold_gpu_staged", False, 0, 0)]
    ab = {v[0]: [] for v in variants}
    gid = 10
    snap = None
    for rnd in range(2):
        for name, zc, flags, drv in variants:
            L.cndp_node_gpu_umem_reset()
            if zc:
                L.cndp_node_gpu_umem_add(pool.base, pool.mem.nbytes)
            os.environ["CNDP_GPU_MQ_FLAGS"] = str(flags)
            gid += 1
            assert H.harness_graph_create(gid) == 0
            for ip, d, nh in routes:
                cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
            H.harness_driver_writes(drv)
            H.harness_rx_parse(drv)
            pool.hdr["udata64"] = 0
            H.harness_drive(b"ip4_lookup", ptrs, n, burst, 1)  # warm-up (and the results checked below)
            if rnd == 0 and name == "gpu_zero_copy":
                snap = pool.hdr["udata64"].copy()  # node_mbuf_priv1 as the GPU node left it, primary form
            t = H.harness_drive(b"ip4_lookup", ptrs, n, burst, passes)
            H.harness_driver_writes(0)
            H.harness_rx_parse(0)
            H.harness_graph_destroy()
            ab[name].append(n * passes / t / 1e6 if t > 0 else 0.0)
    os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
    for name, v in ab.items():
        l3[name + "_Mpps"] = round(float(np.median(v)), 2) if min(v) > 0 else None
    l3["ab_rounds"] = {k: [round(x, 2) for x in v] for k, v in ab.items()}
    L.cndp_node_gpu_umem_reset()
    gpu_priv1 = pool.hdr["udata64"].copy()  # after the last (cold, staged) run
    fib = NodeFib()
    t24, t8 = (x.copy() for x in fib.image())
    pool.hdr["udata64"] = 0
    O.ip4_lookup_mbufs(ptrs, n, (t24, t8), burst, 1)
    # every mbuf's priv1 from the GPU node (primary form, and the last cold
    # run) against the CPU node loop's
    l3["results_equal_cpu_node"] = bool(snap is not None and np.array_equal(snap, pool.hdr["udata64"]))
    l3["cold_results_equal_cpu_node"] = bool(np.array_equal(gpu_priv1, pool.hdr["udata64"]))
    # the CPU legs in the same two header states (primary: driver writes +
    # soft parse before each burst, as the GPU legs had them)
    O.set_driver_writes(True)
    O.rx_ip4_lookup_mbufs(ptrs, n, (t24, t8), burst, 1)
    t = O.rx_ip4_lookup_mbufs(ptrs, n, (t24, t8), burst, passes)
    l3["cpu_1core_Mpps"] = round(n * passes / t / 1e6, 2)
    O.set_driver_writes(False)
    O.ip4_lookup_mbufs(ptrs, n, (t24, t8), burst, 1)
    t = O.ip4_lookup_mbufs(ptrs, n, (t24, t8), burst, passes)
    l3["cold_cpu_1core_Mpps"] = round(n * passes / t / 1e6, 2)
    l3["cpu_chain"] = ("the ip4_lookup node loop over the same mbufs on one core (oracle/oracle.c "
                       "orc_ip4_lookup_mbufs); primary form with the receive driver's header writes and "
                       "pktdev_rx's soft parse before each burst (orc_rx_ip4_lookup_mbufs), as the GPU legs")
    l3["supported_build"] = ("no: the GPU ip4_lookup node behind CNDP's own pktdev_rx is measured for the "
                             "record; cndp_amd/node/ip4_lookup_gpu.c links only with pktdev_rx_gpu.c, so an "
                             "l3fwd-graph build gets l3fwd_rx_chain's node (INTEGRATION.md section 2)")
    NodeFib.fini()
    res["l3fwd_ip4_lookup"] = l3
    # ---- l3fwd: the ip4_lookup + ip4_rewrite node pair, chained as a graph
    # walk runs them (ip4_lookup's enqueues fill ip4_rewrite's stream)
    res["l3fwd_lookup_rewrite"] = l3fwd_pair(H, L, pool, ptrs, n, burst, passes, routes)
    res["l3fwd_rx_chain"] = l3fwd_rx_chain(L, pool, ptrs, n, passes, routes)
    del ptrs, pool
    # ---- cnet: eth_rx + ptype + ip4_input / ip6_input
    nc = n // 4
    v6 = pktgen.v6_routes()
    cl = Classifier(dev.index)
    f4 = Fib("nb4", N.CNE_FIB_DIR24_8, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
    for i, (ip, d, _) in enumerate(routes):
        node_ip4_add_input(f4, ip, d, i)
    f6 = Fib6("nb6", N.CNE_FIB_TRIE, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15)
    for ip, d, i in v6:
        node_ip6_add_input(f6, ip, d, i)
    cl.set_fib(f4, f6)
    pool = MbufPool(nc)
    pool.fill(pktgen.imix(nc, v4routes=routes, v6routes=v6, seed=98))
    ptrs = pool.ptrs(np.arange(nc))
    hdr0 = pool.hdr.copy()
    cn = {}
    D = N.CNDP_MQ_F_DEVICE_HEADERS

    def cnet_queue(zc, flags):
        umem = None
        if zc:
            cl.host_register(pool.mem)
            umem = pool.base
        q = MbufQueue(cl, N.CNDP_MQ_CNET, flags=flags, batch=8192, depth=4, umem=umem)
        # eth_rx advances data_off by l2_len in every mbuf it returns: each pass
        # starts from the received mbufs again (headers restored outside the clock)
        t = 0.0
        for p in range(passes + 1):  # pass 0 warms up
            pool.hdr[:] = hdr0
            dt = H.harness_mq_drive(q.h, ptrs, nc, burst, 1)
            if dt < 0:
                t = -1.0
                break
            t += dt if p else 0.0
        q.close()
        if zc:
            cl.host_unregister(pool.mem)
        return round(nc * passes / t / 1e6, 2) if t > 0 else None

    # the same through the GPU eth_rx graph node (cndp_amd/node/eth_rx_gpu.c):
    # graph walks pull 256-mbuf bursts from the port, finished mbufs leave on
    # the ptype / ip4_input / ip6_input edges
    HC = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "libcnet_harness.so"))
    HC.harness_rx_load.argtypes = [ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint32]
    HC.harness_cnet_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    HC.harness_eth_rx_port.argtypes = [ctypes.c_uint32, ctypes.c_uint16]
    HC.harness_walk_until.argtypes = [ctypes.c_uint64]
    HC.harness_walk_until.restype = ctypes.c_double
    HC.harness_cnet_set(f4.h, f6.h)
    HC.harness_eth_rx_port(0, 0)

    gids = iter(range(40, 80))
    # the fields eth_rx / ptype / ip4_input / ip6_input write, after the GPU
    # node's first pass from a fresh graph (ptype node state 0)
    cnet_fields = ("packet_type", "ol_flags", "tx_offload", "lport", "data_off", "data_len")
    snap, snap_cold = {}, {}

    HC.harness_rx_driver_writes.argtypes = [ctypes.c_int]

    def cnet_node(zc, flags, drv=1):
        gid = next(gids)
        L.cndp_node_gpu_umem_reset()
        if zc:
            L.cndp_node_gpu_umem_add(ctypes.c_void_p(pool.base), ctypes.c_uint64(pool.mem.nbytes))
        os.environ["CNDP_GPU_MQ_FLAGS"] = str(flags)
        assert HC.harness_graph_create(gid) == 0
        # the receive stub's data_len / data_off writes (xskdev.c:296-297), as
        # the CPU chain's receive does (oracle/cnet_chain.c walk)
        HC.harness_rx_driver_writes(drv)
        t = 0.0
        for p in range(passes + 1):  # pass 0 warms up
            pool.hdr[:] = hdr0
            HC.harness_rx_load(0, ptrs, nc)
            HC.harness_reset_counts()
            dt = HC.harness_walk_until(nc)
            if dt < 0:
                t = -1.0
                break
            if p == 0 and drv and not snap:
                snap.update({f: pool.hdr[f].copy() for f in cnet_fields})
            if p == 0 and not drv and not snap_cold:
                snap_cold.update({f: pool.hdr[f].copy() for f in cnet_fields})
            t += dt if p else 0.0
        HC.harness_rx_driver_writes(0)
        HC.harness_graph_destroy()
        os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
        return round(nc * passes / t / 1e6, 2) if t > 0 else None

    # interleaved, two rounds (box noise), the median reported and both kept;
    # host headers (the eth_rx node's default) against the device reading
    # them (CNDP_MQ_F_DEVICE_HEADERS: k_mq_cnet_hdr, one more launch and a
    # PCIe read per mbuf before the classify)
    cvars = [("eth_rx_node_zero_copy", lambda: cnet_node(True, 0)),
             ("eth_rx_node_zero_copy_device_headers", lambda: cnet_node(True, D)),
             ("eth_rx_node_staged", lambda: cnet_node(False, 0)),
             ("cold_eth_rx_node_zero_copy", lambda: cnet_node(True, 0, 0)),
             ("cold_eth_rx_node_zero_copy_device_headers", lambda: cnet_node(True, D, 0)),
             ("queue_zero_copy", lambda: cnet_queue(True, 0)),
             ("queue_zero_copy_device_headers", lambda: cnet_queue(True, D)),
             ("queue_staged", lambda: cnet_queue(False, 0))]
    rounds = {k: [] for k, _ in cvars}
    for _ in range(2):
        for k, fn in cvars:
            rounds[k].append(fn())
    for k, v in rounds.items():
        cn[k + "_Mpps"] = round(float(np.median(v)), 2) if all(v) else None
    cn["ab_rounds"] = rounds
    L.cndp_node_gpu_umem_reset()
    # the reference cnet chain on one core over the same mbufs (oracle/cnet_chain.c:
    # eth_rx -> ptype -> ip4_input / ip6_input per 256-mbuf walk, as the GPU
    # nodes replace them; no flow hash, as neither writes one)
    pool.hdr[:] = hdr0
    t4c, t6c = tuple(x.copy() for x in f4.image()), tuple(x.copy() for x in f6.image())
    cpus, _, _ = host_cpus()
    rx_len = hdr0["data_len"].copy()
    O.cnet_chain(ptrs, nc, rx_len, int(hdr0["data_off"][0]), t4c, t6c, cpus=cpus[:1])
    # every field the replaced nodes write, GPU eth_rx node (first pass) against the CPU chain
    cn["results_equal_cpu_chain"] = bool(snap) and all(np.array_equal(snap[f], pool.hdr[f]) for f in cnet_fields)
    cn["cold_results_equal_cpu_chain"] = bool(snap_cold) and all(np.array_equal(snap_cold[f], pool.hdr[f])
                                                                 for f in cnet_fields)
    cn["header_state"] = HEADER_STATE_NOTE + ("; queue_*: the cnet queue alone (harness_mq_drive), no receive, "
                                              "cold headers")
    pool.hdr[:] = hdr0
    t = O.cnet_chain(ptrs, nc, rx_len, int(hdr0["data_off"][0]), t4c, t6c, iters=passes, cpus=cpus[:1])
    pool.hdr[:] = hdr0
    cn["cpu_1core_Mpps"] = round(nc * passes / t / 1e6, 2)
    cn["cpu_chain"] = ("the reference cnet chain per 256-mbuf graph walk over the same pktmbuf_t pool, one "
                       "core (oracle/cnet_chain.c)")
    cn["mbufs"] = nc
    cn["frames"] = "IMIX 64/570/1500 7:4:1, IPv4+IPv6"
    res["cnet"] = cn
    # ---- C1: cndpfwd loopback, one 512-packet request clamped to two 256-bursts
    c1 = pktgen.cndpfwd_udp(512)
    pool = MbufPool(512)
    pool.fill(c1)
    ptrs = pool.ptrs(np.arange(512))
    H.harness_mq_latency.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16,
                                     ctypes.c_int, ctypes.c_void_p]
    lat = {}
    reps = 400
    # the queue's batch holds the whole request (one launch for both bursts);
    # batch 256 (a launch per burst) beside it
    for zc in (True, False):
        umem = None
        if zc:
            cl.host_register(pool.mem)
            umem = pool.base
        for batch in (512, 256):
            q = MbufQueue(cl, N.CNDP_MQ_MAC_SWAP, batch=batch, depth=2, umem=umem)
            us = np.zeros(reps)
            rc = H.harness_mq_latency(q.h, ptrs, 512, 256, reps, us.ctypes.data)
            q.close()
            key = ("gpu_zero_copy" if zc else "gpu_staged") + ("" if batch == 512 else "_batch256")
            lat[key] = ({"median_us": round(float(np.median(us[20:])), 1),
                         "p99_us": round(float(np.percentile(us[20:], 99)), 1)} if rc == 0 else None)
        if zc:
            cl.host_unregister(pool.mem)
    host = pool.mem.copy()
    t = time.perf_counter()
    for _ in range(reps):
        O.mac_swap(host, 512, stride=2048, data_off=256)
    lat["cpu_1core_us"] = round((time.perf_counter() - t) / reps * 1e6, 2)
    lat["request"] = ("512 packets, -b 512 clamped to 256 (parse-args.c:394-397): two bursts submitted to a "
                      "MAC-swap queue of batch 512 (one launch), depth 2")
    res["c1_loopback"] = lat
    cl.close()
    return res


def _lcore_run(cpus, nthreads, reset, walk, passes, post=None):
    """nthreads worker lcores, thread k pinned to cpus[k]: per pass every thread
    resets its own state (reset(k), untimed), then after a barrier runs
    walk(k) on its own graph / pool; the pass takes as long as its slowest
    thread.  Pass 0 warms up (post(k, 0) sees its results).  Returns the
    seconds of passes 1..passes (sum of the per-pass maxima)."""
    import threading
    bar = threading.Barrier(nthreads)
    secs = [[0.0] * (passes + 1) for _ in range(nthreads)]
    errs = []

    def lcore(k):
        try:
            os.sched_setaffinity(0, {cpus[k % len(cpus)]})  # this thread only (Linux)
        except OSError:
            pass
        try:
            for p in range(passes + 1):
                reset(k)
                bar.wait(timeout=300)
                t0 = time.perf_counter()
                if walk(k) is False:
                    raise RuntimeError(f"lcore {k}: walk failed")
                secs[k][p] = time.perf_counter() - t0
                if post:
                    post(k, p)
                bar.wait(timeout=300)
        except BaseException as ex:  # reported; the barrier must not wait forever
            errs.append(ex)
            bar.abort()

    th = [threading.Thread(target=lcore, args=(k,)) for k in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return sum(max(secs[k][p] for k in range(nthreads)) for p in range(1, passes + 1))


def node_lcores(dev, threads=(1, 2, 4, 8), m: int = 1 << 18, mc: int = 1 << 17, passes: int = 4) -> dict:
    """One graph per worker lcore, all on one GPU (l3fwd-graph fwd.c:205-236;
    cnet-graph cnet-graph.c:360): T host threads, each pinned to a core and
    walking its own graph over its own port's UMEM pool -- the GPU pktdev_rx
    node (l3fwd receive chain) and the GPU eth_rx node (cnet), one context and
    queue per graph -- beside the same node chains on the CPU, T pinned threads
    over the same pools (oracle/oracle.c orc_l3rx_chain_mbufs,
    oracle/cnet_chain.c).  The GPU nodes in three forms (the queue's frame and
    header access, CNDP_GPU_MQ_FLAGS / UMEM registration): device headers (the
    kernels read header and frame in place), host headers (the host reads the
    header, the kernel the frame), staged (the host copies the bytes the parse
    reads into pinned staging).  Rates are aggregate Mpps over the T pools
    (each pass as long as its slowest lcore); every pool's results are compared
    with the CPU chain's for every form at every T (results_equal_cpu_chain)."""
    import ctypes
    from cndp_amd import native as N
    from cndp_amd import pktgen
    from cndp_amd.fib import Fib, Fib6, NodeFib, cne_node_ip4_route_add, node_ip4_add_input, node_ip6_add_input
    from cndp_amd.mbuf import MbufPool
    from oracle import oracle as O
    cpus, _, quota = host_cpus()
    n_cpu = min(len(cpus), int(-(-quota // 1))) if quota else len(cpus)  # the CPU quota, in CPUs
    threads = [t for t in threads if t <= max(1, n_cpu)]
    tmax = max(threads)
    # lcore k on core cpus[k]: distinct physical cores spread over the L3 domains,
    # the same cores for the GPU and the CPU legs
    cpus = spread_cpus(cpus, tmax)
    L = N.lib()
    routes = pktgen.l3fwd_routes()
    D = N.CNDP_MQ_F_DEVICE_HEADERS

    def harness(name, cnet):
        H = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", name))
        H.harness_rx_load.argtypes = [ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint32]
        H.harness_walk_until.argtypes = [ctypes.c_uint64]
        H.harness_walk_until.restype = ctypes.c_double
        H.harness_clone.restype = ctypes.c_uint32
        H.harness_clone.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        H.harness_graph_new.restype = ctypes.c_void_p
        H.harness_graph_use.argtypes = [ctypes.c_void_p]
        H.harness_graph_free.argtypes = [ctypes.c_void_p]
        H.harness_graph_patterns.argtypes = [ctypes.c_void_p, ctypes.c_int]
        H.harness_rx_driver_writes.argtypes = [ctypes.c_int]
        if cnet:
            H.harness_eth_rx_port.argtypes = [ctypes.c_uint32, ctypes.c_uint16]
            H.harness_cnet_set.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        else:
            H.harness_pktdev_rx_port.argtypes = [ctypes.c_uint32, ctypes.c_uint16]
            H.harness_register_cls_node()
        H.harness_edges_reset()
        H.harness_drop_clones()
        return H

    def graphs_for(H, T, pats_of, gid0):
        gs = []
        for k in range(T):
            g = H.harness_graph_new()
            H.harness_graph_use(g)
            pats = [x.encode() for x in pats_of(k)]
            H.harness_graph_patterns((ctypes.c_char_p * len(pats))(*pats), len(pats))
            rc = H.harness_graph_create(gid0 + k)
            gs.append(g)
            if rc:
                H.harness_graph_use(None)
                graphs_free(H, gs)
                raise RuntimeError(f"graph create {rc}")
        H.harness_graph_use(None)
        return gs

    def graphs_free(H, gs):
        for g in gs:
            H.harness_graph_use(g)
            H.harness_graph_destroy()
            H.harness_graph_use(None)
            H.harness_graph_free(g)

    def umem(pools, on):
        L.cndp_node_gpu_umem_reset()
        if on:
            for p in pools:
                L.cndp_node_gpu_umem_add(ctypes.c_void_p(p.base), ctypes.c_uint64(p.mem.nbytes))

    def chain(H, pools, hdr0, ptrs, nn, pats_of, gid_base, fields, variants, cpu_walk, after_create=None):
        """Every GPU form, then the CPU chain, at every T; rates and checks."""
        res = {"gpu_Mpps": {v: {} for v, _, _ in variants}, "cpu_Mpps": {},
               "results_equal_cpu_chain": {v: {} for v, _, _ in variants}}
        for ti, T in enumerate(threads):
            snaps = {}
            for vi, (v, flags, zc) in enumerate(variants):
                umem(pools, zc)
                os.environ["CNDP_GPU_MQ_FLAGS"] = str(flags)
                # graph ids < 256: the GPU nodes keep per-graph state by id
                # (GPU_GRAPHS_MAX); a form's graphs are destroyed before the next
                gs = graphs_for(H, T, pats_of, gid_base + vi * tmax)
                os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
                if after_create:
                    after_create()

                def reset(k, gs=gs):
                    H.harness_graph_use(gs[k])
                    pools[k].hdr[:] = hdr0[k]
                    H.harness_rx_load(k, ptrs[k], nn)
                    H.harness_reset_counts()

                snap = snaps.setdefault(v, {})

                def post(k, p, snap=snap):
                    if p == 0:  # from a fresh graph (node state 0, as the CPU chain starts)
                        snap[k] = {f: pools[k].hdr[f].copy() for f in fields}

                try:
                    t = _lcore_run(cpus, T, reset, lambda k: H.harness_walk_until(nn) >= 0, passes, post)
                finally:
                    graphs_free(H, gs)
                res["gpu_Mpps"][v][T] = round(T * nn * passes / t / 1e6, 2)
            cres = {}

            def reset_cpu(k):
                pools[k].hdr[:] = hdr0[k]

            def post_cpu(k, p):
                if p == 0:
                    cres[k] = {f: pools[k].hdr[f].copy() for f in fields}

            t = _lcore_run(cpus, T, reset_cpu, cpu_walk, passes, post_cpu)
            res["cpu_Mpps"][T] = round(T * nn * passes / t / 1e6, 2)
            for v, _, _ in variants:
                res["results_equal_cpu_chain"][v][T] = all(np.array_equal(snaps[v][k][f], cres[k][f])
                                                           for k in range(T) for f in fields)
        best = {T: max(res["gpu_Mpps"][v][T] for v, _, _ in variants) for T in threads}
        res["gpu_best_Mpps"] = best
        res["gpu_best_over_cpu"] = {T: round(best[T] / res["cpu_Mpps"][T], 2) for T in threads}
        return res

    out = {"threads": threads, "mbufs_per_lcore": {"l3fwd": m, "cnet": mc}, "passes": passes, "burst": 256,
           "cpus": cpus[:tmax], "header_state": "driver-written (receive stub / oracle loops, xskdev.c:296-297)"}
    # ---- l3fwd-graph receive chain: the GPU pktdev_rx node per lcore
    HR = harness("librx_harness.so", False)
    NodeFib.fini()
    L.cndp_node_ip4_rewrite_reset()
    pools = []
    for k in range(tmax):
        p = MbufPool(m)
        p.fill(pktgen.packed_ipv4(m, routes=routes, seed=200 + k))
        pools.append(p)
        cid = HR.harness_clone(b"pktdev_rx", str(k).encode())
        assert HR.harness_pktdev_rx_port(cid, k) == 0
    hdr0 = [p.hdr.copy() for p in pools]
    ptrs = [p.ptrs(np.arange(m)) for p in pools]
    HR.harness_rx_driver_writes(1)
    tabs = []

    def l3_routes():
        for ip, d, nh in routes:
            cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
        if not tabs:
            tabs.append(tuple(x.copy() for x in NodeFib().image()))

    def l3_cpu(k):
        O.set_driver_writes(True)
        return O.l3rx_chain_mbufs(ptrs[k], m, tabs[0]) > 0

    try:
        l3 = chain(HR, pools, hdr0, ptrs, m, lambda k: ["ip4*", "pkt_cls", f"pktdev_rx-{k}"], 20,
                   ("packet_type", "udata64"),
                   (("device_headers", D, True), ("host_headers", 0, True),
                    ("device_headers_host_writeback", D | N.CNDP_MQ_F_HOST_WRITEBACK, True),
                    ("host_writeback", N.CNDP_MQ_F_HOST_WRITEBACK, True), ("staged", 0, False)), l3_cpu, l3_routes)
    finally:
        O.set_driver_writes(False)
        HR.harness_rx_driver_writes(0)
        HR.harness_drop_clones()
        HR.harness_pktdev_rx_ports_reset()
        L.cndp_node_gpu_umem_reset()
        NodeFib.fini()
    l3["node"] = ("GPU pktdev_rx node (cndp_amd/node/pktdev_rx_gpu.c): soft parse + pkt_cls + ip4_lookup in one "
                  "queue kernel (device_headers: the node's default); CPU: pktdev_rx's soft parse, pkt_cls and the "
                  "ip4_lookup loop per 256-burst (orc_l3rx_chain_mbufs)")
    out["l3fwd_rx_chain"] = l3
    del pools, ptrs, hdr0
    # ---- cnet: the GPU eth_rx node per lcore
    HC = harness("libcnet_harness.so", True)
    v6 = pktgen.v6_routes()
    f4 = Fib("lc4", N.CNE_FIB_DIR24_8, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_DIR24_8_4B, num_tbl8=256)
    for i, (ip, d, _) in enumerate(routes):
        node_ip4_add_input(f4, ip, d, i)
    f6 = Fib6("lc6", N.CNE_FIB_TRIE, default_nh=1025, max_routes=1024, nh_sz=N.CNE_FIB_TRIE_4B, num_tbl8=1 << 15)
    for ip, d, i in v6:
        node_ip6_add_input(f6, ip, d, i)
    HC.harness_cnet_set(f4.h, f6.h)
    t4c, t6c = tuple(x.copy() for x in f4.image()), tuple(x.copy() for x in f6.image())
    pools = []
    for k in range(tmax):
        p = MbufPool(mc)
        p.fill(pktgen.imix(mc, v4routes=routes, v6routes=v6, seed=300 + k))
        pools.append(p)
        cid = HC.harness_clone(b"eth_rx", str(k).encode())
        assert HC.harness_eth_rx_port(cid, k) == 0
    hdr0 = [p.hdr.copy() for p in pools]
    ptrs = [p.ptrs(np.arange(mc)) for p in pools]
    HC.harness_rx_driver_writes(1)

    def cnet_cpu(k):
        return O.cnet_chain(ptrs[k], mc, hdr0[k]["data_len"], int(hdr0[k]["data_off"][0]), t4c, t6c,
                            cpus=[cpus[k % len(cpus)]], lport=k) > 0

    try:
        cn = chain(HC, pools, hdr0, ptrs, mc, lambda k: [f"eth_rx-{k}", "ptype", "ip4_input", "ip6_input"], 140,
                   ("packet_type", "ol_flags", "tx_offload", "lport", "data_off", "data_len"),
                   (("host_headers", 0, True), ("device_headers", D, True),
                    ("host_writeback", N.CNDP_MQ_F_HOST_WRITEBACK, True), ("staged", 0, False)), cnet_cpu)
    finally:
        HC.harness_rx_driver_writes(0)
        HC.harness_drop_clones()
        HC.harness_eth_rx_ports_reset()
        L.cndp_node_gpu_umem_reset()
    cn["node"] = ("GPU eth_rx node (cndp_amd/node/eth_rx_gpu.c): eth_rx + ptype + ip4_input / ip6_input "
                  "(host_headers: the node's default); CPU: the cnet chain per 256-mbuf walk "
                  "(oracle/cnet_chain.c); IMIX")
    out["cnet_eth_rx"] = cn
    return out


def l3fwd_rx_chain(L, pool, ptrs, n, passes, routes):
    """l3fwd-graph's receive chain pktdev_rx -> pkt_cls -> ip4_lookup as the
    GPU pktdev_rx node runs it (cndp_amd/node/pktdev_rx_gpu.c, CNDP_MQ_F_RX_PARSE:
    the soft parse, pkt_cls and the lookup in one kernel over the mbufs where
    they lie; graph walks pull 256-mbuf bursts from the port and the mbufs
    leave on ip4_rewrite / pkt_drop), against the same three nodes' loops on
    one core over the same mbufs (oracle/oracle.c orc_l3rx_chain_mbufs)."""
    import ctypes
    from cndp_amd import native as N
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    from oracle import oracle as O
    HR = ctypes.CDLL(os.path.join(ROOT, "tests", "node_harness", "librx_harness.so"))
    HR.harness_rx_load.argtypes = [ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint32]
    HR.harness_pktdev_rx_port.argtypes = [ctypes.c_uint32, ctypes.c_uint16]
    HR.harness_walk_until.argtypes = [ctypes.c_uint64]
    HR.harness_walk_until.restype = ctypes.c_double
    HR.harness_register_cls_node()
    # edges copied into this harness by an earlier ip4_rewrite_set_next in the
    # process (the rx node's hook) would make the first runs fuse ip4_rewrite
    HR.harness_edges_reset()
    name = ctypes.create_string_buffer(64)
    fl, ne, e0, e1 = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_char_p(), ctypes.c_char_p()
    k = HR.harness_node_info(0, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
    rx_id = None
    for i in range(k):
        HR.harness_node_info(i, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
        if name.value == b"pktdev_rx":
            rx_id = i
    out = {}
    D = N.CNDP_MQ_F_DEVICE_HEADERS
    hdr0 = pool.hdr.copy()
    assert HR.harness_pktdev_rx_port(rx_id, 0) == 0
    HR.harness_rx_driver_writes.argtypes = [ctypes.c_int]
    # primary form: the receive stub writes every returned mbuf's data_len /
    # data_off as xskdev's receive does (xskdev.c:296-297), so the node sees
    # header lines dirty in this core's cache (pktdev_rx.c:107-125); cold_*:
    # without those writes.  Interleaved, two rounds, medians.
    variants = (("gpu_zero_copy", True, D, 1), ("gpu_zero_copy_host_headers", True, 0, 1), ("gpu_staged", False, 0, 1),
                ("cold_gpu_zero_copy", True, D, 0), ("cold_gpu_zero_copy_host_headers", True, 0, 0))
    ab = {v[0]: [] for v in variants}
    snaps = {}
    gid = 50
    for rnd in range(2):
        for key, zc, flags, drv in variants:
            L.cndp_node_gpu_umem_reset()
            if zc:
                L.cndp_node_gpu_umem_add(pool.base, pool.mem.nbytes)
            os.environ["CNDP_GPU_MQ_FLAGS"] = str(flags)
            gid += 1
            assert HR.harness_graph_create(gid) == 0
            os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
            for ip, d, nh in routes:
                cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
            HR.harness_rx_driver_writes(drv)
            t = 0.0
            for p in range(passes + 1):  # pass 0 warms up
                pool.hdr[:] = hdr0
                HR.harness_rx_load(0, ptrs, n)
                HR.harness_reset_counts()
                dt = HR.harness_walk_until(n)
                if dt < 0:
                    t = -1.0
                    break
                t += dt if p else 0.0
            HR.harness_rx_driver_writes(0)
            if rnd == 0 and key in ("gpu_zero_copy", "cold_gpu_zero_copy"):  # what the chain wrote into every mbuf
                snaps[key] = (pool.hdr["packet_type"].copy(), pool.hdr["udata64"].copy())
            HR.harness_graph_destroy()
            ab[key].append(n * passes / t / 1e6 if t > 0 else 0.0)
    for key, v in ab.items():
        out[key + "_Mpps"] = round(float(np.median(v)), 2) if min(v) > 0 else None
    out["ab_rounds"] = {k: [round(x, 2) for x in v] for k, v in ab.items()}
    # the same three nodes' loops on the CPU over the same (not yet rewritten)
    # frames: every mbuf's packet_type and node_mbuf_priv1 compared, for the
    # GPU chain's primary and cold forms
    pool.hdr[:] = hdr0
    t24c, t8c = (x.copy() for x in NodeFib().image())
    O.l3rx_chain_mbufs(ptrs, n, (t24c, t8c))
    for key, rk in (("gpu_zero_copy", "results_equal_cpu_chain"), ("cold_gpu_zero_copy", "cold_results_equal_cpu_chain")):
        snap = snaps.get(key)
        out[rk] = bool(snap is not None and np.array_equal(snap[0], pool.hdr["packet_type"]) and
                       np.array_equal(snap[1], pool.hdr["udata64"]))
        if snap is not None and not out[rk]:
            bad_pt = np.nonzero(snap[0] != pool.hdr["packet_type"])[0]
            bad_u = np.nonzero(snap[1] != pool.hdr["udata64"])[0]
            out[rk.replace("equal_cpu_chain", "mismatches")] = {
                "packet_type": int(bad_pt.size), "udata64": int(bad_u.size),
                "first": [int(i) for i in np.union1d(bad_pt, bad_u)[:4]],
                "gpu_udata64": [hex(int(snap[1][i])) for i in bad_u[:4]],
                "cpu_udata64": [hex(int(pool.hdr["udata64"][i])) for i in bad_u[:4]]}
    # the whole l3fwd-graph node chain on the device: the rx node chained into
    # the GPU ip4_rewrite node (four tx ports, 12-B MAC rewrites for the 64
    # next hops, as l3fwd-graph sets them up, fwd.c:160-201)
    import random
    HR.harness_chain.argtypes = [ctypes.c_int]
    HR.cne_node_edge_update.restype = ctypes.c_uint16
    HR.cne_node_edge_update.argtypes = [ctypes.c_uint32, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint16]
    HR.cne_node_edge_count.restype = ctypes.c_uint16
    HR.cne_node_edge_count.argtypes = [ctypes.c_uint32]
    rw_id = None
    for i in range(k):
        HR.harness_node_info(i, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
        if name.value == b"ip4_rewrite":
            rw_id = i
    L.cndp_node_ip4_rewrite_reset()
    tbl = np.zeros(64, dtype=O.REWRITE_NH)
    rnd = random.Random(8)
    try:
        for p in range(4):
            nm = ctypes.c_char_p(f"pktdev_tx-{p}".encode())
            HR.cne_node_edge_update(rw_id, 0xFFFF, ctypes.byref(nm), 1)
            assert L.ip4_rewrite_set_next(p, HR.cne_node_edge_count(rw_id) - 1) == 0
        for nh in range(64):
            data = bytes(rnd.randrange(256) for _ in range(12))
            assert L.cne_node_ip4_rewrite_add(nh, ctypes.create_string_buffer(data, 12), 12, nh % 4) == 0
            tbl[nh]["rewrite_len"], tbl[nh]["tx_node"], tbl[nh]["enabled"] = 12, nh % 4 + 1, 1
            tbl[nh]["rewrite_data"][:] = np.frombuffer(data + bytes(44), np.uint8)
        L.cndp_node_gpu_umem_reset()
        L.cndp_node_gpu_umem_add(pool.base, pool.mem.nbytes)
        HR.harness_chain(1)
        # ip4_rewrite in the receive node's kernel (CNDP_MQ_F_REWRITE, the
        # node's default zero-copy), or as the GPU ip4_rewrite node behind it;
        # driver-written headers (cold_*: without)
        for gid, (key, fuse) in enumerate((("gpu_with_rewrite_zero_copy", "1"),
                                           ("gpu_with_rewrite_node_zero_copy", "0"),
                                           ("cold_gpu_with_rewrite_zero_copy", "1"))):
            os.environ["CNDP_GPU_RX_REWRITE"] = fuse
            HR.harness_rx_driver_writes(0 if key.startswith("cold_") else 1)
            assert HR.harness_graph_create(70 + gid) == 0
            os.environ.pop("CNDP_GPU_RX_REWRITE", None)
            for ip, d, nh in routes:
                cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
            t = 0.0
            for p in range(passes + 1):  # pass 0 warms up
                pool.hdr[:] = hdr0
                HR.harness_rx_load(0, ptrs, n)
                HR.harness_reset_counts()
                dt = HR.harness_walk_until(n)
                if dt < 0:
                    t = -1.0
                    break
                t += dt if p else 0.0
            HR.harness_graph_destroy()
            out[key + "_Mpps"] = round(n * passes / t / 1e6, 2) if t > 0 else None
    finally:
        os.environ.pop("CNDP_GPU_RX_REWRITE", None)
        HR.harness_rx_driver_writes(0)
        HR.harness_chain(0)
        HR.harness_edges_reset()
        L.cndp_node_gpu_umem_reset()
    fib = NodeFib()
    t24, t8 = (x.copy() for x in fib.image())
    for pre, drv in (("", True), ("cold_", False)):
        O.set_driver_writes(drv)
        pool.hdr[:] = hdr0
        O.l3rx_chain_mbufs(ptrs, n, (t24, t8))
        t = O.l3rx_chain_mbufs(ptrs, n, (t24, t8), iters=passes)
        out[pre + "cpu_1core_Mpps"] = round(n * passes / t / 1e6, 2)
        pool.hdr[:] = hdr0
        O.l3rx_chain_mbufs(ptrs, n, (t24, t8), rewrite=tbl)
        t = O.l3rx_chain_mbufs(ptrs, n, (t24, t8), iters=passes, rewrite=tbl)
        out[pre + "cpu_1core_with_rewrite_Mpps"] = round(n * passes / t / 1e6, 2)
    O.set_driver_writes(False)
    out["header_state"] = HEADER_STATE_NOTE
    out["cpu_chain"] = ("pktdev_rx's soft parse, pkt_cls and the ip4_lookup node loop per 256-burst over the "
                        "same mbufs, one core (oracle/oracle.c orc_l3rx_chain_mbufs); _with_rewrite: then "
                        "ip4_rewrite_node_process over the mbufs ip4_lookup sent to it")
    pool.hdr[:] = hdr0
    L.cndp_node_ip4_rewrite_reset()
    NodeFib.fini()
    return out


def l3fwd_pair(H, L, pool, ptrs, n, burst, passes, routes):
    """GPU ip4_lookup + GPU ip4_rewrite nodes (tests/node_harness chained
    walks: pktdev_rx bursts -> ip4_lookup -> ip4_rewrite -> pktdev_tx-<port>)
    against the same two nodes' loops on one core (oracle/oracle.c
    orc_l3fwd_nodes_mbufs).  Four tx ports, 12-B MAC rewrites for the 64 next
    hops, as l3fwd-graph sets them up (fwd.c:160-201, pktdev_ctrl.c:75-86)."""
    import ctypes
    import random
    from cndp_amd import native as N
    from cndp_amd.fib import NodeFib, cne_node_ip4_route_add
    from oracle import oracle as O
    H.cne_node_edge_update.restype = ctypes.c_uint16
    H.cne_node_edge_update.argtypes = [ctypes.c_uint32, ctypes.c_uint16, ctypes.c_void_p, ctypes.c_uint16]
    H.cne_node_edge_count.restype = ctypes.c_uint16
    H.cne_node_edge_count.argtypes = [ctypes.c_uint32]
    H.harness_chain.argtypes = [ctypes.c_int]
    name = ctypes.create_string_buffer(64)
    fl, ne, e0, e1 = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_char_p(), ctypes.c_char_p()
    k = H.harness_node_info(0, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
    rw_id = None
    for i in range(k):
        H.harness_node_info(i, name, ctypes.byref(fl), ctypes.byref(ne), ctypes.byref(e0), ctypes.byref(e1))
        if name.value == b"ip4_rewrite":
            rw_id = i
    L.cndp_node_ip4_rewrite_reset()
    tbl = np.zeros(64, dtype=O.REWRITE_NH)
    rnd = random.Random(7)
    out = {}
    try:
        for p in range(4):
            nm = ctypes.c_char_p(f"pktdev_tx-{p}".encode())
            H.cne_node_edge_update(rw_id, 0xFFFF, ctypes.byref(nm), 1)
            assert L.ip4_rewrite_set_next(p, H.cne_node_edge_count(rw_id) - 1) == 0
        for nh in range(64):
            data = bytes(rnd.randrange(256) for _ in range(12))
            assert L.cne_node_ip4_rewrite_add(nh, ctypes.create_string_buffer(data, 12), 12, nh % 4) == 0
            tbl[nh]["rewrite_len"], tbl[nh]["tx_node"], tbl[nh]["enabled"] = 12, nh % 4 + 1, 1
            tbl[nh]["rewrite_data"][:] = np.frombuffer(data + bytes(44), np.uint8)
        H.harness_chain(1)
        # zero-copy default: ip4_lookup's queue runs ip4_rewrite too
        # (CNDP_MQ_F_REWRITE, mbufs straight to the pktdev_tx edges), lookup
        # headers on the device / on the host; then the GPU ip4_rewrite node
        # behind it (CNDP_GPU_LOOKUP_REWRITE=0) with the two queues' header
        # forms (lookup / rewrite): both on the device (the nodes' defaults),
        # the rewrite's on the host, both on the host; then staged
        # primary form: the receive driver's header writes before each burst
        # (harness_driver_writes, xskdev.c:296-297), cold_*: without them
        D = N.CNDP_MQ_F_DEVICE_HEADERS
        H.harness_driver_writes.argtypes = [ctypes.c_int]
        for gid, (key, zc, fl, frw, lrw) in enumerate((
                ("gpu_zero_copy", True, D, D, 1),
                ("gpu_zero_copy_lookup_host_headers", True, 0, D, 1),
                ("gpu_zero_copy_rewrite_node", True, D, D, 0),
                ("gpu_zero_copy_rewrite_node_rewrite_host_headers", True, D, 0, 0),
                ("gpu_zero_copy_rewrite_node_host_headers", True, 0, 0, 0),
                ("gpu_staged", False, 0, 0, 0),
                ("cold_gpu_zero_copy", True, D, D, 1))):
            L.cndp_node_gpu_umem_reset()
            if zc:
                L.cndp_node_gpu_umem_add(pool.base, pool.mem.nbytes)
            os.environ["CNDP_GPU_MQ_FLAGS"] = str(fl)
            os.environ["CNDP_GPU_RW_MQ_FLAGS"] = str(frw)
            os.environ["CNDP_GPU_LOOKUP_REWRITE"] = str(lrw)
            assert H.harness_graph_create(30 + gid) == 0
            os.environ.pop("CNDP_GPU_MQ_FLAGS", None)
            os.environ.pop("CNDP_GPU_RW_MQ_FLAGS", None)
            os.environ.pop("CNDP_GPU_LOOKUP_REWRITE", None)
            for ip, d, nh in routes:
                cne_node_ip4_route_add(ip, d, nh, N.IP4_LOOKUP_NEXT_REWRITE)
            H.harness_driver_writes(0 if key.startswith("cold_") else 1)
            H.harness_drive(b"ip4_lookup", ptrs, n, burst, 1)  # warm-up
            t = H.harness_drive(b"ip4_lookup", ptrs, n, burst, passes)
            H.harness_driver_writes(0)
            H.harness_graph_destroy()
            out[key + "_Mpps"] = round(n * passes / t / 1e6, 2) if t > 0 else None
        fib = NodeFib()
        t24, t8 = (x.copy() for x in fib.image())
        for key, drv in (("cpu_1core_Mpps", True), ("cold_cpu_1core_Mpps", False)):
            O.set_driver_writes(drv)
            O.l3fwd_nodes_mbufs(ptrs, n, (t24, t8), tbl, burst, 1)
            t = O.l3fwd_nodes_mbufs(ptrs, n, (t24, t8), tbl, burst, passes)
            out[key] = round(n * passes / t / 1e6, 2)
        O.set_driver_writes(False)
        out["header_state"] = HEADER_STATE_NOTE
        out["cpu_chain"] = ("ip4_lookup's loop then ip4_rewrite_node_process per 256-burst over the same "
                            "mbufs, one core (oracle/oracle.c orc_l3fwd_nodes_mbufs)")
        out["gpu_paths"] = ("gpu_zero_copy*: ip4_rewrite run by ip4_lookup's queue (CNDP_MQ_F_REWRITE, "
                            "the default with registered UMEM); *_rewrite_node*: the GPU ip4_rewrite node "
                            "behind the GPU ip4_lookup node (CNDP_GPU_LOOKUP_REWRITE=0)")
    finally:
        H.harness_chain(0)
        H.harness_edges_reset()
        L.cndp_node_gpu_umem_reset()
        L.cndp_node_ip4_rewrite_reset()
        NodeFib.fini()
    return out


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
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); N > 1 without torchrun's env starts them (launch_ranks)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=0, help="override packets per GPU")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe) rates")
    ap.add_argument("--sweep", action="store_true", help="time every kernel variant (stderr + gpurun_out)")
    ap.add_argument("--extra", default="c2,c4,c5",
                    help="other configs measured after the headline (comma list, '' = none)")
    ap.add_argument("--no-imix", action="store_true", help="same as --extra ''")
    ap.add_argument("--no-node", action="store_true", help="skip the pktmbuf node-boundary rates")
    ap.add_argument("--no-probe", action="store_true", help="skip the same-box access-shape probes")
    ap.add_argument("--frame-mem", default="default", choices=["default", "torch", "uncached", "cached"],
                    help="frame slabs: torch (hipMalloc) tensors or cndp_gpu_frames_alloc memory; "
                         "default = FRAME_MEM per config")
    ap.add_argument("--in-route-frac", type=float, default=0.9,
                    help="share of DIPs inside the route set (SURVEY §8(d): 0.9)")
    ap.add_argument("--ring", type=int, default=0,
                    help="batches in the ring (0 = auto: >= 4 GiB of frames + results, at most 4)")
    ap.add_argument("--load-nt", type=int, default=None)
    ap.add_argument("--cnet-tile", type=int, default=None)
    ap.add_argument("--cnet-spec", type=int, default=None)
    ap.add_argument("--spec-scan", type=int, default=None)
    ap.add_argument("--spec-lists", type=int, default=None)
    ap.add_argument("--spec-types", type=int, default=None)
    ap.add_argument("--stream-bal", type=int, default=None)
    ap.add_argument("--tile", type=int, default=None)
    ap.add_argument("--dir16", type=int, default=None)
    ap.add_argument("--nt", type=int, default=None)
    ap.add_argument("--unroll", type=int, default=None)
    ap.add_argument("--bpc", type=int, default=None)
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and args.gpus is not None and args.gpus != int(env_world):
        sys.exit(f"--gpus {args.gpus} but torchrun started {env_world} ranks")
    if args.frame_mem != "default":
        for k in FRAME_MEM:
            FRAME_MEM[k] = None if args.frame_mem == "torch" else args.frame_mem
    if args.no_imix:
        args.extra = ""

    from cndp_amd import dist as D
    world, rank, local = setup_dist()
    dev = torch.device(f"cuda:{local}")
    if rank == 0:
        import torch.distributed as tdist
        if tdist.is_initialized():
            log(f"[bench] process group: {tdist.get_backend()}, world {tdist.get_world_size()}")
    t0 = time.time()
    st = build_state(args.config, dev, rank, args.packets or None, args.in_route_frac, args.ring)
    torch.cuda.synchronize()
    if rank == 0:
        log(f"[bench] setup {time.time() - t0:.1f}s: {st['desc']}")
    cl, fr, out, mode = st["cl"], st["frames"], st["out"], st["mode"]
    stream = torch.cuda.current_stream(dev)
    cl.set_tuning(nt=args.nt, unroll=args.unroll, blocks_per_cu=args.bpc, tile=args.tile, dir16=args.dir16,
                  load_nt=args.load_nt, cnet_tile=args.cnet_tile, cnet_spec=args.cnet_spec,
                  spec_scan=args.spec_scan, spec_lists=args.spec_lists, spec_types=args.spec_types,
                  stream_bal=args.stream_bal)
    if args.sweep and rank == 0:
        sweep(st, stream, args.config)

    for k in range(args.warmup):
        run_step(st, None, k)
    torch.cuda.synchronize()
    parity = None
    parity_all = None
    if rank == 0 and not args.no_parity:
        parity = parity_sample(st)
        log(f"[bench] parity sample vs oracle: {parity}")
        parity_all = parity_full(st)
        log(f"[bench] full batch vs oracle: {parity_all}")
        run_step(st, None, 0)  # the checks restarted the cnet node model: settle it untimed
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
    probe = None
    if rank == 0 and not args.no_probe and args.config != "c3rw":
        try:
            probe = probe_ceiling(st, stream, args.steps, kern_ms)
            log(f"[bench] same-box probe: {probe}")
        except Exception as ex:  # reported, never fatal for the headline line
            probe = {"probe_error": repr(ex)}

    n = st["n"]
    total_pkts = n * world * args.steps
    value = total_pkts / elapsed / 1e6
    achieved = st["algo"] * n / (kern_ms * 1e-3) / 1e9
    bins = out["bins"].cpu().numpy()
    layout = ("packed 64-B slots" if fr.offsets is None and fr.stride == 64
              else ("IMIX packed at roundup(len,64)" if fr.offsets is not None else f"{fr.stride}-B slots"))
    ring_len = len(st["ring"])
    cpu = e2e = nb = fu = None
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline and args.config != "c3rw":
            cpu = cpu_baseline(st, args.cpu_budget)
        if not args.no_e2e and args.config != "c3rw":
            try:
                e2e = {"packed_slab": e2e_host(st)}
                if args.config in ("c2", "c3"):
                    # the AF_XDP UMEM layout: 2 KiB frames, data at +256 (pktmbuf.c:60-80)
                    from cndp_amd import pktgen
                    um = pktgen.umem_ipv4(1 << 22, routes=st["routes"], seed=5, device=dev)
                    e2e["umem_2KiB_frames"] = e2e_host(st, frames=um)
                    e2e["umem_2KiB_frames"]["packets"] = um.n
                    del um
                log(f"[bench] host-memory rates: {e2e}")
            except Exception as ex:  # reported, never fatal for the headline line
                e2e = {"error": repr(ex)}
    extra = {}
    todo = [c for c in args.extra.split(",") if c and c != args.config] if args.config in ("c2", "c3") else []
    if todo:  # every rank (max over ranks inside)
        del st["ring"], fr, out
        st.pop("frames", None)
        torch.cuda.empty_cache()
    for c in todo:
        try:
            extra[c] = config_line(c, dev, rank, world, max(5, args.steps // 2), args.warmup, not args.no_parity,
                                   not args.no_cpu_baseline, min(args.cpu_budget, 5.0), not args.no_probe)
            if rank == 0:
                log(f"[bench] {c} line: {extra[c]}")
        except Exception as ex:  # reported, never fatal for the headline line
            extra[c] = {"error": repr(ex)}
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_node:
        try:
            nb = node_boundary(dev)
            log(f"[bench] node boundary: {nb}")
        except Exception as ex:  # reported, never fatal for the headline line
            nb = {"error": repr(ex)}
        try:
            nb_lc = node_lcores(dev)
            log(f"[bench] node lcores: {nb_lc}")
        except Exception as ex:  # reported, never fatal for the headline line
            nb_lc = {"error": repr(ex)}
        if isinstance(nb, dict):
            nb["lcore_graphs"] = nb_lc
        try:
            fu = fib_update()
            log(f"[bench] fib update: {fu}")
        except Exception as ex:  # reported, never fatal for the headline line
            fu = {"error": repr(ex)}
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
                       "frame_layout": layout, "frame_memory": frame_mem_name(args.config),
                       "ring_batches": ring_len,
                       "routes": len(st["routes"]), "parallelism": f"dp{world} (replicated FIB, sharded batches)",
                       "parity_sample_vs_oracle": parity, "parity_full_batch_vs_oracle": parity_all,
                       "bins_total": int(bins.sum())},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(args.config),
                         "kernel_ms": round(kern_ms, 5),
                         "algorithmic_bytes_per_pkt": st["algo"], **(probe or {})},
            "cpu_baseline": cpu,
            "configs": extra,
            "node_boundary": nb,
            "host_memory_e2e": e2e,
            "fib_update": fu,
        }
        print(json.dumps(res), flush=True)
    import torch.distributed as tdist
    if tdist.is_initialized():
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
