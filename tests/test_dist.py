"""world_size-2 gloo rehearsal of the multi-GPU path on CPU: each rank
classifies its own contiguous shard (here with the oracle standing in for
the device, since this container has no GPU), then the per-bin counters are
all-reduced once; the result must equal the counters of the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    from cndp_amd import dist as D
    from cndp_amd import pktgen
    from oracle import oracle as O
    import helpers
    w, r, _ = D.init_from_env("gloo")
    assert (w, r) == (world, rank)
    vals = [(ip, d, nh) for ip, d, nh in pktgen.l3fwd_routes()]
    t4 = O.dir24_8_build(vals, helpers.L3FWD_DEF, 256)
    lo, hi = D.shard(n, rank, world)
    fr = pktgen.packed_ipv4(n, routes=pktgen.l3fwd_routes())
    slab = fr.slab.numpy()[lo * 64: hi * 64]
    out = O.classify(O.MODE_L3FWD, slab, hi - lo, stride=64, tables4=t4)
    bins = torch.from_numpy(out["bins"].astype(np.int64))
    D.final_count_reduce(bins)
    mx = D.max_over_ranks([float(rank)], "cpu")
    if rank == 0:
        q.put((bins.numpy().copy(), mx))
    torch.distributed.destroy_process_group()


def test_two_rank_count_reduce():
    n = 40000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in ps:
        p.start()
    bins, mx = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    from cndp_amd import pktgen
    from oracle import oracle as O
    import helpers
    vals = [(ip, d, nh) for ip, d, nh in pktgen.l3fwd_routes()]
    t4 = O.dir24_8_build(vals, helpers.L3FWD_DEF, 256)
    fr = pktgen.packed_ipv4(n, routes=pktgen.l3fwd_routes())
    full = O.classify(O.MODE_L3FWD, fr.slab.numpy(), n, stride=64, tables4=t4)
    assert np.array_equal(bins.astype(np.uint64), full["bins"])
    assert mx == [1.0]


def test_shard_covers_everything():
    from cndp_amd.dist import shard
    for n in (0, 1, 7, 1000, 16777216):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            for (a, b), (c, d) in zip(parts, parts[1:]):
                assert b == c and a <= b


@pytest.mark.gpu
def test_rccl_one_rank_bench():
    """The bench's distributed path over RCCL ("nccl") on the one GPU a box
    has: torchrun with one rank and CNDP_DIST_FORCE=1, so the process group
    exists and the count reduce and the max over ranks are real RCCL
    all-reduces (identities at one rank).  The bins must still count every
    frame of every timed step."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n, steps = 1 << 20, 3
    env = dict(os.environ, CNDP_DIST_FORCE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--config", "c3",
           "--packets", str(n), "--steps", str(steps), "--warmup", "1", "--no-e2e", "--no-cpu-baseline",
           "--no-parity", "--no-imix", "--no-node", "--no-probe", "--ring", "1"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [s for s in r.stdout.splitlines() if s.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    assert rec["config"]["bins_total"] == n * steps
    assert "process group: nccl, world 1" in r.stderr


# ---- bench.py --gpus N: the ranks started by the bench itself ---------------
def _bench():
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    return importlib.import_module("bench")


def test_gpus_flag_reaches_launcher(monkeypatch):
    """`python bench.py --gpus 4 ...` with no torchrun environment hands the
    whole argument list to launch_ranks (which starts the ranks as a child
    torchrun) and exits with its status; with torchrun's environment the
    flag must match the world size."""
    import sys
    B = _bench()
    seen = {}

    def fake(n, argv):
        seen["n"], seen["argv"] = n, list(argv)
        return 7

    monkeypatch.setattr(B, "launch_ranks", fake)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    argv = ["--gpus", "4", "--steps", "2", "--config", "c3"]
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    with pytest.raises(SystemExit) as ex:
        B.main()
    assert ex.value.code == 7 and seen == {"n": 4, "argv": argv}
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as ex:
        B.main()
    assert "torchrun started 2 ranks" in str(ex.value.code)


def test_rank_launch_cmd_and_line_check():
    import json
    import sys
    B = _bench()
    cmd = B.rank_launch_cmd(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")
    good = {"n_gpus": 2, "steps": 3, "config": {"packets_per_gpu": 100, "bins_total": 600}}
    assert B.check_rank_line(json.dumps(good), 2)["n_gpus"] == 2
    for bad in ({**good, "n_gpus": 1}, {**good, "config": {"packets_per_gpu": 100, "bins_total": 300}}):
        with pytest.raises(ValueError):
            B.check_rank_line(json.dumps(bad), 2)


def test_launch_ranks_refuses_too_few_devices(monkeypatch):
    """RCCL needs a device per rank: fewer visible devices than --gpus is an
    error unless CNDP_DIST_BACKEND=gloo (ranks sharing a device)."""
    B = _bench()
    monkeypatch.setattr(B.torch.cuda, "device_count", lambda: 1)
    monkeypatch.delenv("CNDP_DIST_BACKEND", raising=False)
    assert B.launch_ranks(2, ["--gpus", "2"]) == 2


_FAKE_RANK = r'''
import json, os, torch.distributed as dist
dist.init_process_group("gloo")
w, r = dist.get_world_size(), dist.get_rank()
if r == 0:
    print("progress from rank 0", flush=True)
    print(json.dumps({"n_gpus": w, "steps": 2, "config": {"packets_per_gpu": 10, "bins_total": BINS}}), flush=True)
dist.destroy_process_group()
'''


@pytest.mark.parametrize("bins,rc", [(40, 0), (20, 1)])
def test_launch_ranks_runs_torchrun_child(monkeypatch, tmp_path, capsys, bins, rc):
    """The launcher end to end on CPU with a stand-in rank script (gloo, two
    ranks): rank 0's JSON line is printed once, after the check; a line whose
    bin counters miss a rank's packets fails the launch."""
    import sys
    B = _bench()
    script = tmp_path / "rank.py"
    script.write_text(_FAKE_RANK.replace("BINS", str(bins)))
    monkeypatch.setenv("CNDP_DIST_BACKEND", "gloo")
    monkeypatch.setattr(B, "rank_launch_cmd", lambda n, argv, port: [
        sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
        "--master-addr=127.0.0.1", f"--master-port={port}", str(script)])
    assert B.launch_ranks(2, []) == rc
    cap = capsys.readouterr()
    assert "progress from rank 0" in cap.err and "progress" not in cap.out
    assert cap.out.count('"n_gpus": 2') == (1 if rc == 0 else 0)
    assert len(cap.out.splitlines()) == (1 if rc == 0 else 0)   # stdout: the JSON line alone


@pytest.mark.gpu
def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` on the one-GPU box, ranks sharing the device over
    gloo (CNDP_DIST_BACKEND=gloo): the bench starts both ranks itself, and the
    line reports two GPUs and every packet of both ranks' timed steps."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n, steps = 1 << 20, 3
    env = dict(os.environ, CNDP_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--config", "c3", "--packets", str(n), "--steps", str(steps),
           "--warmup", "1", "--no-e2e", "--no-cpu-baseline", "--no-parity", "--no-imix", "--no-node", "--no-probe",
           "--ring", "1"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]   # the JSON line alone
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    assert rec["config"]["bins_total"] == 2 * n * steps
    assert "process group: gloo, world 2" in r.stderr
