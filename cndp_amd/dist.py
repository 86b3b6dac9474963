"""Multi-GPU plumbing: bursts shard across ranks with no data-path collective;
the only exchange is one final all-reduce of the per-bin counters (next-hop /
output-port counts, <= CNDP_BINS_MAX + 2 u64) over RCCL ("nccl" backend on
ROCm, xGMI) -- or gloo on CPU for tests.  One process per GPU.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise the process group from torchrun's env; returns (world, rank, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CNDP_DIST_FORCE=1: a process group (and so the collectives) at one rank
    # too -- RCCL exercised on a one-GPU box (tests/test_dist.py)
    force = os.environ.get("CNDP_DIST_FORCE") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def shard(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) packet range of this rank (host-side burst split)."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def final_count_reduce(bins: torch.Tensor) -> torch.Tensor:
    """Sum the per-bin counters of every rank in place (one collective)."""
    if dist.is_initialized():
        dist.all_reduce(bins, op=dist.ReduceOp.SUM)
    return bins


def max_over_ranks(values: list[float], device) -> list[float]:
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]
