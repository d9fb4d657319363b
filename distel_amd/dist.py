"""Multi-process orchestration for weak scaling (one process per GPU).

DistEL scales by giving every rule type its own processes and sharding keys by
Murmur hash across Redis instances, with an all-to-all "anything new?" barrier per
iteration (``kc/controller/CommunicationHandler.java:49-84``).  The MI355X path
scales the *concept space*: rank i owns a disjoint copy of the ontology
(OntologyMultiplier ×N semantics, ``kc/samples/OntologyMultiplier.java:44-83``),
saturates it on its own GPU, and the ranks only meet for the barrier and the
max-over-ranks timing — there is no data-path collective because the copies share
no concepts.  ``torch.distributed`` (RCCL under the ``nccl`` backend on ROCm,
``gloo`` on CPU) carries those two reductions.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, Optional, Tuple


@dataclass
class Ranks:
    rank: int
    world: int
    local: int
    dist: Optional[object]   # torch.distributed module when world > 1
    device: object           # torch.device used for the reductions


def init_from_env(prefer_nccl: bool = True) -> Ranks:
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    has_cuda = torch.cuda.is_available()
    if has_cuda:  # more ranks than GPUs (a rehearsal on a 1-GPU box) share the cards round-robin
        local = local % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local) if has_cuda else torch.device("cpu")
    if world <= 1:
        return Ranks(rank, 1, local, None, dev)
    import torch.distributed as dist
    # EL_DIST_BACKEND=gloo: the barrier and the two reductions over gloo (RCCL refuses two
    # ranks on one GPU, which a 1-GPU rehearsal of the N-rank launch needs)
    backend = os.environ.get("EL_DIST_BACKEND") or ("nccl" if (prefer_nccl and has_cuda) else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return Ranks(rank, world, local, dist, dev)


def barrier_sync(rk: Ranks) -> None:
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if rk.dist is not None:
        rk.dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def allreduce(rk: Ranks, value: float, op: str = "max") -> float:
    if rk.dist is None:
        return value
    import torch
    dt = torch.float64 if isinstance(value, float) else torch.int64
    t = torch.tensor([value], dtype=dt, device=rk.device)
    rk.dist.all_reduce(t, op={"max": rk.dist.ReduceOp.MAX, "sum": rk.dist.ReduceOp.SUM}[op])
    return t.item()


def run_weak(rk: Ranks, classify: Callable[[], dict], steps: int, warmup: int,
             drain: Optional[Callable[[], None]] = None) -> Tuple[float, int, dict]:
    """Warm up, then time exactly ``steps`` classifications between barriers.  ``drain`` waits
    for work a classification left in flight (asynchronous copy-backs); it runs inside the
    timed region, before the closing barrier.
    Returns (max-over-ranks seconds, derived axioms summed over ranks per step, last stats)."""
    st = {}
    for _ in range(warmup):
        st = classify()
    if drain:
        drain()
    barrier_sync(rk)
    t0 = time.perf_counter()
    for _ in range(steps):
        st = classify()
    if drain:
        drain()
    barrier_sync(rk)
    elapsed = time.perf_counter() - t0
    t_max = float(allreduce(rk, float(elapsed), "max"))
    derived = int(allreduce(rk, int(st["derived"]), "sum"))
    return t_max, derived, st


def gather_objects(rk: Ranks, obj) -> list:
    """Every rank's ``obj`` (picklable), in rank order, on every rank."""
    if rk.dist is None:
        return [obj]
    out = [None] * rk.world
    rk.dist.all_gather_object(out, obj)
    return out


def shutdown(rk: Ranks) -> None:
    if rk.dist is not None and rk.dist.is_initialized():
        rk.dist.destroy_process_group()
