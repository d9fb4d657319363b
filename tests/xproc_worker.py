"""One rank of a cross-process row-partitioned classification (tests/test_xproc.py).

Launched as a child process per rank (RANK / WORLD_SIZE / MASTER_* in the environment), never
exec'd from a process that touched the GPU.  Each rank creates ONE partitioned context on
device 0 whose per-superstep delta all-gather runs through the caller's transport
(EL_XCHG_HOST) over torch.distributed gloo — the exchange protocol of SURVEY.md §8(e) across
real process boundaries, as one context per GPU does under RCCL (CommunicationHandler.java:49-84
is the barrier it replaces).  The rank writes its rows to OUT/rank<r>.npz; the test merges them.

usage: xproc_worker.py WORKLOAD SCALE COPIES OUT
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    name, scale, copies, out = sys.argv[1], float(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import numpy as np
    import torch.distributed as dist

    from distel_amd import engine, generators, ir

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group(backend="gloo")
    base = generators.workload(name, scale)
    ax = ir.replicate(base, copies) if copies > 1 else base
    if copies == world:  # partitions aligned with the OntologyMultiplier copies (configs[3])
        rows = ir.copy_slice(base, copies, rank)
        if rank == 0:
            rows = (0, rows[1])  # ⊥ and ⊤ live on rank 0
    else:
        rows = (0, 0)  # the equal split
    eng = engine.Engine(device=0, partition=engine.Partition(rank, world, engine.XCHG_HOST, rows=rows,
                                                             allgather=engine.gloo_allgather()))
    eng.load(ax)
    eng.init()
    st = eng.saturate()
    x, a = eng.facts()
    lx, lr, ly = eng.links()
    np.savez(os.path.join(out, f"rank{rank}.npz"), x=x, a=a, lx=lx, lr=lr, ly=ly)
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(dict(st), f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
