"""World-size-2 gloo run of the weak-scaling orchestration (CPU).  The GPU engine is not
available here, so each rank's classification is the CPU oracle standing in for
el_saturate; what is tested is the N>1 plumbing bench.py uses: rendezvous, barrier,
max-over-ranks timing and the derived-axiom sum over disjoint copies."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, pipelined):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    from distel_amd import dist as D
    from distel_amd import generators
    rk = D.init_from_env(prefer_nccl=False)
    ax = generators.workload("g1", scale=0.02)
    pool = ThreadPoolExecutor(max_workers=1)
    pending, landed = [], []

    def copy_back(o):  # stands in for an EL_RESULT_ASYNC copy-back on a helper thread
        landed.append(len(o.facts()[0]))
        o.close()

    def classify():
        o = oracle.saturate(ax, 0)
        st = o.stats()
        if pipelined:  # bench.py's two-in-flight schedule: the copy-back lands later
            pending.append(pool.submit(copy_back, o))
        else:
            o.close()
        return st

    def drain():
        for f in pending:
            f.result()
        pending.clear()
    t_max, derived, st = D.run_weak(rk, classify, steps=2, warmup=1, drain=drain if pipelined else None)
    # every classification's copy-back landed inside run_weak (warm-up and timed steps)
    assert not pipelined or (not pending and len(landed) == 3 and set(landed) == {st["s_facts"]})
    q.put((rank, t_max, derived, st["derived"]))
    pool.shutdown()
    D.shutdown(rk)


@pytest.mark.parametrize("pipelined", [False, True])
def test_weak_scaling_two_ranks_gloo(pipelined):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, pipelined)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    t0, t1 = res[0][1], res[1][1]
    assert t0 == t1 > 0                          # every rank reports the same max-over-ranks time
    assert res[0][2] == res[1][2] == world * res[0][3]   # Σ derived over the disjoint copies
