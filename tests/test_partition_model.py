"""CPU checks of the row-partition exchange protocol (oracle/partition_model.py), the
protocol the HIP engine runs with el_config.exchange != NONE:
in-process ranks against the naive fixpoint and the KATs, and a world-size-2 gloo run in
which the all-gather really crosses processes."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

import kat
import naive
import partition_model as pm
from distel_amd import generators

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("path", kat.kat_files(), ids=lambda p: os.path.basename(p))
def test_kat_partition_model(path):
    ax, exp = kat.load_kat(path)
    for parts in (1, 2, 3):
        S, R, _ = pm.saturate_inprocess(ax, min(parts, ax.n_concepts), compat_range=False)
        kat.check(exp, S, R)


def test_partition_model_equals_naive():
    for seed in range(200):
        ax = generators.random_small(seed, n=6 + seed % 34, n_roles=1 + seed % 4)
        S0, R0 = naive.saturate(ax, distel_range=True)  # the model's own (DistEL) range rule
        for parts in (2, 3, 5):
            S, R, _ = pm.saturate_inprocess(ax, min(parts, ax.n_concepts))
            assert S == S0 and R == R0, (seed, parts)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, seeds, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch.distributed as dist
    import partition_model as pm
    from distel_amd import generators
    dist.init_process_group("gloo")

    def allgather(obj):
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out
    res = []
    for seed in seeds:
        ax = generators.random_small(seed, n=30, n_roles=3)
        lo, hi = pm.ranges(ax.n_concepts, world)[rank]
        r = pm.Rank(ax, lo, hi)
        steps = pm.run(r, allgather)
        res.append((seed, steps, {x: sorted(v) for x, v in r.S.items()}, sorted(r.links)))
    q.put((rank, res))
    dist.destroy_process_group()


def test_partition_model_gloo_two_ranks():
    world, seeds = 2, list(range(300, 312))
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seeds, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, seed in enumerate(seeds):
        ax = generators.random_small(seed, n=30, n_roles=3)
        S0, R0 = naive.saturate(ax, distel_range=True)
        S, R = {}, set()
        steps = set()
        for rank in range(world):
            s, st, rows, links = out[rank][i]
            assert s == seed
            steps.add(st)
            S.update({x: set(v) for x, v in rows.items()})
            R |= set(links)
        assert len(steps) == 1          # every rank stops at the same superstep
        assert S == S0 and R == R0, seed


def test_partition_model_aligned_copies_send_nothing():
    """OntologyMultiplier copies on ranks aligned with them: no record is routed to another
    rank (no other window holds a copy's concepts) — the exchange carries the counts only —
    and the union is still the naive closure of the whole ×k ontology."""
    from distel_amd import ir
    aligned = 0
    for seed in range(120):
        if aligned >= 6:
            break
        base = generators.random_small(500 + seed, n=12 + seed % 20, n_roles=1 + seed % 3)
        k = 3
        ax = ir.replicate(base, k)
        bounds = [ir.copy_slice(base, k, i) for i in range(k)]
        bounds[0] = (0, bounds[0][1])
        rs = [pm.Rank(ax, lo, hi) for lo, hi in bounds]
        wins = [(r.lo, r.hi, r.win) for r in rs]
        for r in rs:
            r.set_windows(wins)
        # (a base with axioms on ⊤ — ⊤ ⊑ C — puts every copy's C into every row: those copies are
        # not disjoint, and their windows overlap)
        disjoint = all(w[1] <= v[0] or v[1] <= w[0] for i, (_, _, w) in enumerate(wins) for _, _, v in wins[i + 1:])
        aligned += disjoint
        while True:
            out = [r.step() for r in rs]
            for o in out:
                if disjoint:  # (⊥ / ⊤-keyed records are in every window: the copies share them)
                    assert all(p[0][1] < 2 for p in o["props"]) and all(a[0] < 2 for a in o["acts"]), seed
                    assert all(x[0] < 2 for x in o["xlinks"]), seed
            if [r.absorb(out) for r in rs][0] == 0:
                break
        S, R = {}, set()
        for r in rs:
            S.update(r.S)
            R |= r.links
        S0, R0 = naive.saturate(ax, distel_range=True)
        assert S == S0 and R == R0, seed
    assert aligned >= 6, aligned
