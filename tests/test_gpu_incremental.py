"""GPU: incremental classification.  An ontology split into a base
and increments, classified base-first with el_add_axioms in between, must reach exactly the
closure the CPU oracle computes from scratch on the union (size-independent property: the
least fixpoint does not depend on the order axioms arrive in), while the first superstep after
an increment re-triggers only what the new axioms reach (test_increment_is_a_delta).  The random ontologies carry
range axioms, so these runs read ranges DistEL's way (EL_FLAG_COMPAT_DISTEL_RANGE): increments
are refused with ELK range fillers (test_increment_rejects_elk_ranges)."""
import numpy as np
import pytest

import kat
from distel_amd import engine, generators
from distel_amd.ir import Axioms

pytestmark = pytest.mark.gpu


def _split(ax: Axioms, parts: int, seed: int, grow: bool):
    """parts increments of ax; with grow, increment k only mentions concept ids below a
    rising cut (the id space extends as increments arrive)."""
    rng = np.random.default_rng(seed)
    fam = {k: getattr(ax, k) for k in ("sub", "ex_rhs", "ex_lhs", "subrole", "chain", "domain", "range")}
    conj = [(ax.conj_ops[ax.conj_ptr[i]:ax.conj_ptr[i + 1]].tolist(), int(ax.conj_b[i])) for i in range(ax.n_conj)]
    cols = {"sub": (0, 1), "ex_rhs": (0, 2), "ex_lhs": (1, 2), "subrole": (), "chain": (), "domain": (1,), "range": (1,)}
    cuts = sorted(rng.integers(2, ax.n_concepts + 1, parts - 1).tolist()) + [ax.n_concepts] if grow else \
        [ax.n_concepts] * parts
    owner = {}
    for k, a in fam.items():  # the first part whose cut covers the axiom's concepts, then random later
        need = a[:, list(cols[k])].max(axis=1) if len(cols[k]) and len(a) else np.zeros(len(a), np.int64)
        first = np.searchsorted(np.array(cuts), need, side="right") if grow else np.zeros(len(a), np.int64)
        owner[k] = np.maximum(first, rng.integers(0, parts, len(a)))
    conj_need = [max(ops + [b]) for ops, b in conj]
    conj_owner = [max(int(np.searchsorted(np.array(cuts), m, side="right")) if grow else 0, int(rng.integers(0, parts)))
                  for m in conj_need]
    out = []
    for q in range(parts):
        n = cuts[q]
        out.append(Axioms.build(n, ax.n_roles, kind=ax.kind[:n],
                                conj=[c for c, o in zip(conj, conj_owner) if o == q],
                                **{k: a[owner[k] == q] for k, a in fam.items()}))
    return out


def _check(ax, pieces, oracle_lib):
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(pieces[0])
    eng.init()
    eng.saturate()
    for inc in pieces[1:]:
        eng.add_axioms(inc)
        st = eng.saturate()
    o = oracle_lib.saturate(ax, 0, compat_range=True)
    gx, ga = eng.facts()
    ox, oa = o.facts()
    assert np.array_equal(gx, ox) and np.array_equal(ga, oa), "S(X) differs from the from-scratch closure"
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c), "R(r) differs from the from-scratch closure"
    assert st["derived"] == o.stats()["derived"]
    eng.close()


def test_increments_random(oracle_lib):
    for seed in range(60):
        ax = generators.random_small(seed, n=10 + seed % 40, n_roles=1 + seed % 4)
        _check(ax, _split(ax, 2 + seed % 3, seed, grow=bool(seed % 2)), oracle_lib)


@pytest.mark.parametrize("name,scale", [("g1", 0.1), ("g2", 0.05), ("g5", 0.03)])
def test_increments_workloads(name, scale, oracle_lib):
    ax = generators.workload(name, scale)
    _check(ax, _split(ax, 3, 7, grow=False), oracle_lib)
    _check(ax, _split(ax, 3, 8, grow=True), oracle_lib)


def test_increment_before_init(oracle_lib):
    ax = generators.random_small(5, n=30, n_roles=3)
    a, b = _split(ax, 2, 5, grow=True)
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(a)
    eng.add_axioms(b)  # nothing saturated yet: a plain reload of old ∪ inc
    eng.init()
    eng.saturate()
    o = oracle_lib.saturate(ax, 0, compat_range=True)
    assert np.array_equal(np.stack(eng.facts()), np.stack(o.facts()))
    eng.close()


def test_increment_rejects_shrink():
    ax = generators.random_small(6, n=30, n_roles=3)
    eng = engine.Engine(device=0)
    eng.load(ax)
    small = Axioms.build(10, ax.n_roles, kind=ax.kind[:10])
    with pytest.raises(engine.ElError) as e:
        eng.add_axioms(small)
    assert e.value.code == engine.EL_EINVAL
    eng.close()


def test_increment_rejects_elk_ranges():
    """ELK range fillers are numbered after the caller's concepts, which an increment may
    extend: with range axioms, increments need the DistEL range reading."""
    ax = generators.random_small(6, n=30, n_roles=3)
    inc = Axioms.build(ax.n_concepts, ax.n_roles, kind=ax.kind, range=[(0, 5)])
    eng = engine.Engine(device=0)
    eng.load(ax)
    eng.init()
    eng.saturate()
    with pytest.raises(engine.ElError) as e:
        eng.add_axioms(inc)
    assert e.value.code == engine.EL_EINVAL
    eng.close()


@pytest.mark.parametrize("name,scale", [("g3", 0.05), ("g5", 0.03), ("g3x", 0.02)])
def test_increment_is_a_delta(name, scale, oracle_lib):
    """A 1 % increment re-triggers only the logged facts and links its axioms reach (their index
    rows changed: AxiomLoader's currInc-scored keys, Type1_1AxiomProcessor.java:138-141), not
    every logged fact; the closure still equals the from-scratch closure of the union."""
    from distel_amd import ir
    ax = generators.workload(name, scale)
    base, inc = ir.split_increment(ax, 0.01, seed=3)
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(base)
    eng.init()
    before = eng.saturate()
    eng.add_axioms(inc)
    st = eng.saturate()
    tr_s, tr_l, _ = eng.trace()
    o = oracle_lib.saturate(ax, 0, compat_range=True)
    gx, ga = eng.facts()
    ox, oa = o.facts()
    assert np.array_equal(gx, ox) and np.array_equal(ga, oa), "S(X) differs from the from-scratch closure"
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c), "R(r) differs from the from-scratch closure"
    assert st["derived"] == o.stats()["derived"]
    # the first superstep's triggers: a fraction of the logs
    assert 0 < tr_s[0] < before["s_facts"] // 2, (int(tr_s[0]), before["s_facts"])
    assert tr_l[0] < max(before["links"] // 2, 1)
    eng.close()


@pytest.mark.parametrize("seed", range(12))
def test_two_increments_one_saturate(seed, oracle_lib):
    """Two el_add_axioms before one el_saturate (round-5 advisor, high): the second increment's
    carry-over must keep what the first one's axioms reach — the re-trigger masks of both are
    merged — or the facts only the first increment reaches stay below the watermarks."""
    ax = generators.random_small(100 + seed, n=20 + seed * 3, n_roles=1 + seed % 4)
    pieces = _split(ax, 3, 100 + seed, grow=bool(seed % 2))
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(pieces[0])
    eng.init()
    eng.saturate()
    eng.add_axioms(pieces[1])
    eng.add_axioms(pieces[2])
    st = eng.saturate()
    o = oracle_lib.saturate(ax, 0, compat_range=True)
    assert np.array_equal(np.stack(eng.facts()), np.stack(o.facts())), "S(X) differs from the union's closure"
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c), "R(r) differs from the union's closure"
    assert st["derived"] == o.stats()["derived"]
    eng.close()


def test_two_increments_one_saturate_g3(oracle_lib):
    from distel_amd import ir
    ax = generators.workload("g3", 0.03)
    base, inc = ir.split_increment(ax, 0.02, seed=11)
    inc1, inc2 = _split(inc, 2, 11, grow=False)
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(base)
    eng.init()
    eng.saturate()
    eng.add_axioms(inc1)
    eng.add_axioms(inc2)
    st = eng.saturate()
    o = oracle_lib.saturate(ax, 0, compat_range=True)
    assert np.array_equal(np.stack(eng.facts()), np.stack(o.facts()))
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c)
    assert st["derived"] == o.stats()["derived"]
    eng.close()


def test_increment_then_init_is_a_fresh_run(oracle_lib):
    """el_add_axioms, then el_init, then el_saturate (round-5 advisor, medium): the re-init drops
    the carried-over re-trigger lists, so the run equals a fresh load of old ∪ inc — closure,
    per-superstep deltas and per-kernel event counters alike."""
    from distel_amd import ir
    ax = generators.workload("g1", 0.05)
    base, inc = ir.split_increment(ax, 0.02, seed=4)
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(base)
    eng.init()
    eng.saturate()
    eng.add_axioms(inc)
    eng.init()
    st = eng.saturate()
    ref = engine.Engine(device=0, compat_range=True)
    ref.load(eng.ax)
    ref.init()
    st_ref = ref.saturate()
    assert np.array_equal(np.stack(eng.facts()), np.stack(ref.facts()))
    assert [np.asarray(t).tolist() for t in eng.trace()] == [np.asarray(t).tolist() for t in ref.trace()]
    assert st["derived"] == st_ref["derived"] == oracle_lib.saturate(ax, 0, compat_range=True).stats()["derived"]
    for ke, kr in zip(eng.kernel_stats(), ref.kernel_stats()):  # (el_init zeroes the counters)
        assert ke["events"] == kr["events"], ke["kernel"]
    ref.close()
    eng.close()
