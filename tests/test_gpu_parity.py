"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

Bit-exact comparison of S(X), R(r), the per-superstep deltas and the per-kernel
algorithmic event counters — integer/bitset work, no tolerance.  Runs on a real
MI355X only (``-m gpu``).
"""
import os
import random

import numpy as np
import pytest

import kat
from distel_amd import engine, generators, ir
from distel_amd.engine import AxiomDistributionType as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def oracle_mod(oracle_lib):
    return oracle_lib


def _gpu(ax, profile=False):
    eng, st = engine.classify(ax, device=0, profile=profile)
    return eng, st


def _assert_same(eng, o, events=True, trace=True):
    gx, ga = eng.facts()
    ox, oa = o.facts()
    assert np.array_equal(gx, ox) and np.array_equal(ga, oa)
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c)
    if trace:
        for g, c in zip(eng.trace(), o.trace()):
            assert np.array_equal(g, c)
    if events:
        assert np.array_equal(eng.events(), o.events())


@pytest.mark.parametrize("path", kat.kat_files(), ids=lambda p: os.path.basename(p))
def test_kat_gpu(path, oracle_mod):
    ax, exp = kat.load_kat(path)
    eng, st = _gpu(ax)
    S, R = kat.to_sets(*eng.facts(), *eng.links())
    kat.check(exp, S, R)
    _assert_same(eng, oracle_mod.saturate(ax, 0))
    eng.close()


def test_range_readings_gpu(oracle_mod):
    """Hazard H1 both ways: ELK's reading (default) on the ELK range KATs and random
    ontologies with ranges is covered by test_kat_gpu / test_fuzz_gpu; DistEL's reading
    (EL_FLAG_COMPAT_DISTEL_RANGE, RolePairHandler.java:471-479) on its KAT and on random
    ontologies, bit-exact with the oracle's DistEL range rule (events and deltas included)."""
    ax, exp = kat.load_kat(kat.compat_file("compat_range_distel.elax"))
    eng, _ = engine.classify(ax, device=0, compat_range=True)
    kat.check(exp, *kat.to_sets(*eng.facts(), *eng.links()))
    _assert_same(eng, oracle_mod.saturate(ax, 0, compat_range=True))
    eng.close()
    eng = engine.Engine(device=0, compat_range=True)
    for seed in range(150):
        ax = generators.random_small(7700 + seed, n=8 + seed % 50, n_roles=1 + seed % 5)
        eng.load(ax)
        eng.init()
        eng.saturate()
        _assert_same(eng, oracle_mod.saturate(ax, 0, compat_range=True))
    eng.close()
    # ELK's reading: the fresh fillers are reported, and every one is B ⊓ ranges*(r)
    ax, _ = kat.load_kat(os.path.join(kat.GOLDEN, "kat_range.elax"))
    eng, _ = engine.classify(ax, device=0)
    b, r = eng.fresh_fillers()
    assert b.size == 1 and eng.copy_result().row_hi == ax.n_concepts
    eng.close()


def test_fuzz_gpu(oracle_mod):
    eng = engine.Engine(device=0)
    for seed in range(300):
        ax = generators.random_small(seed, n=8 + seed % 60, n_roles=1 + seed % 5)
        eng.load(ax)
        eng.init()
        st = eng.saturate()
        o = oracle_mod.saturate(ax, 0)
        _assert_same(eng, o)
        assert st["derived"] == o.stats()["derived"]
    eng.close()


def test_step_schedules(oracle_mod):
    """Per-rule entry points (el_step) in random orders reach the same fixpoint, with the
    same 'changed' answers as the oracle after every call."""
    rnd = random.Random(7)
    for seed in range(40):
        ax = generators.random_small(1000 + seed, n=30, n_roles=3)
        eng = engine.Engine(device=0)
        eng.load(ax)
        eng.init()
        o = oracle_mod.Oracle(ax, 0)
        o.init()
        idle = set()  # rule types that reported "no change" since the last change
        calls = 0
        while len(idle) < len(T) and calls < 20000:
            r = rnd.choice(list(T))
            a = eng.step(r)
            b = o.step(r)
            assert a == b
            idle = set() if a else idle | {r}
            calls += 1
        _assert_same(eng, o, trace=False)
        o2 = oracle_mod.saturate(ax, 0)
        _assert_same(eng, o2, events=False, trace=False)
        eng.close()


def test_g1_scaled(oracle_mod):
    ax = generators.workload("g1", scale=0.25)
    eng, st = _gpu(ax)
    _assert_same(eng, oracle_mod.saturate(ax, 0))
    eng.close()


def test_g2_full(oracle_mod):
    ax = generators.workload("g2")
    eng, st = _gpu(ax, profile=True)
    o = oracle_mod.saturate(ax, 0)
    _assert_same(eng, o)
    assert st["derived"] == o.stats()["derived"]
    ks = eng.kernel_stats()
    assert sum(k["ms"] for k in ks) > 0
    eng.close()


def test_g5_scaled(oracle_mod):
    ax = generators.workload("g5", scale=0.05)
    eng, st = _gpu(ax)
    _assert_same(eng, oracle_mod.saturate(ax, 0))
    eng.close()


def test_replicated_block_diagonal():
    """×k disjoint copies (OntologyMultiplier): the closure of copy i is copy 0's
    closure shifted by i·m — a size-independent property at full G1 size."""
    base = generators.workload("g1")
    k = 4
    rep = ir.replicate(base, k)
    e0, s0 = _gpu(base)
    ek, sk = _gpu(rep)
    assert sk["derived"] == k * s0["derived"]
    bx, ba = e0.facts()
    kx, ka = ek.facts()
    m = base.n_concepts - 2
    shift = lambda v, i: np.where(v < 2, v, v + i * m)
    for i in range(k):
        sel = (kx >= 2 + i * m) & (kx < 2 + (i + 1) * m)
        own = bx >= 2
        assert np.array_equal(kx[sel], shift(bx[own], i))
        assert np.array_equal(ka[sel], shift(ba[own], i))
    e0.close()
    ek.close()


def test_reinit_idempotent():
    ax = generators.workload("g1", scale=0.2)
    eng = engine.Engine(device=0)
    eng.load(ax)
    eng.init()
    a = eng.saturate()
    f1 = eng.facts()
    eng.init()
    b = eng.saturate()
    f2 = eng.facts()
    assert a["derived"] == b["derived"]
    assert all(np.array_equal(x, y) for x, y in zip(f1, f2))
    # saturating a saturated state is a no-op
    c = eng.saturate()
    assert c["supersteps"] == 0 and c["derived"] == b["derived"]
    eng.close()


def test_export_layouts(oracle_mod):
    ax, _ = kat.load_kat(os.path.join(kat.GOLDEN, "kat_individuals.elax"))
    eng, _ = _gpu(ax)
    k, v = eng.export_result(engine.LAYOUT_X_TO_B)
    kb, vb = eng.export_result(engine.LAYOUT_B_TO_X)
    assert sorted(zip(k.tolist(), v.tolist())) == sorted(zip(vb.tolist(), kb.tolist()))
    assert 0 not in set(k.tolist())  # ⊥ is never a result-node member key
    eng.close()


def test_empty_and_edge():
    # only ⊥/⊤
    ax = ir.Axioms.build(2, 0)
    eng, st = _gpu(ax)
    assert st["s_facts"] == 2 and st["links"] == 0
    eng.close()
    # no axioms but many concepts
    ax = ir.Axioms.build(5000, 3)
    eng, st = _gpu(ax)
    assert st["s_facts"] == 2 + 2 * 4998 and st["supersteps"] == 1
    eng.close()


def test_told_cycle_large_subtree(oracle_mod):
    """A told 2-cycle (A ≡ B) at the top of a 3000-concept subtree (a random tree of depth up to
    ~40 with existentials into it): every concept below the cycle is closed by the Jacobi
    relaxation instead of the Kahn levels (advisor, round 3: the relaxation's capacity cliff).
    Bit-exact against the oracle."""
    rng = np.random.default_rng(7)
    n = 3002
    a, b = 2, 3
    sub = [(a, b), (b, a)]
    for c in range(4, n):  # each concept below one or two earlier ones (a DAG under the cycle)
        sub.append((c, int(rng.integers(2, c))))
        if rng.random() < 0.3:
            sub.append((c, int(rng.integers(2, c))))
    ex_rhs = [(int(rng.integers(2, n)), int(rng.integers(0, 3)), int(rng.integers(2, n))) for _ in range(600)]
    ex_lhs = [(int(rng.integers(0, 3)), int(rng.integers(2, n)), int(rng.integers(2, n))) for _ in range(200)]
    ax = ir.Axioms.build(n, 3, sub=sub, ex_rhs=ex_rhs, ex_lhs=ex_lhs)
    o = oracle_mod.saturate(ax)
    eng, st = _gpu(ax)
    _assert_same(eng, o)
    gx, ga = eng.facts()
    assert np.count_nonzero((gx == 1000) & (ga == a)) == 1  # (deep in the subtree: A and B above it)
    assert np.count_nonzero((gx == 1000) & (ga == b)) == 1
    eng.close()
    o.close()


def test_bad_input_rejected():
    eng = engine.Engine(device=0)
    ax = ir.Axioms.build(4, 1, sub=[(2, 3)])
    ax.sub[0, 1] = 9  # out of range
    with pytest.raises(Exception):
        eng.load(ax)
    with pytest.raises(engine.ElError):
        eng.init()  # state error: nothing loaded
    eng.close()


def test_classifier_rule_types_equals_fused(oracle_mod):
    from distel_amd.classifier import ELClassifier
    ax = generators.workload("g1", scale=0.05)
    with ELClassifier(ax) as a:
        a.classify("rule-types")
        fa = a.engine.facts()
        la = a.engine.links()
    with ELClassifier(ax) as b:
        b.classify("fused")
        fb = b.engine.facts()
        lb = b.engine.links()
    for u, v in zip(fa + la, fb + lb):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("wl", [("g1", 0.25), ("g5", 0.05)], ids=lambda w: f"{w[0]}x{w[1]}")
def test_queue_overflow_exact(wl, oracle_mod, monkeypatch):
    """Candidate queues far too small (EL_QUEUE_CAP): steps overflow, their commit is skipped
    and the step re-runs with larger queues — the closure and every per-step delta are still
    the oracle's (the re-run's generation work is counted again, so events are not compared)."""
    monkeypatch.setenv("EL_QUEUE_CAP", "512")
    ax = generators.workload(wl[0], scale=wl[1])
    eng, st = _gpu(ax)
    _assert_same(eng, oracle_mod.saturate(ax, 0), events=False, trace=True)
    eng.close()


def test_g3_full():
    """BASELINE configs[2] size (SNOMED-shaped, 390k concepts after normalization, 136 M derived
    axioms): closure, links, every per-superstep delta and the per-phase event counts equal
    the CPU oracle's pinned run (tests/golden/runs/g3.json, cross-checked against the SHA-256
    closure pin that the independent worklist saturator confirmed)."""
    from test_gpu_workloads import oracle_run, same_as_run
    ax = generators.workload("g3")
    run = oracle_run("g3")
    assert ax.digest() == run["input_sha256"], "generator output changed"
    eng, st = _gpu(ax)
    same_as_run(eng, st, run)
    assert st["derived"] == 136499458
    eng.close()


def test_h2_compat_gpu(oracle_mod):
    """EL_FLAG_COMPAT_DISTEL_CHAIN: the H2 KAT, and random ontologies against both the literal
    DistEL CR6 restatement (naive) and the C oracle over the expanded chain set (bit-exact,
    events and per-step deltas included); incremental chain axioms re-expand over old ∪ inc."""
    import naive
    ax, exp = kat.load_kat(kat.compat_file("compat_h2_two_chains.elax"))
    eng, _ = engine.classify(ax, device=0, compat_chain=True)
    kat.check(exp, *kat.to_sets(*eng.facts(), *eng.links()))
    eng.close()
    eng = engine.Engine(device=0, compat_chain=True)
    for seed in range(120):
        ax = generators.random_small(9100 + seed, n=8 + seed % 30, n_roles=2 + seed % 4)
        eng.load(ax)
        eng.init()
        eng.saturate()
        _assert_same(eng, oracle_mod.saturate(kat.distel_chain_set(ax), 0))
        if seed < 40:
            assert kat.to_sets(*eng.facts(), *eng.links()) == naive.saturate(ax, distel_chain=True), seed
    eng.close()
    # increment: the second chain sharing r arrives later; H2 must fire for the old links too
    import dataclasses
    full, exp = kat.load_kat(kat.compat_file("compat_h2_two_chains.elax"))
    base = dataclasses.replace(full, chain=full.chain[:1])
    eng = engine.Engine(device=0, compat_chain=True)
    eng.load(base)
    eng.init()
    eng.saturate()
    inc = ir.Axioms.build(full.n_concepts, full.n_roles, kind=full.kind, chain=full.chain[1:])
    eng.add_axioms(inc)
    eng.saturate()
    kat.check(exp, *kat.to_sets(*eng.facts(), *eng.links()))
    eng.close()


def test_flags_unknown_rejected():
    lib = engine.load_library()
    import ctypes as C
    ctx = C.c_void_p()
    cfg = engine._ElConfig(0, 0, 0x80)
    assert lib.el_create(C.byref(ctx), C.byref(cfg)) == engine.EL_EINVAL
