"""Full-size workloads on the GPU against the CPU oracle (bit-exact closure, links,
per-superstep deltas and per-phase event counts).  G3X is compared with the oracle's pinned run
(tests/golden/runs/*.json, tests/golden/make_oracle_runs.py: its order-independent closure
digest, event counters, per-superstep trace and totals) instead of a fresh oracle run, which
took 85–140 s of the GPU box's host per test.

* G3X = G3 + 1 % sibling disjointness (A ⊓ B ⊑ ⊥), domains on 8 roles and ranges on 3: the
  ⊥ rule (TypeBottomAxiomProcessorBase.java:62-123, incl. ⊥ crossing links), domain and range
  (RolePairHandler.java:456-491) at SNOMED scale, where G1–G5 never trip them — ranges both
  ways: DistEL's reading (EL_FLAG_COMPAT_DISTEL_RANGE: range activations) and ELK's (the
  default: fresh range fillers).
* G5 (BASELINE configs[4], role-heavy) at full size: depth-20 chains, 50 transitive roles and
  hub fillers — the heaviest reference rule, T3_2 (ShardInfo.properties:9,
  Type3_2AxiomProcessorBase.java:67-96), over predecessor lists of up to ~39 k entries.
"""
import json
import os

import numpy as np
import pytest

from distel_amd import engine, generators
from distel_amd.result import set_digest

pytestmark = pytest.mark.gpu


def oracle_run(case):
    """The CPU oracle's pinned full-size run (tests/golden/make_oracle_runs.py)."""
    with open(os.path.join(os.path.dirname(__file__), "golden", "runs", f"{case}.json")) as f:
        return json.load(f)


def same_as_run(eng, st, run):
    """Closure and links (order-independent digest), every per-superstep delta and every
    per-phase event counter equal the pinned oracle run; returns the engine's facts and links."""
    fx, fa = eng.facts()
    lx, lr, ly = eng.links()
    assert set_digest(fx, fa, lx, lr, ly) == run["set_digest"]
    for g, c in zip(eng.trace(), run["trace"]):
        assert np.array_equal(g, np.asarray(c))
    assert np.array_equal(eng.events(), np.asarray(run["events"]))
    assert st["derived"] == run["stats"]["derived"]
    return fx, fa, lx, lr, ly


def _same(eng, o):
    gx, ga = eng.facts()
    ox, oa = o.facts()
    assert np.array_equal(gx, ox) and np.array_equal(ga, oa)
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c)
    for g, c in zip(eng.trace(), o.trace()):
        assert np.array_equal(g, c)
    assert np.array_equal(eng.events(), o.events())


def _digests():
    import os
    rows = []
    for line in open(os.path.join(os.path.dirname(__file__), "golden", "closure_digests.txt")):
        if line.strip() and not line.startswith("#"):
            name, scale, d_in, d_out = line.split()
            rows.append((name, float(scale), d_in, d_out))
    return rows


@pytest.mark.parametrize("case", _digests(), ids=lambda c: f"{c[0]}x{c[1]}")
def test_closure_digest_gpu(case):
    """The GPU closure of every pinned workload — G3 at full size (the bench configuration)
    included — hashes to the digest the semi-naive oracle and the independent worklist
    saturator both produced (tests/golden/pin_report.txt)."""
    import hashlib
    name, scale, d_in, d_out = case
    ax = generators.workload(name, scale)
    assert ax.digest() == d_in, "generator output changed"
    eng, _ = engine.classify(ax, device=0)
    h = hashlib.sha256()
    for a in eng.facts() + eng.links():
        h.update(np.ascontiguousarray(a, dtype=np.uint32).tobytes())
    eng.close()
    assert h.hexdigest() == d_out


def test_g3x_bottom_domain_range_full():
    ax = generators.workload("g3x")
    run = oracle_run("g3x_compat")
    assert ax.digest() == run["input_sha256"], "generator output changed"
    eng, st = engine.classify(ax, device=0, compat_range=True)
    x, a, lx, lr, ly = same_as_run(eng, st, run)
    # the rules this workload exists for did fire
    assert st["activations"] > 10_000                      # range activations (Y, C)
    ev = dict(zip(engine.KERNEL_NAMES, eng.events().tolist()))
    assert sum(ev["k_expand:a"]) > 0 and sum(ev["k_commit:a"]) > 0
    unsat = np.zeros(ax.n_concepts, bool)
    unsat[x[a == 0]] = True
    assert unsat.sum() > 100 and np.unique(lx[unsat[ly]]).size > 0  # ⊥, also across links
    for r, d in ax.domain.tolist():                                 # domain: every r-subject is in D
        subj = np.unique(lx[lr == r])
        subj = subj[subj != 1]
        have = np.zeros(ax.n_concepts, bool)
        have[x[a == d]] = True
        assert subj.size and have[subj].all()
    eng.close()


def test_g3x_elk_ranges_full():
    """G3X with ranges read ELK's way (the default): fresh fillers B ⊓ ranges*(r) for the
    range roles' existentials; the caller's rows bit-exact with the oracle's."""
    ax = generators.workload("g3x")
    run = oracle_run("g3x_elk")
    assert ax.digest() == run["input_sha256"], "generator output changed"
    eng, st = engine.classify(ax, device=0)
    same_as_run(eng, st, run)
    fb, fr = eng.fresh_fillers()
    assert fb.size > 100 and set(fr.tolist()) <= {r for r, _ in ax.range.tolist()}
    assert st["activations"] == 0
    eng.close()


def test_g5_full(oracle_lib):
    ax = generators.workload("g5")
    eng, st = engine.classify(ax, device=0)
    o = oracle_lib.saturate(ax, 0)
    _same(eng, o)
    assert st["derived"] == o.stats()["derived"]
    # hub fillers with 10^4 predecessors
    x, r, y = o.links()
    _, fan = np.unique(r.astype(np.int64) * ax.n_concepts + y, return_counts=True)
    assert fan.max() >= 10_000
    eng.close()


def test_g3e_told_cycles(oracle_lib):
    """G3E: G3 + 1 % named equivalences near the roots — told cycles (EquivalentClasses becomes
    two SubClassOf axioms, Normalizer.java:277-279) above most of the taxonomy, so the told
    closure's strongly connected components and everything below them take the cycle path;
    bit-exact with the oracle (closure, links, per-superstep deltas, event counters)."""
    ax = generators.workload("g3e", 0.05)
    eng, st = engine.classify(ax, device=0)
    o = oracle_lib.saturate(ax, 0)
    _same(eng, o)
    assert st["derived"] == o.stats()["derived"]
    eng.close()
