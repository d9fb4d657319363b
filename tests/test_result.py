"""Result-node output format (CPU: fed by the oracle's facts)."""
import os

import numpy as np

import kat
from distel_amd import ir, result


def test_packed_ids():
    # Constants.java:30-31: ⊤ = TOP_ID 1, ⊥ = BOTTOM_ID 0; EntityType digit last
    assert result.packed_id(1, 0) == "0110"
    assert result.packed_id(0, 0) == "0100"
    assert result.packed_id(12345, 2) == "05123452"
    assert result.unpack_ids("0110" + "05123452" + "0231") == ["0110", "05123452", "0231"]


def test_distel_numbering_order():
    ax = ir.parse_text("individual a\nconcept B\nrole r\ndatatype d\nconcept C\nsub B C\n")
    ids, rids = result.distel_numbering(ax)
    names = ax.concept_names
    num = {names[i]: int(ids[i]) for i in range(ax.n_concepts)}
    # classes first (from 2), then individuals, then roles, then datatypes
    assert num["owl:Thing"] == 1 and num["owl:Nothing"] == 0
    assert num["B"] == 2 and num["C"] == 3 and num["a"] == 4
    assert rids.tolist() == [5] and num["d"] == 6


def test_result_node_layouts(oracle_lib):
    ax, _ = kat.load_kat(os.path.join(kat.GOLDEN, "kat_individuals.elax"))
    o = oracle_lib.saturate(ax, 0)
    fx, fa = o.facts()
    rn = result.ResultNode(ax, fx, fa, distel_compat=True)
    db0, db1 = rn.db0(), rn.db1()
    cid = {n: i for i, n in enumerate(ax.concept_names)}
    # ⊤ ∈ S(X) for every class and individual: result[⊤] holds all of them
    assert set(db0[1].tolist()) == {i for i in range(1, ax.n_concepts)}
    # H7: ⊥ ⊑ a for individuals (result[a] ∋ ⊥)
    assert 0 in db0[cid["a"]].tolist() and 0 in db0[cid["b"]].tolist()
    # flip consistency
    pairs0 = {(int(x), b) for b, xs in db0.items() for x in xs}
    pairs1 = {(x, int(b)) for x, bs in db1.items() for b in bs}
    assert pairs0 == pairs1
    lines = list(rn.saxiom_lines(use_names=True))
    assert "a|H" in lines and "a|owl:Thing" in lines
    assert rn.axiom_counter(1)["total_subclass_axioms"] == len(lines)
    rn2 = result.ResultNode(ax, fx, fa, distel_compat=False)
    assert len(list(rn2.saxiom_lines())) == len(lines) - 2


def test_write_saxioms(tmp_path, oracle_lib):
    ax, _ = kat.load_kat(os.path.join(kat.GOLDEN, "kat_cr1_chain.elax"))
    o = oracle_lib.saturate(ax, 0)
    rn = result.ResultNode(ax, *o.facts())
    p = tmp_path / "final-saxioms-distel.txt"
    n = rn.write_saxioms(str(p))
    text = p.read_text().splitlines()
    assert n == len(text) and "0120|0150" in text  # A (id 2) ⊑ D (id 5)


def test_diff_results_elk_conventions(tmp_path):
    """ResultDiffWriter-style comparison: equal sets pass; a missing / extra superclass
    counts once per class; unsatisfiable classes compare on ⊥ only (H4)."""
    from distel_amd.result import diff_results, read_saxioms
    exp = {"A": {"A", "B", "owl:Thing"}, "U": {"U", "owl:Nothing", "A", "B", "C"}, "C": {"C"}}
    got = {"A": {"A", "B", "owl:Thing"}, "U": {"U", "owl:Nothing"}, "C": {"C", "A"}}
    misses, rep = diff_results(exp, got)
    assert misses == 1 and "C -- " in rep[0] and rep[-1] == "No of classes not equal: 1"
    p = tmp_path / "x.txt"
    p.write_text("A|B\nA|A\n# comment\nC|C\n")
    assert read_saxioms(str(p)) == {"A": {"A", "B"}, "C": {"C"}}


def test_cli_normalize(tmp_path):
    import os
    from distel_amd import cli, owl
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "owl", "kat_definitions.ofn")
    out = tmp_path / "norm.ofn"
    assert cli.main(["normalize", src, str(out)]) == 0
    n = owl.parse_functional(out.read_text())
    a = owl.to_axioms(n)                               # already normal: types without normalizing
    b = owl.to_axioms(owl.normalize(owl.parse_functional(open(src).read())))
    assert a.counts() == b.counts()


def test_set_digest_order_independent_and_pinned(oracle_lib):
    """set_digest ignores order, sees every entry, and reproduces the pinned set digest of a
    pinned workload from the oracle's closure (tests/golden/set_digests.txt)."""
    from distel_amd import generators
    rng = np.random.default_rng(7)
    fx, fa = rng.integers(0, 1000, 500).astype(np.uint32), rng.integers(0, 1000, 500).astype(np.uint32)
    lx, lr, ly = (rng.integers(0, 50, 300).astype(np.uint32) for _ in range(3))
    d = result.set_digest(fx, fa, lx, lr, ly)
    p, q = rng.permutation(500), rng.permutation(300)
    assert result.set_digest(fx[p], fa[p], lx[q], lr[q], ly[q]) == d
    fa2 = fa.copy()
    fa2[17] ^= 1
    assert result.set_digest(fx, fa2, lx, lr, ly) != d
    lr2 = lr.copy()
    lr2[3] += 1
    assert result.set_digest(fx, fa, lx, lr2, ly) != d
    pins = {}
    for line in open(os.path.join(os.path.dirname(__file__), "golden", "set_digests.txt")):
        f = line.split()
        if len(f) == 4 and not line.startswith("#"):
            pins[(f[0], float(f[1]))] = (f[2], f[3])
    ax = generators.workload("g1", 0.1)
    assert ax.digest() == pins[("g1", 0.1)][0]
    o = oracle_lib.saturate(ax, 0)
    assert result.set_digest(*o.facts(), *o.links()) == pins[("g1", 0.1)][1]


def test_oracle_run_fixtures_consistent():
    """The pinned full-size oracle runs (tests/golden/runs, what the -m gpu full-size tests compare
    the engine with) match their generators' inputs, and the G3 one matches G3's set-digest pin."""
    import json
    from distel_amd import generators
    here = os.path.join(os.path.dirname(__file__), "golden")
    pins = {}
    for line in open(os.path.join(here, "set_digests.txt")):
        f = line.split()
        if len(f) == 4 and not line.startswith("#"):
            pins[(f[0], float(f[1]))] = (f[2], f[3])
    inputs = {}
    for case in ("g3", "g3x_compat", "g3x_elk"):
        with open(os.path.join(here, "runs", f"{case}.json")) as fh:
            run = json.load(fh)
        name = run["workload"]
        if name not in inputs:
            inputs[name] = generators.workload(name).digest()
        assert run["input_sha256"] == inputs[name]
        ev = np.asarray(run["events"])
        assert ev.ndim == 2 and ev.sum() > 0 and len(run["trace"]) == 3
        assert len(run["trace"][0]) == run["stats"]["supersteps"]
        if case == "g3":  # (no range fillers: every fact is the caller's)
            assert run["set_digest"].startswith(f"{run['stats']['s_facts']}:{run['stats']['links']}:")
    with open(os.path.join(here, "runs", "g3.json")) as fh:
        assert json.load(fh)["set_digest"] == pins[("g3", 1.0)][1]


def test_stream_runs_malformed_raise():
    """A streamed result's run table that does not cover its entries is an error, not an assert
    (python -O keeps the check)."""
    from distel_amd.engine import Stream
    runs = np.array([[5, 3], [6, 7]], np.uint32)
    assert Stream._rows(runs, 2, 7).tolist() == [5, 5, 5, 6, 6, 6, 6]
    for n_runs, n in ((2, 8), (0, 4)):
        try:
            Stream._rows(runs, n_runs, n)
        except ValueError:
            continue
        raise AssertionError("malformed runs accepted")
    bad = np.array([[5, 3], [6, 3]], np.uint32)
    try:
        Stream._rows(bad, 2, 3)
    except ValueError:
        return
    raise AssertionError("empty run accepted")
