"""OWL functional-syntax loader + normalizer on the CPU:
hand-derived known answers, normal-form invariants, and the normalizer's entailments
among the original names against an independent definitorial translation."""
import glob
import os
import random

import numpy as np
import pytest

from distel_amd import ir, owl

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "owl")


def _closure(ax, oracle_lib):
    o = oracle_lib.saturate(ax, 0)
    x, a = o.facts()
    names = ax.concept_names
    S = {}
    for xi, ai in zip(x.tolist(), a.tolist()):
        S.setdefault(names[xi], set()).add(names[ai])
    return S


def _short(iri):
    if iri == owl.NOTHING:
        return "owl:Nothing"
    return iri.rsplit("#", 1)[-1]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "*.ofn"))), ids=os.path.basename)
def test_owl_kat(path, oracle_lib):
    with pytest.warns(UserWarning) if "roles" in path else _nullctx():
        ax = owl.load_functional(path, normalized=False)
    S = _closure(ax, oracle_lib)
    S = {_short(k): {_short(v) for v in vs if v != owl.THING and not v.startswith(owl.GENSYM)}
         for k, vs in S.items() if not k.startswith(owl.GENSYM)}
    for line in open(path, encoding="utf-8"):
        if line.startswith("#! S "):
            lhs, rhs = line[5:].split("=")
            x = lhs.strip()
            assert S.get(x, set()) == set(rhs.split()), x
        elif line.startswith("#! NS "):
            x, b = line[6:].split()
            assert b not in S.get(x, set())


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def test_normal_forms_only():
    text = open(os.path.join(GOLD, "kat_definitions.ofn"), encoding="utf-8").read()
    n = owl.normalize(owl.parse_functional(text))
    for c, d in n.sub:
        basic_c, basic_d = owl.is_basic(c), owl.is_basic(d)
        assert (basic_c and (basic_d or (d[0] == "SOME" and owl.is_basic(d[2])))) or \
               (basic_d and c[0] == "AND" and len(c[1]) == 2 and all(owl.is_basic(x) for x in c[1])) or \
               (basic_d and c[0] == "SOME" and owl.is_basic(c[2])), (c, d)


def test_gensym_deterministic():
    text = open(os.path.join(GOLD, "kat_definitions.ofn"), encoding="utf-8").read()
    a = owl.to_axioms(owl.normalize(owl.parse_functional(text)))
    b = owl.to_axioms(owl.normalize(owl.parse_functional(text)))
    assert a.digest() == b.digest() and a.concept_names == b.concept_names


def test_parse_errors():
    with pytest.raises(owl.ParseError):
        owl.parse_functional("Ontology(SubClassOf(:A :B)")      # unbalanced
    with pytest.raises(owl.ParseError):
        owl.parse_functional("Ontology(SubClassOf(zz:A <b>))")  # unknown prefix
    with pytest.raises(ValueError):  # a complex axiom typed without normalization
        owl.to_axioms(owl.parse_functional(
            "Prefix(:=<http://e/#>) Ontology(SubClassOf(:A ObjectIntersectionOf(:B :C)))"))


def test_normalized_roundtrip(tmp_path, oracle_lib):
    """A normalized EL+ ontology written as functional syntax and read back with
    isNormalized=true classifies exactly like the IR it came from."""
    for seed in range(40):
        ax = ir.replicate(_no_range(seed), 1)
        onto = _ir_to_onto(ax)
        p = tmp_path / f"n{seed}.ofn"
        owl.write_functional(onto, str(p))
        bx = owl.load_functional(str(p), normalized=True)
        Sa = _closure_named(ax, oracle_lib)
        Sb = _closure(bx, oracle_lib)
        assert Sa == Sb, seed


def _no_range(seed):
    from distel_amd import generators
    ax = generators.random_small(seed, n=20, n_roles=3)
    ax.range = np.zeros((0, 2), np.uint32)
    return ax


def _names(ax):
    cn = [owl.NOTHING, owl.THING] + [f"http://t/#c{i}" if ax.kind[i] == 0 else
                                       (f"http://t/#i{i}" if ax.kind[i] == 1 else f"http://t/#d{i}")
                                       for i in range(2, ax.n_concepts)]
    rn = [f"http://t/#r{i}" for i in range(ax.n_roles)]
    return cn, rn


def _closure_named(ax, oracle_lib):
    cn, _ = _names(ax)
    o = oracle_lib.saturate(ax, 0)
    x, a = o.facts()
    S = {}
    for xi, ai in zip(x.tolist(), a.tolist()):
        S.setdefault(cn[xi], set()).add(cn[ai])
    return S


def _ir_to_onto(ax):
    cn, rn = _names(ax)
    o = owl.Ontology(iri="http://t/")

    def e(i):
        k = int(ax.kind[i])
        return ("C", cn[i]) if k == 0 else ("I", cn[i]) if k == 1 else ("D", cn[i])
    for i in range(2, ax.n_concepts):
        {0: o.classes, 1: o.individuals, 3: o.datatypes}[int(ax.kind[i])].add(cn[i])
    o.object_props = set(rn)
    for a, b in ax.sub:
        o.sub.append((e(a), e(b)))
    for i in range(ax.n_conj):
        ops = frozenset(e(j) for j in ax.conj_ops[ax.conj_ptr[i]:ax.conj_ptr[i + 1]])
        o.sub.append((("AND", ops) if len(ops) > 1 else next(iter(ops)), e(ax.conj_b[i])))
    for a, r, b in ax.ex_rhs:
        o.sub.append((e(a), ("SOME", rn[r], e(b))))
    for r, a, b in ax.ex_lhs:
        o.sub.append((("SOME", rn[r], e(a)), e(b)))
    o.subrole = [(rn[r], rn[s]) for r, s in ax.subrole]
    o.chain = [((rn[r], rn[s]), rn[t]) for r, s, t in ax.chain]
    o.domain = [(rn[r], e(d)) for r, d in ax.domain]
    return o


# ---- normalizer vs an independent definitorial translation on random complex ontologies
def _rand_expr(rnd, classes, roles, depth):
    k = rnd.random()
    if depth == 0 or k < 0.35:
        return ("C", rnd.choice(classes))
    if k < 0.65:
        n = rnd.randint(2, 3)
        ops = frozenset(_rand_expr(rnd, classes, roles, depth - 1) for _ in range(n))
        return ("AND", ops) if len(ops) > 1 else next(iter(ops))
    return ("SOME", rnd.choice(roles), _rand_expr(rnd, classes, roles, depth - 1))


def _definitorial(onto):
    """Every complex subexpression e gets X_e ≡ e (both directions): a conservative
    extension whose atomic consequences are exactly the ontology's."""
    out = owl.Ontology(classes=set(onto.classes), object_props=set(onto.object_props))
    names = {}

    def nm(e):
        if owl.is_basic(e):
            return e
        if e in names:
            return names[e]
        x = ("C", f"urn:def#{len(names)}")
        names[e] = x
        out.classes.add(x[1])
        if e[0] == "AND":
            ops = sorted((nm(o) for o in e[1]), key=repr)
            for o in ops:
                out.sub.append((x, o))
            out.sub.append((("AND", frozenset(ops)), x) if len(set(ops)) > 1 else (ops[0], x))
        else:
            f = nm(e[2])
            out.sub.append((x, ("SOME", e[1], f)))
            out.sub.append((("SOME", e[1], f), x))
        return x
    for c, d in onto.sub:
        out.sub.append((nm(c), nm(d)))
    out.chain = list(onto.chain)
    out.subrole = list(onto.subrole)
    return out


def test_normalizer_entailments_match_definitorial(oracle_lib):
    for seed in range(60):
        rnd = random.Random(seed)
        classes = [f"http://r/#C{i}" for i in range(8)]
        roles = [f"http://r/#r{i}" for i in range(2)]
        onto = owl.Ontology(classes=set(classes), object_props=set(roles))
        for _ in range(12):
            onto.sub.append((_rand_expr(rnd, classes, roles, 2), _rand_expr(rnd, classes, roles, 2)))
        if seed % 3 == 0:
            onto.chain.append(((roles[0], roles[1], roles[0]), roles[1]))
        a = _closure(owl.to_axioms(owl.normalize(onto)), oracle_lib)
        d = owl.Ontology(**{**onto.__dict__})
        d.chain = []
        for ch, s in onto.chain:  # the definitorial side splits chains by hand
            d.chain.append(((ch[0], ch[1]), "urn:def#rr"))
            d.chain.append((("urn:def#rr", ch[2]), s))
            d.object_props = d.object_props | {"urn:def#rr"}
        b = _closure(owl.to_axioms(_definitorial(d)), oracle_lib)
        for c in classes:
            assert {x for x in a.get(c, set()) if x in classes or x == owl.NOTHING} == \
                   {x for x in b.get(c, set()) if x in classes or x == owl.NOTHING}, (seed, c)
