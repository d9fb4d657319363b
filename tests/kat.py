"""Known-answer-test fixtures: .elax files with hand-derived '#!' expectations."""
import glob
import os

from distel_amd import ir

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def kat_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "kat_*.elax")))


def load_kat(path):
    text = open(path, encoding="utf-8").read()
    ax = ir.parse_text(text)
    cid = {n: i for i, n in enumerate(ax.concept_names)}
    rid = {n: i for i, n in enumerate(ax.role_names)}
    exp = {"S": {}, "L": [], "NL": [], "NS": []}
    for line in text.splitlines():
        if not line.startswith("#! "):
            continue
        tok = line[3:].split()
        if tok[0] == "S":
            assert tok[2] == "="
            exp["S"][cid[tok[1]]] = {cid[t] for t in tok[3:]}
        elif tok[0] in ("L", "NL"):
            exp[tok[0]].append((cid[tok[1]], rid[tok[2]], cid[tok[3]]))
        elif tok[0] == "NS":
            exp["NS"].append((cid[tok[1]], cid[tok[2]]))
    return ax, exp


def check(exp, S, R):
    """S: dict x -> set, R: set of (x, r, y)."""
    for x, want in exp["S"].items():
        assert S.get(x, set()) == want, (x, S.get(x), want)
    for t in exp["L"]:
        assert t in R, t
    for t in exp["NL"]:
        assert t not in R, t
    for x, b in exp["NS"]:
        assert b not in S.get(x, set()), (x, b)


def to_sets(fx, fa, lx=None, lr=None, ly=None):
    S = {}
    for x, a in zip(fx.tolist(), fa.tolist()):
        S.setdefault(x, set()).add(a)
    R = set()
    if lx is not None:
        R = set(zip(lx.tolist(), lr.tolist(), ly.tolist()))
    return S, R


def compat_file(name):
    return os.path.join(GOLDEN, name)


def distel_chain_set(ax):
    """Test-side mirror of el::distel_chain_set (hazard H2): the chain set DistEL's CR6 applies,
    {r∘s⊑t : s second and t third in some chains whose first role is r}."""
    import dataclasses

    import numpy as np
    by = {}
    for r, s, t in ax.chain.tolist():
        a, b = by.setdefault(r, (set(), set()))
        a.add(s), b.add(t)
    ch = sorted((r, s, t) for r, (ss, tt) in by.items() for s in ss for t in tt)
    return dataclasses.replace(ax, chain=np.asarray(ch, dtype=np.uint32).reshape(-1, 3))
