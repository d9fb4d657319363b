"""Seeded synthetic EL+ ontologies (SURVEY.md §8(d) G1–G5) and a fuzz generator.

No real GO / NCI / SNOMED is available offline, so the benchmark configs of
BASELINE.json are substituted by shaped generators.  All of them are
deterministic for a given seed (numpy PCG64) and produce *normalized* axioms,
i.e. the same input AxiomLoader accepts with ``isNormalized = true``.

Shape model (shared by G1–G3, G5):

* a taxonomy DAG whose classes are ordered by level; level sizes grow
  geometrically, every class has one parent on the previous level plus a
  Poisson number of extra parents on the three levels above it;
* existential restrictions ``A ⊑ ∃r.B`` whose fillers sit strictly above A
  (more general), with roles drawn from a Zipf law;
* full definitions ``A ≡ P ⊓ ∃r.C`` normalized the way DistEL's Normalizer
  does (``kc/init/Normalizer.java:619-784``): ``A ⊑ P``, ``A ⊑ ∃r.C``,
  ``∃r.C ⊑ F``, ``P ⊓ F ⊑ A`` with a fresh class F;
* role inclusions, transitive roles and role chains as the config asks.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .ir import Axioms, KIND_CLASS, KIND_DATATYPE, KIND_INDIVIDUAL, replicate


def _levels(m: int, depth: int, growth: float) -> np.ndarray:
    """Boundaries b[0..depth] of `depth` levels over m classes (geometric sizes)."""
    w = growth ** np.arange(depth, dtype=np.float64)
    b = np.concatenate([[0.0], np.cumsum(w) / w.sum() * m])
    b = np.round(b).astype(np.int64)
    b[-1] = m
    # every level gets at least one class
    for i in range(1, depth + 1):
        b[i] = max(b[i], b[i - 1] + 1) if b[i - 1] < m else m
    return np.minimum(b, m)


def _taxonomy(rng: np.random.Generator, m: int, depth: int, mean_parents: float, growth: float = 1.45,
              window: int = 6):
    """Return (child, parent, level, bounds) over local class indices 0..m-1.

    Every class below level 0 has a first parent on the previous level at the same
    relative position (plus jitter), so subtrees stay local; extra parents (Poisson)
    come from one to three levels up, near the first parent's relative position.
    This keeps ancestor sets realistic (tens, not thousands)."""
    b = _levels(m, depth, growth)
    level = np.searchsorted(b, np.arange(m), side="right") - 1
    idx = np.arange(m)
    mask = level > 0
    kids = idx[mask]
    lv = level[mask]
    rel = (kids - b[lv]) / np.maximum(b[lv + 1] - b[lv], 1)      # relative position in own level

    def pick(lvl, jitter):
        lo, hi = b[lvl], b[lvl + 1]
        pos = lo + np.floor(rel_sel * (hi - lo)).astype(np.int64) + jitter
        return np.clip(pos, lo, hi - 1)
    rel_sel = rel
    first = pick(lv - 1, np.zeros(kids.size, dtype=np.int64))  # a proper tree spine
    ch, pa = [kids], [first]
    extra = rng.poisson(max(mean_parents - 1.0, 0.0), kids.size)
    rep = np.repeat(np.arange(kids.size), extra)
    if rep.size:
        tl = np.maximum(lv[rep] - 1, 0)   # a sibling of the first parent: diamonds re-converge
        rel_sel = rel[rep]
        par = pick(tl, rng.integers(-2, 3, rep.size))
        ch.append(kids[rep])
        pa.append(par)
    c = np.concatenate(ch)
    p = np.concatenate(pa)
    keep = c != p
    pairs = np.unique(np.stack([c[keep], p[keep]], 1), axis=0)
    return pairs[:, 0], pairs[:, 1], level, b


def _zipf_roles(rng: np.random.Generator, n: int, roles: Sequence[int], s: float) -> np.ndarray:
    k = len(roles)
    w = 1.0 / np.arange(1, k + 1, dtype=np.float64) ** s
    w /= w.sum()
    return np.asarray(roles, dtype=np.int64)[rng.choice(k, size=n, p=w)]


def _general_filler(rng: np.random.Generator, a_local: np.ndarray, level: np.ndarray, b: np.ndarray,
                    lift: int = 1, span: int = 4, local: bool = False) -> np.ndarray:
    """A filler above A: a class on a level in [level(A) - lift - span + 1, level(A) - lift]
    (clamped at 0) — more general than A, but not arbitrarily general.  ``local`` keeps the
    filler near A's relative position (definitions name related concepts)."""
    la = level[a_local]
    top = np.maximum(la - lift, 0)
    lv = np.maximum(top - rng.integers(0, span, a_local.size), 0)
    lo, hi = b[lv], b[lv + 1]
    if local:
        rel = (a_local - b[la]) / np.maximum(b[la + 1] - b[la], 1)
        pos = lo + np.floor(rel * (hi - lo)).astype(np.int64) + rng.integers(-3, 4, a_local.size)
        return np.clip(pos, lo, hi - 1)
    return lo + (rng.random(a_local.size) * (hi - lo)).astype(np.int64)


def shaped(seed: int, n: int, n_roles: int, depth: int, mean_parents: float, ex_frac: float, def_frac: float,
           zipf_s: float = 1.1, transitive: Sequence[int] = (), subroles: Sequence[Tuple[int, int]] = (),
           chains: Sequence[Tuple[int, int, int]] = (), domains: Sequence[Tuple[int, int]] = (),
           role_weights: Optional[Sequence[float]] = None, lift: int = 1, growth: float = 1.45,
           hubs: int = 0, hub_frac: float = 0.0, ranges: Sequence[Tuple[int, int]] = (),
           disjoint_frac: float = 0.0, disjoint_mid: int = 0) -> Axioms:
    """Generic shaped generator; ids: 0 ⊥, 1 ⊤, 2..n+1 taxonomy classes, then fresh
    definition classes F.  ``domains`` / ``ranges`` are (role, local class index).
    ``disjoint_frac``·n disjointness axioms A ⊓ B ⊑ ⊥ between neighbouring classes of one
    level (siblings, as DisjointClasses usually are), drawn from the two deepest levels, plus
    ``disjoint_mid`` such pairs four levels up (classes that are fillers: ⊥ crosses links)."""
    rng = np.random.default_rng(seed)
    m = n
    child, parent, level, b = _taxonomy(rng, m, depth, mean_parents, growth)
    base = 2
    sub = [np.stack([child + base, parent + base], 1)]
    # existentials A ⊑ ∃r.B, A below level 0
    n_ex = int(ex_frac * m)
    cand = np.nonzero(level > 0)[0]
    a = cand[rng.integers(0, cand.size, n_ex)]
    if role_weights is not None:
        w = np.asarray(role_weights, dtype=np.float64)
        r = rng.choice(n_roles, size=n_ex, p=w / w.sum())
    else:
        r = _zipf_roles(rng, n_ex, list(range(n_roles)), zipf_s)
    fil = _general_filler(rng, a, level, b, lift)
    if hubs and hub_frac > 0:
        k = int(hub_frac * n_ex)
        hub_ids = rng.choice(b[min(2, depth)], size=hubs, replace=False) if b[min(2, depth)] >= hubs else \
            np.arange(hubs)
        sel = rng.choice(n_ex, size=k, replace=False)
        fil[sel] = hub_ids[rng.integers(0, hubs, k)]
    ex_rhs = [np.stack([a + base, r, fil + base], 1)]
    # full definitions A ≡ P ⊓ ∃r.C
    n_def = int(def_frac * m)
    cand2 = np.nonzero(level >= 2)[0]
    da = rng.choice(cand2, size=min(n_def, cand2.size), replace=False)
    # P = the first listed parent of A (a parent on the previous level)
    first_parent = np.full(m, -1, dtype=np.int64)
    order = np.argsort(child, kind="stable")
    cs, ps = child[order], parent[order]
    firsts = np.unique(cs, return_index=True)
    first_parent[firsts[0]] = ps[firsts[1]]
    dp = first_parent[da]
    ok = dp >= 0
    da, dp = da[ok], dp[ok]
    nd = da.size
    if role_weights is not None:
        w = np.asarray(role_weights, dtype=np.float64)
        dr = rng.choice(n_roles, size=nd, p=w / w.sum())
    else:
        dr = _zipf_roles(rng, nd, list(range(n_roles)), zipf_s)
    dc = _general_filler(rng, da, level, b, lift + 1, local=True)
    F = base + m + np.arange(nd)
    ex_rhs.append(np.stack([da + base, dr, dc + base], 1))
    ex_lhs = np.stack([dr, dc + base, F], 1)
    conj_ops = np.stack([dp + base, F], 1).reshape(-1)
    conj_ptr = np.arange(0, 2 * nd + 1, 2)
    conj_b = da + base
    N = base + m + nd
    conj_ptr = conj_ptr.astype(np.int64)
    if disjoint_frac > 0:
        deep = np.nonzero((level >= depth - 2) & (np.arange(m) + 1 < m))[0]  # the two deepest levels
        deep = deep[level[np.minimum(deep + 1, m - 1)] == level[deep]]  # B = A + 1 on the same level
        da_ = rng.choice(deep, size=min(int(disjoint_frac * m), deep.size), replace=False)
        mid = np.nonzero((level == depth - 4) & (np.arange(m) + 1 < m))[0]
        mid = mid[level[np.minimum(mid + 1, m - 1)] == level[mid]]
        da_ = np.concatenate([da_, rng.choice(mid, size=min(disjoint_mid, mid.size), replace=False)])
        conj_ops = np.concatenate([conj_ops, np.stack([da_ + base, da_ + 1 + base], 1).reshape(-1)])
        conj_ptr = np.concatenate([conj_ptr, conj_ptr[-1] + 2 * np.arange(1, da_.size + 1)])
        conj_b = np.concatenate([conj_b, np.zeros(da_.size, dtype=np.int64)])
    ax = Axioms(
        n_concepts=int(N), n_roles=int(n_roles), kind=np.zeros(N, dtype=np.uint8),
        sub=np.ascontiguousarray(np.concatenate(sub).astype(np.uint32)),
        conj_ptr=conj_ptr.astype(np.uint32), conj_ops=conj_ops.astype(np.uint32), conj_b=conj_b.astype(np.uint32),
        ex_rhs=np.ascontiguousarray(np.concatenate(ex_rhs).astype(np.uint32)),
        ex_lhs=np.ascontiguousarray(ex_lhs.astype(np.uint32)),
        subrole=np.asarray(list(subroles), dtype=np.uint32).reshape(-1, 2),
        chain=np.asarray([(t, t, t) for t in transitive] + list(chains), dtype=np.uint32).reshape(-1, 3),
        domain=np.asarray([(rr, c + base) for rr, c in domains], dtype=np.uint32).reshape(-1, 2),
        range=np.asarray([(rr, c + base) for rr, c in ranges], dtype=np.uint32).reshape(-1, 2))
    ax.validate()
    return ax


# ------------------------------------------------------------------ G1..G5

def g1_go(seed: int = 0x60, n: int = 20_000) -> Axioms:
    """G1 "GO-like": 8 roles — part_of (0, transitive), regulates (1) ⊒
    positively_regulates (2), negatively_regulates (3), has_part (4), occurs_in (5),
    happens_during (6), ends_during (7); regulates ∘ part_of ⊑ regulates."""
    return shaped(seed, n, n_roles=8, depth=15, mean_parents=1.6, ex_frac=0.4, def_frac=0.05,
                  role_weights=[0.35, 0.15, 0.12, 0.12, 0.1, 0.08, 0.05, 0.03], lift=2,
                  transitive=[0], subroles=[(2, 1), (3, 1)], chains=[(1, 0, 1)], domains=[(5, 0)])


def g2_nci(seed: int = 0x4C1, n: int = 70_000) -> Axioms:
    """G2 "NCI-like": 60 roles, tree-like (mean 1.2 parents), 0.6·N existentials, no chains."""
    return shaped(seed, n, n_roles=60, depth=18, mean_parents=1.2, ex_frac=0.6, def_frac=0.05, zipf_s=1.1,
                  subroles=[(i, i + 30) for i in range(0, 10)], domains=[(40, 1), (41, 2)])


def g3_snomed(seed: int = 0x5C7, n: int = 300_000) -> Axioms:
    """G3 "SNOMED-shaped": 60 roles (Zipf 1.1), mean 1.7 parents, depth 24, 0.8·N
    existentials, 0.3·N full definitions, 10 r ⊑ s, 2 chains + 3 transitive roles."""
    sub = [(10 + i, 50 + i) for i in range(10)]
    return shaped(seed, n, n_roles=60, depth=24, mean_parents=1.7, ex_frac=0.8, def_frac=0.3, zipf_s=1.1,
                  transitive=[57, 58, 59], subroles=sub, chains=[(20, 57, 20), (21, 58, 21)], lift=2,
                  growth=1.4)


def g3_bottom_domain_range(seed: int = 0x5C7, n: int = 300_000) -> Axioms:
    """G3 with the rules G3 never trips: 1 % disjointness axioms A ⊓ B ⊑ ⊥ between sibling
    classes (⊥, TypeBottomAxiomProcessorBase.java:62-123), domains on 8 roles and ranges on 3
    (RolePairHandler.java:456-491; ranges with DistEL's semantics, hazard H1)."""
    sub = [(10 + i, 50 + i) for i in range(10)]
    domains = [(r, 1 + r % 7) for r in (0, 3, 5, 8, 12, 20, 33, 44)]
    ranges = [(r, 2 + r % 5) for r in (6, 17, 25)]
    return shaped(seed, n, n_roles=60, depth=24, mean_parents=1.7, ex_frac=0.8, def_frac=0.3, zipf_s=1.1,
                  transitive=[57, 58, 59], subroles=sub, chains=[(20, 57, 20), (21, 58, 21)], lift=2,
                  growth=1.4, domains=domains, ranges=ranges, disjoint_frac=0.01, disjoint_mid=30)


def g3_equivalences(seed: int = 0x5C7, n: int = 300_000, frac: float = 0.01) -> Axioms:
    """G3E: G3 plus frac·N named equivalences A ≡ B between neighbouring classes near the roots
    (the first ids: the top levels of the taxonomy).  DistEL's Normalizer turns every EquivalentClasses(A B)
    into two SubClassOf axioms (Normalizer.java:277-279), so each one is a told cycle A ⊑ B ⊑ A,
    and everything below it is closed as a strongly connected component of the told graph."""
    ax = g3_snomed(seed, n)
    rng = np.random.default_rng(seed ^ 0xE9)
    top = max(4, n // 15)
    k = max(1, int(frac * n))
    a = rng.choice(np.arange(2, 2 + top, dtype=np.int64), size=min(k, top - 1), replace=False)
    b = a + 1  # a neighbour on the same level: small cycles, not one giant component
    keep = (b < ax.n_concepts) & (ax.kind[a] == KIND_CLASS) & (ax.kind[np.minimum(b, ax.n_concepts - 1)] == KIND_CLASS)
    eq = np.stack([a[keep], b[keep]], axis=1)
    sub = np.concatenate([ax.sub, eq, eq[:, ::-1]]).astype(np.uint32)
    import dataclasses
    return dataclasses.replace(ax, sub=np.ascontiguousarray(sub))


def g4_snomed_x(copies: int = 8, seed: int = 0x5C7, n: int = 300_000) -> Axioms:
    """G4: ``copies`` disjoint copies of G3 (OntologyMultiplier semantics)."""
    return replicate(g3_snomed(seed, n), copies)


def g5_role_heavy(seed: int = 0x20E, n: int = 100_000) -> Axioms:
    """G5 "role-heavy": 200 roles, chains r_i ∘ r_{i+1} ⊑ r_{i+2} (depth 20),
    50 transitive roles, hub fillers with many predecessors."""
    chains = [(i, i + 1, i + 2) for i in range(20)]
    trans = list(range(100, 150))
    sub = [(150 + i, 100 + i) for i in range(50)]
    return shaped(seed, n, n_roles=200, depth=20, mean_parents=1.4, ex_frac=1.0, def_frac=0.1, zipf_s=0.9,
                  transitive=trans, subroles=sub, chains=chains, lift=3, hubs=16, hub_frac=0.1)


WORKLOADS = {
    "g1": g1_go,
    "g2": g2_nci,
    "g3": g3_snomed,
    "g3x": g3_bottom_domain_range,
    "g3e": g3_equivalences,
    "g5": g5_role_heavy,
}


def workload(name: str, scale: float = 1.0) -> Axioms:
    """Named workload, optionally scaled down (tests) — scale multiplies N."""
    if name == "g4":
        return g4_snomed_x(n=int(300_000 * scale))
    fn = WORKLOADS[name]
    default_n = {"g1": 20_000, "g2": 70_000, "g3": 300_000, "g3x": 300_000, "g3e": 300_000, "g5": 100_000}[name]
    return fn(n=max(64, int(default_n * scale)))


# ------------------------------------------------------------------ fuzz

def random_small(seed: int, n: int = 24, n_roles: int = 3, density: float = 1.0) -> Axioms:
    """Small random EL+ ontology exercising every rule (⊥, individuals, datatypes,
    n-ary conjunctions, role hierarchy with cycles, chains, domain, range)."""
    rng = np.random.default_rng(seed)
    N = n
    kind = np.zeros(N, dtype=np.uint8)
    ids = np.arange(2, N)
    n_ind = rng.integers(0, max(1, N // 8) + 1)
    n_dt = rng.integers(0, 3)
    perm = rng.permutation(ids)
    ind = perm[:n_ind]
    dts = perm[n_ind:n_ind + n_dt]
    kind[ind] = KIND_INDIVIDUAL
    kind[dts] = KIND_DATATYPE
    cls = np.setdiff1d(ids, dts)  # classes + individuals may appear as subclasses
    anyc = np.concatenate([[0, 1], cls])
    k = lambda f: int(rng.poisson(f * density * N))
    pick = lambda pool, sz: pool[rng.integers(0, pool.size, sz)]
    ns = k(0.8)
    sub = np.stack([pick(np.concatenate([[1], cls]), ns), pick(np.concatenate([[0], cls]), ns)], 1)
    conj = []
    for _ in range(k(0.25)):
        ar = int(rng.integers(1, 4))
        ops = pick(np.concatenate([[1], cls]), ar).tolist()
        rhs = int(pick(np.concatenate([[0], cls]), 1)[0]) if rng.random() > 0.1 else 0
        conj.append((ops, rhs))
    R = n_roles
    ne = k(0.5)
    fill_pool = np.concatenate([cls, dts, [1]]) if dts.size else np.concatenate([cls, [1]])
    ex_rhs = np.stack([pick(np.concatenate([[1], cls]), ne), rng.integers(0, R, ne), pick(fill_pool, ne)], 1)
    nl = k(0.3)
    ex_lhs = np.stack([rng.integers(0, R, nl), pick(np.concatenate([[1], cls, dts]), nl),
                       pick(np.concatenate([[0], cls]), nl)], 1)
    nsr = int(rng.poisson(0.6 * R * density))
    subrole = np.stack([rng.integers(0, R, nsr), rng.integers(0, R, nsr)], 1)
    nch = int(rng.poisson(0.5 * R * density))
    chain = np.stack([rng.integers(0, R, nch), rng.integers(0, R, nch), rng.integers(0, R, nch)], 1)
    nd = int(rng.poisson(0.3 * R))
    domain = np.stack([rng.integers(0, R, nd), pick(cls, nd)], 1) if cls.size else np.zeros((0, 2))
    nr = int(rng.poisson(0.2 * R))
    rng_ax = np.stack([rng.integers(0, R, nr), pick(cls, nr)], 1) if cls.size else np.zeros((0, 2))
    return Axioms.build(N, R, kind=kind, sub=sub, conj=conj, ex_rhs=ex_rhs, ex_lhs=ex_lhs, subrole=subrole,
                        chain=chain, domain=domain, range=rng_ax)
