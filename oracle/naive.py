"""Pure-Python naive EL+ fixpoint.  TEST INFRASTRUCTURE ONLY (tiny inputs).

A third, deliberately literal restatement of the completion rules, written set
by set so it reads like the reference's rule kernels (file:line per rule).  It
is used to cross-check the C oracle on the known-answer tests.
"""
from __future__ import annotations

from typing import Dict, Set, Tuple

BOTTOM, TOP = 0, 1
DATATYPE = 3


def saturate(ax, distel_chain: bool = False,
             distel_range: bool = False) -> Tuple[Dict[int, Set[int]], Set[Tuple[int, int, int]]]:
    """distel_chain: CR6 as DistEL runs it (hazard H2), restated literally from the store
    layout: DB1["Yr"] holds X for (X,Y) in R(r), r first in a chain; DB4["Yr"] holds Z for
    (Y,Z) in R(s), s second in a chain whose FIRST role is r (RolePairHandler.java:395-443);
    CR6 adds (X,Z) to the t of every chain whose first role is r, without checking s
    (Type5AxiomProcessorBase.java:128-143)."""
    if not distel_range and len(ax.range):
        # ranges read ELK's way: normalize them away first (distel_amd.ir.elk_ranges); the
        # fresh fillers' rows are internal
        from distel_amd import ir
        n_user = ax.n_concepts
        S, R = saturate(ir.elk_ranges(ax)[0], distel_chain, True)
        return {x: v for x, v in S.items() if x < n_user}, {t for t in R if t[0] < n_user}
    n = ax.n_concepts
    kind = [int(k) for k in ax.kind]
    # init: S(X) = {X, ⊤}  (AxiomLoader.java:1237-1245, individuals :1281-1289)
    S: Dict[int, Set[int]] = {}
    for x in range(n):
        S[x] = {x}
        if x not in (TOP, BOTTOM) and kind[x] != DATATYPE:
            S[x].add(TOP)
    R: Set[Tuple[int, int, int]] = set()  # (x, r, y): (x, y) ∈ R(r)
    sub = [tuple(map(int, t)) for t in ax.sub]
    conj = [([int(o) for o in ax.conj_ops[ax.conj_ptr[i]:ax.conj_ptr[i + 1]]], int(ax.conj_b[i]))
            for i in range(ax.n_conj)]
    ex_rhs = [tuple(map(int, t)) for t in ax.ex_rhs]
    ex_lhs = [tuple(map(int, t)) for t in ax.ex_lhs]
    subrole = [tuple(map(int, t)) for t in ax.subrole]
    chain = [tuple(map(int, t)) for t in ax.chain]
    domain = [tuple(map(int, t)) for t in ax.domain]
    rng = [tuple(map(int, t)) for t in ax.range]
    changed = True
    while changed:
        before = (sum(len(s) for s in S.values()), len(R))
        for x in range(n):
            for a, b in sub:  # CR1  Type1_1AxiomProcessorBase.java:22-43
                if a in S[x]:
                    S[x].add(b)
            for ops, b in conj:  # CR2  Type1_2AxiomProcessorBase.java:45-66
                if all(o in S[x] for o in ops):
                    S[x].add(b)
            for a, r, b in ex_rhs:  # CR3  Type2AxiomProcessorBase.java:45-75
                if a in S[x]:
                    R.add((x, r, b))
        for (x, r, y) in list(R):
            for rr, a, b in ex_lhs:  # CR4  Type3_2AxiomProcessorBase.java:67-96
                if rr == r and a in S[y]:
                    S[x].add(b)
            for r1, s in subrole:  # CR5  Type4AxiomProcessorBase.java:38-76
                if r1 == r:
                    R.add((x, s, y))
            if distel_chain:  # CR6 over the "Yr" keys (H2)
                seconds = {s for r1, s, _ in chain if r1 == r}
                thirds = {t for r1, _, t in chain if r1 == r}
                db4 = {z for (y2, s2, z) in R if y2 == y and s2 in seconds}
                for t in thirds:
                    for z in db4:
                        R.add((x, t, z))
            else:
                for r1, s, t in chain:  # CR6  Type5AxiomProcessorBase.java:115-154 (s checked)
                    if r1 == r:
                        for (y2, s2, z) in list(R):
                            if y2 == y and s2 == s:
                                R.add((x, t, z))
            if BOTTOM in S[y]:  # ⊥  TypeBottomAxiomProcessorBase.java:62-123
                S[x].add(BOTTOM)
            for r1, d in domain:  # domain  RolePairHandler.java:480-490
                if r1 == r and x != TOP and kind[x] != DATATYPE:
                    S[x].add(d)
            for r1, c in rng:  # range, DistEL's reading (H1, closed)  RolePairHandler.java:471-479
                if r1 == r and y != TOP and kind[y] != DATATYPE:
                    for z in range(n):
                        if y in S[z]:
                            S[z].add(c)
        changed = (sum(len(s) for s in S.values()), len(R)) != before
    return S, R
