"""Set-level model of the row-partitioned saturation protocol.  TEST INFRASTRUCTURE ONLY.

This restates, with Python sets on tiny inputs, exactly the exchange protocol the HIP
engine runs when a context owns only the rows [lo, hi) of S (el_config.part_*,
SURVEY.md §8(e)).  It exists so the protocol itself — what is exchanged, when, and why
the union of the partitions is the same closure as one engine — is checked on the CPU
(in-process ranks, and world-size-2 gloo ranks) independently of the kernels.

Per rank q (owner of the concepts X in [lo_q, hi_q)):

* local state  S(X) for owned X; links (X, r, Y) for owned X; preds[(r, Y)] = {owned X};
* replicated   props {((r, Y), B)} (CR4 half-1 records, Type3_1AxiomProcessorBase.java:
               208-234); range activations {(Y, C)} (RolePairHandler.java:471-479);
               chain links {(Y, s, Z)} with s the second role of some chain
               (the successor lists CR6 reads, Type5AxiomProcessorBase.java:115-154).

One Jacobi superstep reads only the state after step t-1 and the deltas of t-1:

  ΔS (X, A)      CR1, CR2, CR3 (row-local); CR4 half-1 → props ((r, X), B) for ∃r.A ⊑ B;
                 A = ⊥ → props ((r, X), ⊥) for every role (⊥ rides the CR4 machinery, so no
                 rank ever reads a row it does not own); A = Y with an active range (Y, C)
  Δlinks         CR4 half-2 (props of (r, Y)), CR5, CR6 with r first (chain links of Y),
                 domain, range activations
  Δprops         preds[(r, Y)] × {B}                 (Type3_2AxiomProcessor part 1)
  Δacts          owned X with Y ∈ S(X) get C          (K10, ScriptsCollection.java:45-62)
  Δchain links   (X, r, Y), r second of p ∘ r ⊑ t: preds[(p, X)] × (·, t, Y)

then commits locally — its own new props, activations and chain links join its replicated
sets at once — and ALL-GATHERS those some OTHER rank can use (the delta exchange of SURVEY.md
§8(e)): a record keyed by concept y (((r, y), B), (y, C), (y, s, z)) only matters to a rank whose
rows can reach y, i.e. y in its column window (el_ctx::column_window: the span of every concept
its rows can hold), so only those are sent; every rank imports the others'.  The fixpoint is
reached when the sum over ranks of all local deltas (and records sent) is zero (the
all-gathered counts double as the termination reduction, CommunicationHandler.java:49-84).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, Dict, List, Sequence, Set, Tuple

BOTTOM, TOP = 0, 1
DATATYPE = 3


def ranges(n: int, parts: int) -> List[Tuple[int, int]]:
    """Contiguous row ranges, as equal as possible."""
    return [(n * q // parts, n * (q + 1) // parts) for q in range(parts)]


class _Static:
    def __init__(self, ax):
        self.n = ax.n_concepts
        self.kind = [int(k) for k in ax.kind]
        self.roles = list(range(ax.n_roles))
        self.told = defaultdict(list)
        for a, b in ax.sub:
            self.told[int(a)].append(int(b))
        self.conj_of = defaultdict(list)
        for i in range(ax.n_conj):
            ops = [int(o) for o in ax.conj_ops[ax.conj_ptr[i]:ax.conj_ptr[i + 1]]]
            for o in set(ops):
                self.conj_of[o].append((ops, int(ax.conj_b[i])))
        self.exr = defaultdict(list)
        for a, r, b in ax.ex_rhs:
            self.exr[int(a)].append((int(r), int(b)))
        self.exl = defaultdict(list)
        for r, a, b in ax.ex_lhs:
            self.exl[int(a)].append((int(r), int(b)))
        self.sup = defaultdict(list)
        for r, s in ax.subrole:
            self.sup[int(r)].append(int(s))
        self.chf = defaultdict(list)   # r first:  (s, t)
        self.chs = defaultdict(list)   # s second: (r, t)
        for r, s, t in ax.chain:
            self.chf[int(r)].append((int(s), int(t)))
            self.chs[int(s)].append((int(r), int(t)))
        self.dom = defaultdict(list)
        for r, d in ax.domain:
            self.dom[int(r)].append(int(d))
        self.rng = defaultdict(list)
        for r, c in ax.range:
            self.rng[int(r)].append(int(c))

    def plain(self, x: int) -> bool:
        return x != TOP and self.kind[x] != DATATYPE


class Rank:
    def __init__(self, ax, lo: int, hi: int):
        self.k = _Static(ax)
        self.lo, self.hi = lo, hi
        self.win = self._window()
        self.others: List[Tuple[int, int]] = []  # the other ranks' windows (set_windows)
        self.S: Dict[int, Set[int]] = {}
        self.links: Set[Tuple[int, int, int]] = set()
        self.preds: Dict[Tuple[int, int], Set[int]] = defaultdict(set)
        self.props: Dict[Tuple[int, int], Set[int]] = defaultdict(set)
        self.acts: Set[Tuple[int, int]] = set()
        self.succ: Dict[int, Set[Tuple[int, int]]] = defaultdict(set)   # Y -> {(s, Z)} chain links
        self.dS: List[Tuple[int, int]] = []
        self.dL: List[Tuple[int, int, int]] = []
        self.dP: List[Tuple[Tuple[int, int], int]] = []
        self.dA: List[Tuple[int, int]] = []
        self.dX: List[Tuple[int, int, int]] = []
        for x in range(lo, hi):  # AxiomLoader.java:1237-1245, individuals :1281-1289
            self.S[x] = {x}
            self.dS.append((x, x))
            if self.k.plain(x) and x != BOTTOM:
                self.S[x].add(TOP)
                self.dS.append((x, TOP))

    def _window(self) -> Tuple[int, int]:
        """[c_lo, c_hi): the span of every concept the owned rows can hold — closed under told
        supers, conjunction conclusions, existential fillers and CR4 conclusions, and the domains
        and ranges of every role their links can carry (an existential's role, its super-roles and
        the chains' results), as el_ctx::column_window computes it."""
        k = self.k
        seen = set(range(self.lo, self.hi)) | {BOTTOM, TOP}
        stack = sorted(seen)  # (⊥ and ⊤ are in every row: their closures too)
        roles, rstack = set(), []

        def add(c):
            if c not in seen:
                seen.add(c)
                stack.append(c)

        def add_role(r):
            if r not in roles:
                roles.add(r)
                rstack.append(r)
        while stack or rstack:
            if stack:
                a = stack.pop()
                for b in k.told[a]:
                    add(b)
                for _, b in k.conj_of[a]:
                    add(b)
                for r, b in k.exr[a]:
                    add(b)
                    add_role(r)
                for _, b in k.exl[a]:
                    add(b)
                continue
            r = rstack.pop()
            for s in k.sup[r]:
                add_role(s)
            for _, t in k.chf[r]:
                add_role(t)
            for _, t in k.chs[r]:
                add_role(t)
            for c in k.dom[r] + k.rng[r]:
                add(c)
        inner = [c for c in seen if c >= 2]
        return (min(inner), max(inner) + 1) if inner else (2, 2)

    def set_windows(self, wins: Sequence[Tuple[int, int, Tuple[int, int]]]) -> None:
        """Every rank's (lo, hi, window), all-gathered once (el_ctx::exchange_windows)."""
        self.others = [w for lo, hi, w in wins if (lo, hi) != (self.lo, self.hi)]

    def remote(self, y: int) -> bool:
        """Some other rank's rows can reach concept y (⊥ and ⊤ are in every window)."""
        return any(y < 2 or lo <= y < hi for lo, hi in self.others)

    # -- generation + local commit; returns the records to all-gather
    def step(self):
        k, S = self.k, self.S
        cs: Set[Tuple[int, int]] = set()
        cl: Set[Tuple[int, int, int]] = set()
        cp: Set[Tuple[Tuple[int, int], int]] = set()
        ca: Set[Tuple[int, int]] = set()
        for x, a in self.dS:
            for b in k.told[a]:
                cs.add((x, b))
            for ops, b in k.conj_of[a]:
                if all(o in S[x] for o in ops):
                    cs.add((x, b))
            for r, b in k.exr[a]:
                cl.add((x, r, b))
            for r, b in k.exl[a]:
                cp.add(((r, x), b))
            if a == BOTTOM:
                for r in k.roles:
                    cp.add(((r, x), BOTTOM))
            for (y, c) in self.acts:
                if y == a:
                    cs.add((x, c))
        for x, r, y in self.dL:
            for b in self.props[(r, y)]:
                cs.add((x, b))
            for s in k.sup[r]:
                cl.add((x, s, y))
            for s, t in k.chf[r]:
                for s2, z in self.succ[y]:
                    if s2 == s:
                        cl.add((x, t, z))
            if k.plain(x):
                for d in k.dom[r]:
                    cs.add((x, d))
            if k.plain(y):
                for c in k.rng[r]:
                    ca.add((y, c))
        for pid, b in self.dP:
            for x in self.preds[pid]:
                cs.add((x, b))
        for y, c in self.dA:
            for x in range(self.lo, self.hi):
                if y in S[x]:
                    cs.add((x, c))
        for x, r, y in self.dX:
            for p, t in k.chs[r]:
                for x2 in self.preds[(p, x)]:
                    cl.add((x2, t, y))
        # commit
        self.dS = sorted(f for f in cs if f[1] not in S[f[0]])
        for x, a in self.dS:
            S[x].add(a)
        self.dL = sorted(l for l in cl if l not in self.links)
        for x, r, y in self.dL:
            self.links.add((x, r, y))
            self.preds[(r, y)].add(x)
        new_p = sorted(p for p in cp if p[1] not in self.props[p[0]])
        new_a = sorted(a for a in ca if a not in self.acts)
        new_x = [l for l in self.dL if k.chs[l[1]]]
        self._own = (new_p, new_a, new_x)
        return {"props": [p for p in new_p if self.remote(p[0][1])], "acts": [a for a in new_a if self.remote(a[0])],
                "xlinks": [l for l in new_x if self.remote(l[0])], "ds": len(self.dS), "dl": len(self.dL),
                "dp": len(new_p), "da": len(new_a), "dx": len(new_x), "rows": (self.lo, self.hi)}

    # -- this rank's own new records, then the other ranks' records it was sent
    def absorb(self, gathered: Sequence[dict]) -> int:
        dP, dA, dX = [], [], []
        own_p, own_a, own_x = self._own
        for pid, b in own_p:
            self.props[pid].add(b)
            dP.append((pid, b))
        for y, c in own_a:
            self.acts.add((y, c))
            dA.append((y, c))
        for x, r, y in own_x:
            self.succ[x].add((r, y))
            dX.append((x, r, y))
        for g in gathered:
            if g["rows"] == (self.lo, self.hi):
                continue
            for pid, b in g["props"]:
                if b not in self.props[pid]:
                    self.props[pid].add(b)
                    dP.append((pid, b))
            for y, c in g["acts"]:
                if (y, c) not in self.acts:
                    self.acts.add((y, c))
                    dA.append((y, c))
            for x, r, y in g["xlinks"]:
                self.succ[x].add((r, y))
                dX.append((x, r, y))
        self.dP, self.dA, self.dX = dP, dA, dX
        return sum(g["ds"] + g["dl"] + g["dp"] + g["da"] + g["dx"] + len(g["props"]) + len(g["acts"]) +
                   len(g["xlinks"]) for g in gathered)


def run(rank: Rank, allgather: Callable[[object], List[object]], max_steps: int = 100000) -> int:
    """Drive one rank to the global fixpoint (after the one-time window exchange); returns the
    superstep count."""
    rank.set_windows(allgather((rank.lo, rank.hi, rank.win)))
    for t in range(1, max_steps + 1):
        if rank.absorb(allgather(rank.step())) == 0:
            return t
    raise RuntimeError("no fixpoint")


def saturate_inprocess(ax, parts: int, compat_range: bool = True):
    """All ranks in one process, in lock-step.  Returns (S, R, supersteps) as plain sets.
    The model's range rule is DistEL's (compat_range); compat_range=False reads ranges ELK's
    way, as the engine does by default: the ontology goes through distel_amd.ir.elk_ranges and
    the fresh fillers' rows are left out."""
    n_user = ax.n_concepts
    if not compat_range:
        from distel_amd import ir
        ax = ir.elk_ranges(ax)[0]
    rs = [Rank(ax, lo, hi) for lo, hi in ranges(ax.n_concepts, parts)]
    wins = [(r.lo, r.hi, r.win) for r in rs]
    for r in rs:
        r.set_windows(wins)
    t = 0
    while True:
        t += 1
        out = [r.step() for r in rs]
        tot = [r.absorb(out) for r in rs]
        assert len(set(tot)) == 1
        if tot[0] == 0:
            break
    S: Dict[int, Set[int]] = {}
    R: Set[Tuple[int, int, int]] = set()
    for r in rs:
        S.update(r.S)
        R |= r.links
    S = {x: v for x, v in S.items() if x < n_user}
    R = {l for l in R if l[0] < n_user}
    return S, R, t
