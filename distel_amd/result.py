"""Result-node output format (the engine's output boundary).

The reference keeps the classification on one result node: DB0 holds, for every
subsumer B, a ZSET ``B -> {X : B ∈ S(X)}`` keyed by packed ids
(``kc/init/AxiomLoader.java:1237-1245``); ``ResultRearranger`` flips it into DB1
``X -> {B}`` plus a ``resultKeys`` set (``kc/test/ResultRearranger.java:57-105``)
and ``ELClassifierTest.writeResultsToFile`` prints ``X|B`` lines to
``final-saxioms-distel.txt`` (``kc/test/ELClassifierTest.java:448-469``).  This
module produces the same layouts from the engine's facts:

* packed ids: 2-digit decimal length, decimal id, 1-digit EntityType
  (``kc/misc/Util.java:95-103``), e.g. ⊤ = ``"0110"``, ⊥ = ``"0100"``;
* DistEL's id assignment order (``AxiomLoader.mapConceptToID`` :1155-1341):
  ⊤ = 1, classes from 2, then individuals, then object properties, then
  datatypes; ⊥ keeps BOTTOM_ID 0;
* with ``distel_compat=True`` the individuals' ``⊥ ⊑ a`` entries the loader
  writes (H7, ``AxiomLoader.java:1284-1289``) are added to the result node;
* ``axiom_counter`` = ``AxiomCounter.getAxiomCountAfterClassification``
  (``kc/output/analysis/AxiomCounter.java:168-216``): Σ ZCARD over result keys and
  Σ |R(r)|.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np

from .ir import Axioms, BOTTOM, KIND_CLASS, KIND_DATATYPE, KIND_INDIVIDUAL, KIND_ROLE, TOP


def packed_id(num: int, entity_type: int) -> str:
    """``Util.getPackedID`` (kc/misc/Util.java:95-103)."""
    s = str(int(num))
    return f"{len(s):02d}{s}{int(entity_type)}"


def unpack_ids(packed: str) -> List[str]:
    """``Util.unpackIDs`` (kc/misc/Util.java:105-117)."""
    out, i = [], 0
    while i < len(packed):
        n = int(packed[i:i + 2]) + 3
        out.append(packed[i:i + n])
        i += n
    return out


def distel_numbering(ax: Axioms) -> Tuple[np.ndarray, np.ndarray]:
    """DistEL counter ids for concepts and roles, in mapConceptToID order."""
    n = ax.n_concepts
    ids = np.zeros(n, dtype=np.int64)
    ids[BOTTOM], ids[TOP] = 0, 1
    nxt = 2
    kind = ax.kind
    for want in (KIND_CLASS, KIND_INDIVIDUAL):
        sel = np.nonzero(kind[2:] == want)[0] + 2
        ids[sel] = np.arange(nxt, nxt + sel.size)
        nxt += sel.size
    rids = np.arange(nxt, nxt + ax.n_roles, dtype=np.int64)
    nxt += ax.n_roles
    sel = np.nonzero(kind[2:] == KIND_DATATYPE)[0] + 2
    ids[sel] = np.arange(nxt, nxt + sel.size)
    return ids, rids


class ResultNode:
    """The classification in the reference's result-node shapes."""

    def __init__(self, ax: Axioms, fact_x: np.ndarray, fact_a: np.ndarray, distel_compat: bool = True):
        self.ax = ax
        kind = ax.kind
        keep = (fact_x != BOTTOM) & (kind[fact_x] != KIND_DATATYPE)  # result rows: classes, individuals
        x = fact_x[keep].astype(np.int64)
        a = fact_a[keep].astype(np.int64)
        if distel_compat:  # H7: individuals get ⊥ ⊑ a, i.e. result[a] ∋ ⊥
            ind = np.nonzero(kind == KIND_INDIVIDUAL)[0]
            x = np.concatenate([x, np.full(ind.size, BOTTOM)])
            a = np.concatenate([a, ind])
        order = np.lexsort((x, a))
        self.b_key, self.b_member = a[order], x[order]          # DB0: B -> {X}
        order = np.lexsort((a, x))
        self.x_key, self.x_member = x[order], a[order]          # DB1: X -> {B}
        self._num, self._rnum = distel_numbering(ax)

    # ------------------------------------------------------------ layouts
    def db0(self) -> Dict[int, np.ndarray]:
        """result node DB0: B -> sorted {X}."""
        return _group(self.b_key, self.b_member)

    def db1(self) -> Dict[int, np.ndarray]:
        """ResultRearranger DB1: X -> sorted {B}."""
        return _group(self.x_key, self.x_member)

    def pid(self, c: int) -> str:
        k = int(self.ax.kind[c])
        return packed_id(self._num[c], k)

    def name(self, c: int) -> str:
        return self.ax.concept_name(c)

    def saxiom_lines(self, use_names: bool = False) -> Iterable[str]:
        """``final-saxioms-distel.txt``: one ``X|B`` line per subsumption."""
        f = self.name if use_names else self.pid
        for x, b in zip(self.x_key.tolist(), self.x_member.tolist()):
            yield f"{f(x)}|{f(b)}"

    def write_saxioms(self, path: str, use_names: bool = False) -> int:
        n = 0
        with open(path, "w", encoding="utf-8") as out:
            for line in self.saxiom_lines(use_names):
                out.write(line + "\n")
                n += 1
        return n

    def axiom_counter(self, links: int) -> Dict[str, int]:
        """AxiomCounter totals: Σ ZCARD over result keys, Σ |R(r)|."""
        return {"total_subclass_axioms": int(self.b_key.size), "total_r_values": int(links)}


def _group(keys: np.ndarray, vals: np.ndarray) -> Dict[int, np.ndarray]:
    out: Dict[int, np.ndarray] = {}
    if keys.size == 0:
        return out
    cut = np.nonzero(np.diff(keys))[0] + 1
    for ks, vs in zip(np.split(keys, cut), np.split(vals, cut)):
        out[int(ks[0])] = vs
    return out


# ------------------------------------------------------------------ ELK diff
def read_saxioms(path: str) -> Dict[str, set]:
    """``X|B`` lines (``final-saxioms-distel.txt`` layout) → {X: {B}}."""
    out: Dict[str, set] = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            x, b = line.rsplit("|", 1)
            out.setdefault(x, set()).add(b)
    return out


BOTTOM_NAMES = ("owl:Nothing", "http://www.w3.org/2002/07/owl#Nothing", "<http://www.w3.org/2002/07/owl#Nothing>")


def diff_results(expected: Dict[str, set], got: Dict[str, set], bottom: Optional[str] = None,
                 top: Optional[str] = None, classes: Optional[Iterable[str]] = None) -> Tuple[int, List[str]]:
    """Per-class comparison as ``ELClassifierTest.rearrangeAndCompareResults``
    (kc/test/ELClassifierTest.java:363-447) / ``ResultDiffWriter.writeDiffResults``
    (kc/output/ResultDiffWriter.java:34-99): a class differs when its superclass sets
    differ.  ⊥ itself is skipped (:379-382); an unsatisfiable class (⊥ in either set)
    is compared on ⊥-membership only, since ELK lists every class as its superclass and
    DistEL only ⊥ (H4).  ``top`` (if given) is added to every expected set
    (the reasoner's answer omits owl:Thing, :390).  Returns (differing classes, report)."""
    keys = sorted(set(expected) | set(got)) if classes is None else sorted(classes)
    if bottom is None:  # whichever spelling of owl:Nothing the files use
        seen = set(expected) | set(got) | {b for v in list(expected.values()) + list(got.values()) for b in v}
        bottom = next((b for b in BOTTOM_NAMES if b in seen), BOTTOM_NAMES[0])
    misses, report = 0, []
    for x in keys:
        if x == bottom:
            continue
        want = set(expected.get(x, set())) | {x}
        if top is not None:
            want.add(top)
        have = set(got.get(x, set())) | {x}
        if bottom in want or bottom in have:
            if (bottom in want) != (bottom in have):
                misses += 1
                report.append(f"{x} -- unsatisfiable in {'expected' if bottom in want else 'result'} only")
            continue
        if want != have:
            misses += 1
            miss, extra = sorted(want - have), sorted(have - want)
            report.append(f"{x} -- {len(have)}, {len(want)}" + "".join(f"\n  {x} -ne- {b}" for b in miss) +
                          "".join(f"\n\t -- {b}" for b in extra))
    report.append(f"No of classes not equal: {misses}")
    return misses, report


def _mix64(k: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    k = k ^ (k >> np.uint64(33))
    k = k * np.uint64(0xFF51AFD7ED558CCD)
    k = k ^ (k >> np.uint64(33))
    k = k * np.uint64(0xC4CEB9FE1A85EC53)
    return k ^ (k >> np.uint64(33))


def set_digest(fx: np.ndarray, fa: np.ndarray, lx: np.ndarray, lr: np.ndarray, ly: np.ndarray) -> str:
    """Order-independent digest of a closure: the S facts (x, a) and the links (x, r, y) as sets.
    Each entry is hashed on its own (two independent 64-bit mixes) and the hashes are summed mod
    2^64, so the facts and links may come in any order (a streamed result's commit order, several
    partitions' rows) and nothing is sorted: O(entries), vectorised.  Duplicates are not removed
    (a closure has none).  Returns "<n_facts>:<n_links>:<16 hex digits> x 4"."""
    with np.errstate(over="ignore"):
        kf = (fx.astype(np.uint64) << np.uint64(32)) | fa.astype(np.uint64)
        kl = (lx.astype(np.uint64) << np.uint64(32)) | ly.astype(np.uint64)
        kl = _mix64(kl) ^ (lr.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        parts = []
        for k, salt in ((kf, 0x243F6A8885A308D3), (kl, 0x13198A2E03707344)):
            for s2 in (0, 0xA4093822299F31D0):
                h = _mix64(k ^ np.uint64(salt ^ s2))
                parts.append(int(h.sum(dtype=np.uint64)))
    return f"{fx.size}:{lx.size}:" + "".join(f"{p:016x}" for p in parts)
