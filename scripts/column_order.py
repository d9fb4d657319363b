#!/usr/bin/env python3
"""How many distinct bit-matrix lines the S commits touch under other column orders (CPU, from
the oracle's fact log): per superstep, distinct 128-B lines of the new facts with the column of a
concept = its id (the engine's order), its rank by told-descendant count (a predictor computable
from the told axioms: how many concepts have it in their told closure, i.e. the init facts), and
its rank by final frequency (how many rows hold it at the fixpoint: the ideal, a result of the
saturation).  Usage: scripts/column_order.py [workload] [scale]  ->  JSON on stdout."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from distel_amd import generators  # noqa: E402


def rank_of(counts):
    order = np.argsort(-counts, kind="stable")
    r = np.empty_like(order)
    r[order] = np.arange(order.size)
    return r.astype(np.uint64)


def main():
    workload = sys.argv[1] if len(sys.argv) > 1 else "g3"
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    ax = generators.workload(workload, scale)
    o = oracle.saturate(ax, 0)
    n = int(o.lib.elo_num_facts(o.ctx))
    x = np.zeros(n, np.uint32)
    a = np.zeros(n, np.uint32)
    import ctypes as C
    p = lambda v: v.ctypes.data_as(C.POINTER(C.c_uint32))
    o.lib.elo_copy_log(o.ctx, p(x), p(a), n)
    ds, _, _ = o.trace()
    o.close()
    N = ax.n_concepts
    n_init = int(ds[0])  # (the oracle's step 0: the init facts, X ∈ S(X), ⊤ and the told closure)
    words = ((N + 31) // 32 + 3) // 4 * 4
    told_desc = np.bincount(a[:n_init], minlength=N).astype(np.float64)  # rows holding A after init
    # conclusions of CR4 (∃r.A ⊑ B) and CR2 (⊓ ⊑ B) and their told closures: (B, A) init pairs
    concl = np.bincount(ax.ex_lhs[:, 2].astype(np.int64), minlength=N).astype(np.float64) + \
        np.bincount(ax.conj_b.astype(np.int64), minlength=N)
    # existential fillers: A ⊑ ∃r.B makes (X, B)-links, the CR4 inputs
    fill = np.bincount(ax.ex_rhs[:, 2].astype(np.int64), minlength=N).astype(np.float64)
    xi, ai = x[:n_init].astype(np.int64), a[:n_init].astype(np.int64)
    up = lambda w: np.bincount(ai, weights=w[xi], minlength=N)  # Σ over B with A ∈ told*(B) of w(B)
    # CR4 conclusion volume: ∃r.A ⊑ B concludes B for every X with an r-link to a Y holding A, so
    # B's expected rows ~ (rows holding A after init) × (r-links per concept, from A ⊑ ∃r.C axioms)
    R = int(max(ax.ex_rhs[:, 1].max(initial=0), ax.ex_lhs[:, 0].max(initial=0))) + 1
    nr = np.bincount(ax.ex_rhs[:, 1].astype(np.int64), minlength=R).astype(np.float64)
    el = ax.ex_lhs.astype(np.int64)
    vol = np.bincount(el[:, 2], weights=told_desc[el[:, 1]] * nr[el[:, 0]], minlength=N)
    # the same with told-descendant counts from the told DAG alone (no closure: desc(B) = 1 + Σ over
    # told subs A of desc(A), multiple inheritance over-counted; cycles left at their own count)
    sub = ax.sub.astype(np.int64)
    nsub = np.bincount(sub[:, 1], minlength=N)
    order_e = np.argsort(sub[:, 0], kind="stable")
    ptr = np.zeros(N + 1, np.int64)
    np.add.at(ptr, sub[:, 0] + 1, 1)
    ptr = np.cumsum(ptr)
    sup = sub[order_e, 1]
    dag = np.ones(N)
    pending = nsub.copy()
    stack = list(np.nonzero(pending == 0)[0])
    while stack:
        A = stack.pop()
        for B in sup[ptr[A]:ptr[A + 1]]:
            dag[B] += dag[A]
            pending[B] -= 1
            if pending[B] == 0:
                stack.append(B)
    vol_dag = np.bincount(el[:, 2], weights=dag[el[:, 1]] * nr[el[:, 0]], minlength=N)
    def hot_front(score, k):  # the k highest-scoring concepts first, everyone else in id order
        hot = np.argsort(-score, kind="stable")[:k]
        key = np.arange(N, dtype=np.float64) + k
        key[hot] = np.arange(k)
        return rank_of(-key)
    orders = {
        "dag_hot4k": hot_front(vol_dag, 4096),
        "dag_hot16k": hot_front(vol_dag, 16384),
        "dag_hot64k": hot_front(vol_dag, 65536),
        "cr4_volume_dag": rank_of(vol_dag + dag),
        "cr4_volume_up": rank_of(up(vol) + told_desc),
        "cr4_volume": rank_of(vol + told_desc),
        "id": np.arange(N, dtype=np.uint64),
        "told_descendants": rank_of(told_desc),
        "conclusions_up": rank_of(up(concl)),
        "conclusions_x_desc_up": rank_of(up(concl * told_desc)),
        "conclusions_up_plus_desc": rank_of(up(concl) * 1000 + told_desc),
        "final_frequency": rank_of(np.bincount(a, minlength=N)),
    }
    out = {"workload": workload, "scale": scale, "concepts": N, "facts": n, "init": n_init, "orders": {}}
    for name, col in orders.items():
        steps, pos = [], 0
        for d in ds.tolist():
            bit = x[pos:pos + d].astype(np.uint64) * np.uint64(32 * words) + col[a[pos:pos + d]]
            steps.append(int(np.unique(bit >> np.uint64(10)).size))
            pos += d
        allbits = x.astype(np.uint64) * np.uint64(32 * words) + col[a]
        out["orders"][name] = {"lines128_per_step": steps, "lines128_total": int(sum(steps)),
                               "lines128_final": int(np.unique(allbits >> np.uint64(10)).size)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
