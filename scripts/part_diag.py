#!/usr/bin/env python3
"""Row-partitioned (exchange) path diagnostics on ONE GPU.

weak (default): ×k of a workload (OntologyMultiplier copies) on k row partitions aligned with the
copies; strong: the workload itself (ONE ontology) on k unaligned row partitions balanced by told
edges (ir.balanced_rows), with the union's closure digest checked against
tests/golden/closure_digests.txt.  In ONE process (EL_XCHG_LOCAL: one thread per partition, the
same collective supersteps as RCCL), beside the whole-ontology classification of one copy.  Every engine runs with HIP-event kernel timing
(profile mode).  Per classification and rank: el_init / el_saturate (+ streamed result) wall,
supersteps, exchange bytes received, and the per-kernel table.  One JSON line per leg.

    python scripts/part_diag.py [workload] [scale] [copies] [steps] [weak|strong]
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distel_amd import engine, generators, ir  # noqa: E402


def mem_used_gb():
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")
        free, total = ctypes.c_size_t(0), ctypes.c_size_t(0)
        hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
        return round((total.value - free.value) / 1e9, 2)
    except OSError:
        return None


def pinned_digest(wl, scale, ax):
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "closure_digests.txt")
    want = None
    for line in open(path):
        if line.strip() and not line.startswith("#"):
            n, sc, d_in, d_out = line.split()
            if n == wl and float(sc) == scale and d_in == ax.digest():
                want = d_out
    return want


def union_digest(engs):
    import hashlib
    import numpy as np
    h = hashlib.sha256()  # (ascending disjoint row ranges: the sorted rows concatenate in rank order)
    facts = [e.facts() for e in engs]
    links = [e.links() for e in engs]
    for k in range(2):
        h.update(np.concatenate([f[k] for f in facts]).astype(np.uint32).tobytes())
    for k in range(3):
        h.update(np.concatenate([l[k] for l in links]).astype(np.uint32).tobytes())
    return h.hexdigest()


def kernels(e):
    return {k["kernel"]: [k["launches"], round(k["ms"], 3)] for k in e.kernel_stats() if k["launches"]}


def classify(e, out):
    t0 = time.perf_counter()
    e.init()
    t1 = time.perf_counter()
    e.stream_result(out, release=False)
    st = e.saturate()
    t2 = time.perf_counter()
    e.result_wait()
    t3 = time.perf_counter()
    return {"init_ms": round(1e3 * (t1 - t0), 3), "saturate_ms": round(1e3 * (t2 - t1), 3),
            "tail_ms": round(1e3 * (t3 - t2), 3), "supersteps": st["supersteps"], "derived": st["derived"],
            "exchange_bytes": st.get("exchange_bytes", 0), "kernels": kernels(e)}


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "g3"
    scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    mode = sys.argv[5] if len(sys.argv) > 5 else "weak"
    base = generators.workload(wl, scale)
    e = engine.Engine(device=0, profile=True)
    e.load(base)
    out = engine.Stream()
    for s in range(steps):
        r = classify(e, out)
        r.update(leg="whole", step=s)
        print(json.dumps(r), flush=True)
    e.close()

    if mode == "strong":
        ax = base
        bounds = ir.balanced_rows(base, k)
    else:
        ax = ir.replicate(base, k)
        bounds = [ir.copy_slice(base, k, i) for i in range(k)]
        bounds[0] = (0, bounds[0][1])
    group = engine.LocalGroup(k)
    engs = [engine.Engine(device=0, profile=True,
                          partition=engine.Partition(q, k, engine.XCHG_LOCAL, group=group, rows=bounds[q]))
            for q in range(k)]
    t = time.time()
    for x in engs:
        x.load(ax)
    print(json.dumps({"leg": "load", "mode": mode, "rows": bounds, "s": round(time.time() - t, 3),
                      "mem_gb": mem_used_gb()}), flush=True)
    outs = [engine.Stream() for _ in range(k)]
    for s in range(steps):
        res = [None] * k
        errs = []

        def run(q):
            try:
                res[q] = classify(engs[q], outs[q])
            except BaseException as exc:  # noqa: BLE001
                errs.append(exc)
        th = [threading.Thread(target=run, args=(q,)) for q in range(k)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        wall = time.perf_counter() - t0
        if errs:
            raise errs[0]
        print(json.dumps({"leg": f"{mode}{k}", "step": s, "wall_ms": round(1e3 * wall, 3),
                          "derived": sum(r["derived"] for r in res), "mem_gb": mem_used_gb(), "ranks": res}),
              flush=True)
    if mode == "strong":
        want = pinned_digest(wl, scale, base)
        got = union_digest(engs)
        print(json.dumps({"leg": "digest", "pinned": want, "union": got, "equal": want == got}), flush=True)
    for x in engs:
        x.close()
    group.close()


if __name__ == "__main__":
    main()
