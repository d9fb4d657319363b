#!/usr/bin/env python3
"""Row-partitioned (exchange) path diagnostics on ONE GPU.

×k of a workload (OntologyMultiplier copies) on k row partitions aligned with the copies, in ONE
process (EL_XCHG_LOCAL: one thread per partition, the same collective supersteps as RCCL), beside
the whole-ontology classification of one copy.  Every engine runs with HIP-event kernel timing
(profile mode).  Per classification and rank: el_init / el_saturate (+ streamed result) wall,
supersteps, exchange bytes received, and the per-kernel table.  One JSON line per leg.

    python scripts/part_diag.py [workload] [scale] [copies] [steps]
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distel_amd import engine, generators, ir  # noqa: E402


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
    base = generators.workload(wl, scale)
    e = engine.Engine(device=0, profile=True)
    e.load(base)
    out = engine.Stream()
    for s in range(steps):
        r = classify(e, out)
        r.update(leg="whole", step=s)
        print(json.dumps(r), flush=True)
    e.close()

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
    print(json.dumps({"leg": "load", "s": round(time.time() - t, 3)}), flush=True)
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
        print(json.dumps({"leg": f"x{k}", "step": s, "wall_ms": round(1e3 * wall, 3),
                          "derived": sum(r["derived"] for r in res), "ranks": res}), flush=True)
    for x in engs:
        x.close()
    group.close()


if __name__ == "__main__":
    main()
