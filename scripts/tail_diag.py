#!/usr/bin/env python3
"""Copy-back tail diagnostics: per-classification init / saturate / tail
(el_result_wait after el_saturate returned) of the streamed result, for several engines run
one after another in ONE process — the schedule in which the tail was seen (a second engine, or
a bench leg after another leg).  Variants by argv: whole | part1 (one-rank LOCAL partition) |
rccl1 (one-rank RCCL partition).  Each engine classifies `steps` times; one JSON line per engine.

    python scripts/tail_diag.py g3 5 whole part1 whole rccl1 whole
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.path.exists("/opt/rocm/lib/libamdhip64.so.7") and os.environ.get("EL_HIP_RUNTIME", "system") == "system":
    import ctypes
    ctypes.CDLL("/opt/rocm/lib/libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
from distel_amd import engine, generators  # noqa: E402


def main():
    if os.environ.get("NUMA") == "1":  # bind every thread to the GPU's NUMA node, as bench.py does
        import bench
        print(json.dumps({"numa": bench.bind_gpu_numa(0)}), flush=True)
    wl = sys.argv[1]
    steps = int(sys.argv[2])
    ax = generators.workload(wl)
    keep = os.environ.get("KEEP_STREAMS") == "1"
    kept = []
    for i, kind in enumerate(sys.argv[3:]):
        if kind == "whole":
            e = engine.Engine(device=0)
        elif kind == "part1":
            e = engine.Engine(device=0, partition=engine.Partition(0, 1, engine.XCHG_LOCAL,
                                                                   group=engine.LocalGroup(1)))
        else:
            e = engine.Engine(device=0, partition=engine.Partition(0, 1, engine.XCHG_RCCL,
                                                                   rccl_id=engine.rccl_unique_id()))
        e.load(ax)
        out = engine.Stream()
        rows = []
        for s in range(steps):
            t0 = time.perf_counter()
            e.init()
            t1 = time.perf_counter()
            e.stream_result(out, release=True)
            e.saturate()
            t2 = time.perf_counter()
            e.result_wait()
            t3 = time.perf_counter()
            rows.append([round(1e3 * (t1 - t0), 2), round(1e3 * (t2 - t1), 2), round(1e3 * (t3 - t2), 2)])
        print(json.dumps({"engine": i, "kind": kind, "init_sat_tail_ms": rows}), flush=True)
        e.close()
        if keep:
            kept.append(out)


if __name__ == "__main__":
    main()
