#!/usr/bin/env python3
"""configs[3] shape at full size on ONE GPU: OntologyMultiplier ×8 of G3 (3.1 M concepts),
8 row partitions aligned with the copies in one process (EL_XCHG_LOCAL: the same exchange
protocol as RCCL, in-process all-gather), each with its compacted column window.  Prints one
JSON line: device memory per partition (hipMemGetInfo deltas), wall times, and the
size-independent check derived(×8) = 8 × derived(G3) (the copies share no concepts).

    python scripts/g4_full.py [scale] [copies]
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distel_amd import engine, generators, ir  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def used_gb():
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
    return (total.value - free.value) / 1e9


def heartbeat():
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(30)
            print(f"... {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    out = {"workload": f"G3 x{k} (scale {scale})", "copies": k}
    base = generators.workload("g3", scale=scale)
    u0 = used_gb()
    t = time.time()
    eng, st = engine.classify(base, device=0)
    out["g3_whole"] = {"derived": st["derived"], "supersteps": st["supersteps"], "device_gb": round(used_gb() - u0, 2),
                       "s": round(time.time() - t, 2)}
    eng.close()
    print(json.dumps(out), flush=True)
    ax = ir.replicate(base, k)
    bounds = [ir.copy_slice(base, k, i) for i in range(k)]
    bounds[0] = (0, bounds[0][1])
    u0 = used_gb()
    t = time.time()
    engs, sts = engine.classify_partitioned(ax, k, rows=bounds)
    wall = time.time() - t
    out["partitioned"] = {"concepts": ax.n_concepts, "derived": sum(s["derived"] for s in sts),
                          "supersteps": sorted({s["supersteps"] for s in sts}),
                          "device_gb_total": round(used_gb() - u0, 2),
                          "device_gb_per_partition": round((used_gb() - u0) / k, 2),
                          "load_plus_saturate_s": round(wall, 1)}
    out["check_derived_eq_k_times_g3"] = out["partitioned"]["derived"] == k * out["g3_whole"]["derived"]
    for e in engs:
        e.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
