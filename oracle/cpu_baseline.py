"""CPU baseline for bench.py (TEST INFRASTRUCTURE: the CPU oracle timed, never the product).

Run as a child process of bench.py, so that no process that touched the GPU forks: this
process imports no GPU code, generates the workload and classifies it with the CPU oracle
(oracle/el_oracle.c, semi-naive Jacobi, one thread per classification) on P worker
processes at once — P concurrent classifications, one per host core, which is what P cores
of the host sustain on this metric (the reference itself, Java + Redis, cannot run here).
The fastest of the P runs is also reported as the one-core figure, with its index build
(elo_create: the told closure and the rows over it, the GPU's el_init work) split out.

Usage: python oracle/cpu_baseline.py WORKLOAD SCALE PROCS  ->  one JSON line on stdout.
"""
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def _one(args):
    workload, scale = args
    import oracle
    from distel_amd import generators
    ax = generators.workload(workload, scale)
    t0 = time.perf_counter()
    o = oracle.Oracle(ax, 0)  # elo_create: the index incl. the told closure and its rows
    t1 = time.perf_counter()
    o.init()
    o.saturate()
    dt = time.perf_counter() - t0
    d = o.stats()["derived"]
    o.close()
    return t0, t0 + dt, dt, d, t1 - t0


def main():
    workload, scale, procs = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
    ctx = mp.get_context("fork")      # this process never touched a GPU
    with ctx.Pool(procs) as pool:
        runs = pool.map(_one, [(workload, scale)] * procs)
    wall = max(r[1] for r in runs) - min(r[0] for r in runs)
    derived = sum(r[3] for r in runs)
    single = min(runs, key=lambda r: r[2])  # the fastest classification: the 1-core figure
    print(json.dumps({"single_s": single[2], "single_derived": single[3], "single_create_s": single[4],
                      "procs": procs, "wall_s": wall,
                      "derived": derived, "per_run_s": [round(r[2], 4) for r in runs]}))


if __name__ == "__main__":
    main()
