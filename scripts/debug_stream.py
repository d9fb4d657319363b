"""GPU diagnostic: the streamed result over random ontologies on one reused engine (release on),
compared with the GPU's own facts() of a fresh engine; prints what differs (values, runs, counts).
Usage: python scripts/debug_stream.py [seeds]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from distel_amd import engine, generators  # noqa: E402


def main():
    seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    eng = engine.Engine(device=0)
    strm = engine.Stream()
    bad = 0
    for seed in range(seeds):
        ax = generators.random_small(4400 + seed, n=8 + seed % 50, n_roles=1 + seed % 4)
        ref = engine.Engine(device=0)
        ref.load(ax)
        ref.init()
        rst = ref.saturate()
        rx, ra = ref.facts()
        ref.close()
        eng.load(ax)
        eng.init()
        eng.stream_result(strm, release=True)
        st = eng.saturate()
        eng.result_wait()
        x, a = strm.facts(ax.n_concepts)
        ok = np.array_equal(x, rx) and np.array_equal(a, ra)
        if not ok:
            bad += 1
            xs, bs = strm.fact_rows()
            print(f"seed {seed}: n={ax.n_concepts} facts {strm.n_facts} (ref {rst['s_facts']}) runs {strm.n_s_runs} "
                  f"links {strm.n_links} runs {strm.n_l_runs}; stats {st['s_facts']} {st['links']}")
            runs = strm.s_run[:strm.n_s_runs]
            print("  runs[:12]", runs[:12].tolist())
            print("  values sorted equal:", np.array_equal(np.sort(bs), np.sort(ra)))
            print("  x multiset equal:", np.array_equal(np.sort(xs), np.sort(rx)))
            if bad > 3:
                break
    print("bad", bad, "of", seeds)
    eng.close()


if __name__ == "__main__":
    main()
