"""Confirm the committed closure digests with the independent worklist saturator, and extend
them to larger workloads (TEST INFRASTRUCTURE: run on the CPU, minutes at full G3).

    python oracle/pin_digests.py [name:scale ...]     (default: every case below)

For each case: generator input digest, semi-naive oracle closure digest, worklist closure
digest; they must agree.  New agreeing cases are appended to tests/golden/closure_digests.txt;
the run is logged to tests/golden/pin_report.txt.
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE]
import oracle  # noqa: E402
import worklist  # noqa: E402
from distel_amd import generators  # noqa: E402

CASES = [("g1", 1.0), ("g2", 1.0), ("g3", 0.1), ("g5", 0.3), ("g5", 1.0), ("g3", 1.0)]
DIGESTS = os.path.join(ROOT, "tests", "golden", "closure_digests.txt")
REPORT = os.path.join(ROOT, "tests", "golden", "pin_report.txt")


def main():
    cases = [(a.split(":")[0], float(a.split(":")[1])) for a in sys.argv[1:]] or CASES
    have = {tuple(l.split()[:2]) for l in open(DIGESTS) if not l.startswith("#")}
    with open(REPORT, "a") as rep:
        for name, scale in cases:
            ax = generators.workload(name, scale)
            t0 = time.time()
            o = oracle.saturate(ax, 0)
            h = worklist.Closure(o.facts(), o.links()).digest()
            st = o.stats()
            o.close()
            t1 = time.time()
            w = worklist.saturate(ax).digest()
            t2 = time.time()
            line = (f"{name} {scale} concepts={ax.n_concepts} facts={st['s_facts']} links={st['links']} "
                    f"oracle={h} worklist={w} {'AGREE' if h == w else 'DIFFER'} "
                    f"oracle_s={t1 - t0:.1f} worklist_s={t2 - t1:.1f}")
            print(line, flush=True)
            rep.write(line + "\n")
            if h == w and (name, str(scale)) not in have:
                with open(DIGESTS, "a") as f:
                    f.write(f"{name} {scale} {ax.digest()} {h}\n")
            if h != w:
                sys.exit(1)


if __name__ == "__main__":
    main()
