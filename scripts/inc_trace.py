#!/usr/bin/env python3
"""The increment's part of a rocprofv3 kernel trace of `bench.py --increment F --steps 1
--warmup 0`: every kernel from the last k_retrigger on (the migrate tail, then the saturation
of the increment), per-kernel totals, and the wall-clock span with the GPU-idle gaps > 50 us.
Usage: scripts/inc_trace.py DB"""
import collections
import glob
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from rpd_stats import load  # noqa: E402


def main():
    db = glob.glob(sys.argv[1], recursive=True)[0]
    rows = [(n.replace("(anonymous namespace)::", "").split("(")[0], s, e) for n, s, e, _ in load(db)]
    last = max(i for i, r in enumerate(rows) if r[0] == "k_retrigger")
    # the increment's saturation ends at the last k_commit after it
    end = max(i for i, r in enumerate(rows) if r[0] == "k_commit" and i > last)
    part = rows[last:end + 1]
    t0, t1 = part[0][1], max(r[2] for r in part)
    agg = collections.OrderedDict()
    for n, s, e in part:
        g = agg.setdefault(n, [0, 0])
        g[0] += 1
        g[1] += e - s
    print(f"span k_retrigger -> last k_commit: {(t1 - t0) / 1e6:.3f} ms, kernels {len(part)}, "
          f"supersteps (k_commit launches) {agg.get('k_commit', [0])[0]}")
    busy = 0
    cur_s, cur_e = part[0][1], part[0][2]
    gaps = []
    for n, s, e in part[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            if s - cur_e > 50_000:
                gaps.append(((s - cur_e) / 1e3, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"GPU busy {busy / 1e6:.3f} ms; idle gaps > 50 us: {len(gaps)}, "
          f"{sum(g for g, _ in gaps) / 1e3:.3f} ms; largest: " +
          ", ".join(f"{g:.0f} us before {n}" for g, n in sorted(gaps, reverse=True)[:8]))
    print("kernel,calls,total_ms,avg_us")
    for k, (c, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k},{c},{ns / 1e6:.3f},{ns / c / 1e3:.2f}")


if __name__ == "__main__":
    main()
