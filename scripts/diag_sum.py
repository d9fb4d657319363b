#!/usr/bin/env python3
"""Summarise scripts/part_diag.py output: per leg and step the wall times, supersteps and the
kernels that took the most time (HIP events)."""
import json
import sys

for line in open(sys.argv[1]):
    d = json.loads(line)
    if d["leg"] == "load":
        print("load", d["s"])
        continue
    ranks = [d] if d["leg"] == "whole" else d["ranks"]
    head = f"{d['leg']} step {d['step']}" + (f" wall {d['wall_ms']} ms" if "wall_ms" in d else "")
    print(head, "derived", d.get("derived", ranks[0]["derived"]))
    for q, r in enumerate(ranks):
        top = sorted(r["kernels"].items(), key=lambda kv: -kv[1][1])[:6]
        print(f"  rank {q}: init {r['init_ms']} sat {r['saturate_ms']} tail {r['tail_ms']} steps {r['supersteps']} "
              f"xbytes {r['exchange_bytes']} | " + " ".join(f"{k}:{v[0]}x{v[1]}" for k, v in top))
