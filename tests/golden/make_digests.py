"""Regenerate tests/golden/closure_digests.txt: SHA-256 of generator inputs and of their
closures (facts sorted by (x, a) then links sorted by (x, r, y)) computed by the CPU oracle.

    python tests/golden/make_digests.py                      # the small cases (rewrites the file)
    python tests/golden/make_digests.py --append g3 0.5      # one more line (e.g. G3 @ 50 %, round 5)

(oracle/pin_digests.py appends the large cases the worklist saturator confirms.)"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from distel_amd import generators  # noqa: E402

CASES = [("g1", 0.1), ("g2", 0.05), ("g3", 0.01), ("g5", 0.02)]
append = len(sys.argv) == 4 and sys.argv[1] == "--append"
if append:
    CASES = [(sys.argv[2], float(sys.argv[3]))]

with open(os.path.join(HERE, "closure_digests.txt"), "a" if append else "w") as f:
    if not append:
        f.write("# workload scale input_sha256 closure_sha256  (tests/golden/make_digests.py)\n")
    for name, scale in CASES:
        ax = generators.workload(name, scale)
        o = oracle.saturate(ax, 0)
        h = hashlib.sha256()
        for a in o.facts() + o.links():
            h.update(np.ascontiguousarray(a).tobytes())
        f.write(f"{name} {scale} {ax.digest()} {h.hexdigest()}\n")
        print(name, scale, o.stats())
