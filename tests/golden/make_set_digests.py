"""Regenerate tests/golden/set_digests.txt: the order-independent closure digests
(distel_amd.result.set_digest) of pinned workloads, computed by the CPU oracle.  Each case is
cross-checked against its SHA-256 closure digest in closure_digests.txt (the oracle and the
independent worklist saturator agree on those, pin_report.txt) before its set digest is written.

    python tests/golden/make_set_digests.py [workload:scale ...]   (default: every pinned case)
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from distel_amd import generators  # noqa: E402
from distel_amd.result import set_digest  # noqa: E402

pinned = {}
for line in open(os.path.join(HERE, "closure_digests.txt")):
    f = line.split()
    if len(f) == 4 and not line.startswith("#"):
        pinned[(f[0], float(f[1]))] = (f[2], f[3])
want = [(a.split(":")[0], float(a.split(":")[1])) for a in sys.argv[1:]] or sorted(pinned)
out = os.path.join(HERE, "set_digests.txt")
rows = {}
if os.path.exists(out):
    for line in open(out):
        f = line.split()
        if len(f) == 4 and not line.startswith("#"):
            rows[(f[0], float(f[1]))] = line.rstrip("\n")
for name, scale in want:
    ax = generators.workload(name, scale)
    d_in, d_out = pinned[(name, scale)]
    assert ax.digest() == d_in, f"{name} {scale}: generator output changed"
    o = oracle.saturate(ax, 0)
    fx, fa = o.facts()
    lx, lr, ly = o.links()
    h = hashlib.sha256()
    for a in (fx, fa, lx, lr, ly):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == d_out, f"{name} {scale}: oracle closure differs from the pinned SHA-256"
    rows[(name, scale)] = f"{name} {scale} {d_in} {set_digest(fx, fa, lx, lr, ly)}"
    print(rows[(name, scale)], flush=True)
    del o, fx, fa, lx, lr, ly
with open(out, "w") as f:
    f.write("# workload scale input_sha256 set_digest  (tests/golden/make_set_digests.py; "
            "distel_amd.result.set_digest of the oracle closure)\n")
    for k in sorted(rows):
        f.write(rows[k] + "\n")
