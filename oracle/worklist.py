"""ctypes wrapper of the independent worklist saturator (oracle/worklist.c).
TEST INFRASTRUCTURE ONLY: it pins the semi-naive oracle (oracle/el_oracle.c) — it shares no code
with it — and is never the product path or the timed baseline."""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess
import sys
from typing import Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libel_worklist.so")
_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    sys.path.insert(0, os.path.dirname(HERE))
    from distel_amd.engine import _ElAxioms  # the boundary struct layout only
    lib = C.CDLL(LIB)
    P = C.c_void_p
    u32p = C.POINTER(C.c_uint32)
    lib.wl_saturate.argtypes = [C.POINTER(_ElAxioms), C.c_int, C.POINTER(P)]
    lib.wl_num_facts.argtypes = [P]
    lib.wl_num_facts.restype = C.c_uint64
    lib.wl_num_links.argtypes = [P]
    lib.wl_num_links.restype = C.c_uint64
    lib.wl_copy_facts.argtypes = [P, u32p, u32p]
    lib.wl_copy_links.argtypes = [P, u32p, u32p, u32p]
    lib.wl_free.argtypes = [P]
    lib.wl_free.restype = None
    _lib = lib
    return lib


class Closure:
    """facts (x, a) sorted by (x, a); links (x, r, y) sorted by (x, r, y)."""

    def __init__(self, facts, links):
        self._facts, self._links = facts, links

    def facts(self) -> Tuple[np.ndarray, np.ndarray]:
        return self._facts

    def links(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        return self._links

    def digest(self) -> str:
        """SHA-256 over the facts then the links (the layout of tests/golden/closure_digests.txt)."""
        h = hashlib.sha256()
        for a in self._facts + self._links:
            h.update(np.ascontiguousarray(a, dtype=np.uint32).tobytes())
        return h.hexdigest()


def saturate(ax, distel_range: bool = False) -> Closure:
    """The closure of ax by worklist completion.  Ranges are read ELK's way (folded into fresh
    existential fillers, as the engine's default), DistEL's way (K10, hazard H1) with
    distel_range=True."""
    from distel_amd.engine import AxiomsView
    lib = _load()
    view = AxiomsView(ax)
    h = C.c_void_p()
    rc = lib.wl_saturate(C.byref(view.struct), 1 if distel_range else 0, C.byref(h))
    try:
        if rc != 0:
            raise MemoryError("worklist saturator: out of memory")
        nf, nl = int(lib.wl_num_facts(h)), int(lib.wl_num_links(h))
        p = lambda v: v.ctypes.data_as(C.POINTER(C.c_uint32))
        x, a = np.zeros(nf, np.uint32), np.zeros(nf, np.uint32)
        lib.wl_copy_facts(h, p(x), p(a))
        lx, lr, ly = (np.zeros(nl, np.uint32) for _ in range(3))
        lib.wl_copy_links(h, p(lx), p(lr), p(ly))
    finally:
        lib.wl_free(h)
    return Closure((x, a), (lx, lr, ly))
