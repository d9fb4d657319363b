"""ctypes wrapper of the CPU oracle (oracle/el_oracle.c).  TEST INFRASTRUCTURE ONLY.

Importable by tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline``
leg — as the checker or the timed CPU baseline, never as the product path.
Parity: "parity unpinned" with respect to the reference's own outputs (the
Java/Redis reference cannot run here and ships no fixtures); pinned by the
hand-derived KATs in tests/golden/ and by naive-vs-semi-naive agreement.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libel_oracle.so")

NUM_KERNELS = 17
NUM_EVENTS = 8

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from distel_amd.engine import _ElAxioms  # the boundary struct layout only
    lib = C.CDLL(LIB)
    P = C.c_void_p
    u32p = C.POINTER(C.c_uint32)
    u64p = C.POINTER(C.c_uint64)
    lib.elo_create.argtypes = [C.POINTER(P), C.POINTER(_ElAxioms), C.c_int]
    lib.elo_init.argtypes = [P]
    lib.elo_step.argtypes = [P, C.c_int, C.POINTER(C.c_int)]
    lib.elo_saturate.argtypes = [P]
    for f in ("elo_num_facts", "elo_num_links", "elo_num_init", "elo_num_acts"):
        getattr(lib, f).argtypes = [P]
        getattr(lib, f).restype = C.c_uint64
    lib.elo_supersteps.argtypes = [P]
    lib.elo_supersteps.restype = C.c_uint32
    lib.elo_copy_facts.argtypes = [P, u32p, u32p, C.c_size_t]
    lib.elo_copy_log.argtypes = [P, u32p, u32p, C.c_size_t]
    lib.elo_copy_links.argtypes = [P, u32p, u32p, u32p, C.c_size_t]
    lib.elo_trace.argtypes = [P, u64p, u64p, u64p, C.c_size_t]
    lib.elo_events.argtypes = [P, u64p, C.c_size_t]
    lib.elo_error.argtypes = [P]
    lib.elo_error.restype = C.c_char_p
    lib.elo_destroy.argtypes = [P]
    lib.elo_destroy.restype = None
    _lib = lib
    return lib


class Oracle:
    """mode 0 = semi-naive Jacobi supersteps (GPU-identical deltas/events), 1 = naive fixpoint.

    Range axioms are read the way the engine reads them: ELK-style by default (the ontology is
    first put through distel_amd.ir.elk_ranges, the mirror of the engine's el::elk_ranges, and
    facts() / links() cover the given concepts' rows), DistEL's way (hazard H1, el_oracle.c's
    range rule) with compat_range=True.  stats(), trace() and events() are the whole closure's,
    like the engine's el_stats."""

    def __init__(self, ax, mode: int = 0, compat_range: bool = False):
        from distel_amd.engine import AxiomsView
        from distel_amd import ir
        self.lib = _load()
        self.ctx = C.c_void_p()
        self.n_user = ax.n_concepts
        if not compat_range:
            ax, _, _ = ir.elk_ranges(ax)
        self._view = AxiomsView(ax)
        rc = self.lib.elo_create(C.byref(self.ctx), C.byref(self._view.struct), mode)
        if rc != 0:
            msg = self.lib.elo_error(self.ctx).decode() if self.ctx else ""
            raise ValueError(f"oracle create failed ({rc}): {msg}")
        self.mode = mode

    def close(self):
        if self.ctx:
            self.lib.elo_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def init(self):
        self.lib.elo_init(self.ctx)

    def step(self, rule: int) -> bool:
        ch = C.c_int(0)
        rc = self.lib.elo_step(self.ctx, int(rule), C.byref(ch))
        if rc != 0:
            raise ValueError("elo_step failed")
        return bool(ch.value)

    def saturate(self):
        self.lib.elo_saturate(self.ctx)

    @property
    def supersteps(self) -> int:
        return int(self.lib.elo_supersteps(self.ctx))

    def stats(self) -> dict:
        f = int(self.lib.elo_num_facts(self.ctx))
        i = int(self.lib.elo_num_init(self.ctx))
        l = int(self.lib.elo_num_links(self.ctx))
        return dict(s_facts=f, s_init=i, links=l, derived=f - i + l, supersteps=self.supersteps,
                    activations=int(self.lib.elo_num_acts(self.ctx)))

    def facts(self) -> Tuple[np.ndarray, np.ndarray]:
        n = int(self.lib.elo_num_facts(self.ctx))
        x = np.zeros(n, np.uint32)
        a = np.zeros(n, np.uint32)
        p = lambda v: v.ctypes.data_as(C.POINTER(C.c_uint32))
        self.lib.elo_copy_facts(self.ctx, p(x), p(a), n)
        keep = x < self.n_user  # (ELK range fillers are internal rows)
        return x[keep], a[keep]

    def links(self):
        n = int(self.lib.elo_num_links(self.ctx))
        x, r, y = (np.zeros(n, np.uint32) for _ in range(3))
        p = lambda v: v.ctypes.data_as(C.POINTER(C.c_uint32))
        self.lib.elo_copy_links(self.ctx, p(x), p(r), p(y), n)
        order = np.lexsort((y, r, x))
        order = order[x[order] < self.n_user]
        return x[order], r[order], y[order]

    def trace(self):
        n = self.supersteps
        a, b, c = (np.zeros(max(n, 1), np.uint64) for _ in range(3))
        p = lambda v: v.ctypes.data_as(C.POINTER(C.c_uint64))
        self.lib.elo_trace(self.ctx, p(a), p(b), p(c), max(n, 1))
        return a[:n], b[:n], c[:n]

    def events(self) -> np.ndarray:
        ev = np.zeros(NUM_KERNELS * NUM_EVENTS, np.uint64)
        self.lib.elo_events(self.ctx, ev.ctypes.data_as(C.POINTER(C.c_uint64)), ev.size)
        return ev.reshape(NUM_KERNELS, NUM_EVENTS)


def saturate(ax, mode: int = 0, compat_range: bool = False) -> Oracle:
    o = Oracle(ax, mode, compat_range)
    o.init()
    o.saturate()
    return o
