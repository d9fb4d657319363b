"""ctypes binding of the C-ABI (include/el_gpu.h) — the only way Python reaches the GPU.

There is deliberately no CPU fallback: if ``libel_gpu.so`` is missing or no HIP
device is visible, every call raises ``ElError``.  (The CPU oracle under
``oracle/`` is test infrastructure and is never imported from here.)
"""
from __future__ import annotations

import ctypes as C
import enum
import os
from typing import Callable, Dict, Iterator, List, Optional, Tuple

import numpy as np

from .ir import Axioms

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libel_gpu.so")
if os.environ.get("EL_LIB_VARIANT"):  # A/B of a differently compiled build (scripts/build_variant.sh)
    LIB_PATH = os.path.join(_HERE, "lib", "variants", f"libel_gpu_{os.environ['EL_LIB_VARIANT']}.so")

EL_OK, EL_EINVAL, EL_ENOMEM, EL_EHIP, EL_ESTATE, EL_ERANGE = 0, -1, -2, -3, -4, -5
LAYOUT_X_TO_B, LAYOUT_B_TO_X = 0, 1
EL_FLAG_COMPAT_DISTEL_CHAIN = 0x1  # el_config.flags: hazard H2 reproduced (include/el_gpu.h)
EL_FLAG_COMPAT_DISTEL_RANGE = 0x2  # el_config.flags: DistEL's range reading (H1); default ELK's
EL_RESULT_RELEASE = 0x1  # el_result.flags: the state is released behind the copy-back
EL_RESULT_ASYNC = 0x2    # el_result.flags: return once enqueued; el_result_wait() = landed

# work phases (el_kernel); "kernel:role" where several phases share one launch
KERNEL_NAMES = ["k_expand:s", "k_expand:l", "k_jobs", "k_expand:a", "k_commit:s", "k_commit:l", "k_commit:a",
                "k_reloc_claim", "k_reloc_commit", "k_reloc_move", "k_reloc_move:ovf", "k_init", "k_rehash",
                "k_expand:p", "k_commit:p", "k_commit_told", "k_closure"]
EVENT_NAMES = ["trig", "row", "ent", "test", "hash", "emit", "job", "rmw"]
EVENT_BYTES = [8, 8, 4, 4, 8, 8, 16, 8]
NUM_KERNELS = len(KERNEL_NAMES)
ABI_VERSION = 8  # include/el_gpu.h EL_ABI_VERSION
XCHG_NONE, XCHG_LOCAL, XCHG_RCCL, XCHG_HOST = 0, 1, 2, 3
NUM_EVENTS = len(EVENT_NAMES)


class AxiomDistributionType(enum.IntEnum):
    """Rule types = ``kc/init/AxiomDistributionType.java:9-31`` (ordinal order)."""
    CR_TYPE1_1 = 0
    CR_TYPE1_2 = 1
    CR_TYPE2 = 2
    CR_TYPE3_1 = 3
    CR_TYPE3_2 = 4
    CR_TYPE4 = 5
    CR_TYPE5 = 6
    CR_TYPE_BOTTOM = 7


class ElError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"el error {code}: {msg}")
        self.code = code


_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)


class _ElAxioms(C.Structure):
    _fields_ = [
        ("n_concepts", C.c_uint32), ("n_roles", C.c_uint32), ("concept_kind", _u8p),
        ("n_sub", C.c_uint32), ("sub_a", _u32p), ("sub_b", _u32p),
        ("n_conj", C.c_uint32), ("conj_ptr", _u32p), ("conj_ops", _u32p), ("conj_b", _u32p),
        ("n_ex_rhs", C.c_uint32), ("exr_a", _u32p), ("exr_r", _u32p), ("exr_b", _u32p),
        ("n_ex_lhs", C.c_uint32), ("exl_r", _u32p), ("exl_a", _u32p), ("exl_b", _u32p),
        ("n_subrole", C.c_uint32), ("sr_r", _u32p), ("sr_s", _u32p),
        ("n_chain", C.c_uint32), ("ch_r", _u32p), ("ch_s", _u32p), ("ch_t", _u32p),
        ("n_domain", C.c_uint32), ("dom_r", _u32p), ("dom_c", _u32p),
        ("n_range", C.c_uint32), ("rng_r", _u32p), ("rng_c", _u32p),
    ]


class _ElConfig(C.Structure):
    _fields_ = [("device", C.c_int), ("profile", C.c_int), ("flags", C.c_uint32), ("exchange", C.c_int),
                ("part_rank", C.c_uint32), ("part_count", C.c_uint32), ("row_lo", C.c_uint32),
                ("row_hi", C.c_uint32), ("group", C.c_void_p), ("rccl_id", C.c_uint8 * 128),
                ("host_allgather", C.c_void_p), ("host_user", C.c_void_p)]


class _ElStats(C.Structure):
    _fields_ = [("supersteps", C.c_uint32), ("s_facts", C.c_uint64), ("s_init", C.c_uint64),
                ("links", C.c_uint64), ("derived", C.c_uint64), ("activations", C.c_uint64),
                ("propagations", C.c_uint64), ("bytes", C.c_uint64), ("ms", C.c_double),
                ("exchange_bytes", C.c_uint64)]


class _ElKernelStat(C.Structure):
    _fields_ = [("launches", C.c_uint64), ("events", C.c_uint64 * NUM_EVENTS), ("bytes", C.c_uint64),
                ("ms", C.c_double), ("group", C.c_uint32)]


class _ElResult(C.Structure):
    _fields_ = [("row_lo", C.c_uint32), ("row_hi", C.c_uint32), ("n_facts", C.c_uint64), ("n_links", C.c_uint64),
                ("n_pairs", C.c_uint32), ("flags", C.c_uint32), ("s_ptr", C.POINTER(C.c_uint64)), ("s_val", _u32p), ("s_cap", C.c_uint64),
                ("l_ptr", C.POINTER(C.c_uint64)), ("l_pair", _u32p), ("l_cap", C.c_uint64)]


class _ElStream(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("s_b", _u32p), ("s_cap", C.c_uint64), ("s_run", _u32p),
                ("s_run_cap", C.c_uint64), ("l_p", _u32p), ("l_cap", C.c_uint64), ("l_run", _u32p),
                ("l_run_cap", C.c_uint64), ("n_facts", C.c_uint64), ("n_links", C.c_uint64),
                ("n_s_runs", C.c_uint64), ("n_l_runs", C.c_uint64),
                ("s_code", C.POINTER(C.c_uint16)), ("s_esc", _u32p), ("s_esc_cap", C.c_uint64),
                ("n_s_esc", C.c_uint64)]


EL_STREAM_PACKED = 0x4

_SINK = C.CFUNCTYPE(C.c_int, C.c_void_p, _u32p, _u32p, C.c_size_t)
_ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)

EXPORTED_SYMBOLS = [
    "el_abi_version", "el_device_count", "el_create", "el_load", "el_init", "el_step", "el_saturate",
    "el_get_stats", "el_kernel_stats", "el_set_profile", "el_superstep_trace", "el_get_subsumers", "el_copy_facts",
    "el_copy_links", "el_export_result", "el_last_error", "el_destroy", "el_group_create", "el_group_destroy",
    "el_rccl_unique_id", "el_add_axioms", "el_result_info", "el_copy_result", "el_result_wait", "el_pair_table", "el_host_alloc",
    "el_host_free", "el_fresh_fillers", "el_stream_result", "el_stream_codes", "el_pid_table", "el_increment_info",
]

_lib: Optional[C.CDLL] = None


def load_library(path: Optional[str] = None) -> C.CDLL:
    """Load libel_gpu.so (built by ``__graft_entry__.build()``); raise if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("EL_GPU_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise ElError(EL_EHIP, f"HIP extension not built: {p} missing (run __graft_entry__.build())")
    lib = C.CDLL(p)
    P = C.c_void_p
    lib.el_abi_version.restype = C.c_int
    if lib.el_abi_version() != ABI_VERSION:
        raise ElError(EL_EHIP, f"{p}: ABI version {lib.el_abi_version()} != {ABI_VERSION} (rebuild)")
    lib.el_device_count.argtypes = [C.POINTER(C.c_int)]
    lib.el_create.argtypes = [C.POINTER(P), C.POINTER(_ElConfig)]
    lib.el_load.argtypes = [P, C.POINTER(_ElAxioms)]
    lib.el_init.argtypes = [P]
    lib.el_add_axioms.argtypes = [P, C.POINTER(_ElAxioms)]
    lib.el_increment_info.argtypes = [P, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    lib.el_step.argtypes = [P, C.c_int, C.POINTER(C.c_int)]
    lib.el_saturate.argtypes = [P, C.POINTER(_ElStats)]
    lib.el_get_stats.argtypes = [P, C.POINTER(_ElStats)]
    lib.el_kernel_stats.argtypes = [P, C.POINTER(_ElKernelStat), C.c_int]
    if hasattr(lib, "el_set_profile"):  # (ABI 7 builds before round 6 lack it: A/B variants)
        lib.el_set_profile.argtypes = [P, C.c_int]
    lib.el_superstep_trace.argtypes = [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                       C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_get_subsumers.argtypes = [P, C.c_uint32, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_copy_facts.argtypes = [P, _u32p, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_copy_links.argtypes = [P, _u32p, _u32p, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_export_result.argtypes = [P, C.c_int, _SINK, C.c_void_p]
    lib.el_result_info.argtypes = [P, C.POINTER(_ElResult)]
    lib.el_result_wait.argtypes = [P]
    lib.el_copy_result.argtypes = [P, C.POINTER(_ElResult)]
    lib.el_pair_table.argtypes = [P, _u32p, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_pid_table.argtypes = [P, _u32p, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_stream_result.argtypes = [P, C.POINTER(_ElStream)]
    if hasattr(lib, "el_stream_codes"):  # (an A/B variant built from an older source may lack it)
        lib.el_stream_codes.argtypes = [P, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_host_alloc.argtypes = [C.c_size_t]
    lib.el_host_alloc.restype = C.c_void_p
    lib.el_host_free.argtypes = [C.c_void_p]
    lib.el_host_free.restype = None
    lib.el_fresh_fillers.argtypes = [P, _u32p, _u32p, C.c_size_t, C.POINTER(C.c_size_t)]
    lib.el_last_error.argtypes = [P]
    lib.el_last_error.restype = C.c_char_p
    lib.el_destroy.argtypes = [P]
    lib.el_destroy.restype = None
    lib.el_group_create.argtypes = [C.POINTER(P), C.c_int]
    lib.el_group_destroy.argtypes = [P]
    lib.el_group_destroy.restype = None
    lib.el_rccl_unique_id.argtypes = [C.POINTER(C.c_uint8 * 128)]
    if path is None:
        _lib = lib
    return lib


def device_count() -> int:
    lib = load_library()
    n = C.c_int(0)
    lib.el_device_count(C.byref(n))
    return int(n.value)


def _ptr(a: np.ndarray, t=_u32p):
    return a.ctypes.data_as(t) if a.size else None


class AxiomsView:
    """Keeps the numpy columns alive while the C struct points at them."""

    def __init__(self, ax: Axioms):
        ax.validate()
        col = lambda a, j: np.ascontiguousarray(a[:, j], dtype=np.uint32)
        self._keep = []

        def k(a):
            a = np.ascontiguousarray(a, dtype=np.uint32)
            self._keep.append(a)
            return _ptr(a)
        kind = np.ascontiguousarray(ax.kind, dtype=np.uint8)
        self._keep.append(kind)
        s = _ElAxioms()
        s.n_concepts, s.n_roles, s.concept_kind = ax.n_concepts, ax.n_roles, _ptr(kind, _u8p)
        s.n_sub, s.sub_a, s.sub_b = len(ax.sub), k(col(ax.sub, 0)), k(col(ax.sub, 1))
        s.n_conj, s.conj_ptr, s.conj_ops, s.conj_b = ax.n_conj, k(ax.conj_ptr), k(ax.conj_ops), k(ax.conj_b)
        s.n_ex_rhs, s.exr_a, s.exr_r, s.exr_b = (len(ax.ex_rhs), k(col(ax.ex_rhs, 0)), k(col(ax.ex_rhs, 1)),
                                                 k(col(ax.ex_rhs, 2)))
        s.n_ex_lhs, s.exl_r, s.exl_a, s.exl_b = (len(ax.ex_lhs), k(col(ax.ex_lhs, 0)), k(col(ax.ex_lhs, 1)),
                                                 k(col(ax.ex_lhs, 2)))
        s.n_subrole, s.sr_r, s.sr_s = len(ax.subrole), k(col(ax.subrole, 0)), k(col(ax.subrole, 1))
        s.n_chain, s.ch_r, s.ch_s, s.ch_t = (len(ax.chain), k(col(ax.chain, 0)), k(col(ax.chain, 1)),
                                             k(col(ax.chain, 2)))
        s.n_domain, s.dom_r, s.dom_c = len(ax.domain), k(col(ax.domain, 0)), k(col(ax.domain, 1))
        s.n_range, s.rng_r, s.rng_c = len(ax.range), k(col(ax.range, 0)), k(col(ax.range, 1))
        self.struct = s


def pinned_array(n: int, dtype) -> np.ndarray:
    """numpy array over page-locked host memory (el_host_alloc), freed with the array."""
    import weakref
    lib = load_library()
    dt = np.dtype(dtype)
    nbytes = max(1, int(n)) * dt.itemsize
    p = lib.el_host_alloc(nbytes)
    if not p:
        raise ElError(EL_ENOMEM, f"el_host_alloc({nbytes}) failed")
    raw = (C.c_uint8 * nbytes).from_address(p)
    arr = np.frombuffer(raw, dtype=np.uint8, count=nbytes).view(dt)[:int(n)]
    weakref.finalize(raw, lib.el_host_free, p)
    return arr


class Result:
    """Result copy-back (el_copy_result): CSR rows over [row_lo, row_hi).
    S(x) = s_val[s_ptr[x - row_lo]:s_ptr[x - row_lo + 1]] (ascending);
    links of x = pair ids l_pair[l_ptr[..]:l_ptr[..]] (ascending), pair q = (pair_role[q], pair_y[q])."""

    def __init__(self):
        self.row_lo = self.row_hi = 0
        self.n_facts = self.n_links = self.n_pairs = 0
        self.s_ptr = self.s_val = self.l_ptr = self.l_pair = None

    def _fit(self, rows: int, n_facts: int, n_links: int, pinned: bool) -> None:
        alloc = pinned_array if pinned else (lambda n, dt: np.empty(n, dt))
        if self.s_ptr is None or self.s_ptr.size != rows + 1:
            self.s_ptr = alloc(rows + 1, np.uint64)
            self.l_ptr = alloc(rows + 1, np.uint64)
        if self.s_val is None or self.s_val.size < n_facts:
            self.s_val = alloc(n_facts + n_facts // 8, np.uint32)
        if self.l_pair is None or self.l_pair.size < n_links:
            self.l_pair = alloc(n_links + n_links // 8, np.uint32)

    def facts(self) -> Tuple[np.ndarray, np.ndarray]:
        """(x, a) pairs sorted by (x, a)."""
        rows = np.arange(self.row_lo, self.row_hi, dtype=np.uint32)
        cnt = np.diff(self.s_ptr.astype(np.int64))
        return np.repeat(rows, cnt), self.s_val[:self.n_facts].copy()

    def subsumers(self, x: int) -> np.ndarray:
        i = x - self.row_lo
        return self.s_val[int(self.s_ptr[i]):int(self.s_ptr[i + 1])]


class Stream:
    """Streamed result (el_stream_result): the result node's writes in commit order, as they are
    committed, row-run encoded — S facts s_b[i] with the runs (x, end) of s_run, links l_p[i]
    (pair ids, Engine.pid_table()) with the runs of l_run.  Page-locked buffers, reused across
    classifications; complete after Engine.result_wait().

    packed (EL_STREAM_PACKED): the facts' values cross as 16-bit codes s_code[i] (the value's bit
    column, Engine.stream_codes() maps it back) with the values of code 0xFFFF in s_esc, in order —
    2 B per fact instead of 4 (G3: 96.6 % of the facts coded); fact_rows() decodes."""

    def __init__(self, packed: bool = False):
        self.packed = packed
        self.n_facts = self.n_links = self.n_s_runs = self.n_l_runs = self.n_s_esc = 0
        self.s_b = self.l_p = self.s_run = self.l_run = self.s_code = self.s_esc = None
        self.code_table: Optional[np.ndarray] = None  # (set by Engine.stream_result)
        self._st = _ElStream()

    def fit(self, n_facts: int, n_links: int, n_s_runs: int = 0, n_l_runs: int = 0, n_s_esc: int = 0) -> None:
        """Buffers for at least these counts (runs: a quarter of the entries unless known;
        escapes: an eighth of the facts unless known)."""
        grow = lambda n: n + n // 8 + 1024
        if self.packed:
            if self.s_code is None or self.s_code.size < n_facts:
                self.s_code = pinned_array(grow(n_facts), np.uint16)
            ne = n_s_esc or n_facts // 8
            if self.s_esc is None or self.s_esc.size < ne:
                self.s_esc = pinned_array(grow(ne), np.uint32)
        elif self.s_b is None or self.s_b.size < n_facts:
            self.s_b = pinned_array(grow(n_facts), np.uint32)
        if self.l_p is None or self.l_p.size < n_links:
            self.l_p = pinned_array(grow(n_links), np.uint32)
        rs, rl = n_s_runs or n_facts // 4, n_l_runs or n_links // 4
        if self.s_run is None or self.s_run.shape[0] < rs:
            self.s_run = pinned_array(2 * grow(rs), np.uint32).reshape(-1, 2)
        if self.l_run is None or self.l_run.shape[0] < rl:
            self.l_run = pinned_array(2 * grow(rl), np.uint32).reshape(-1, 2)

    @staticmethod
    def _rows(runs: np.ndarray, n_runs: int, n: int) -> np.ndarray:
        """Per-entry x from the runs (x, end)."""
        if n_runs == 0:
            if n:
                raise ValueError(f"malformed runs: {n} entries but no run")
            return np.zeros(0, np.uint32)
        r = runs[:n_runs]
        ends = r[:, 1].astype(np.int64)
        lens = np.diff(np.concatenate(([0], ends)))
        if ends[-1] != n or not (lens > 0).all():
            raise ValueError("malformed runs: the run ends do not cover the entries in ascending order")
        return np.repeat(r[:, 0], lens)

    def values(self) -> np.ndarray:
        """The facts' values b in commit order (packed: decoded from the codes and escapes)."""
        if not self.packed:
            return self.s_b[:self.n_facts].copy()
        codes = self.s_code[:self.n_facts]
        esc = codes == 0xFFFF
        if int(esc.sum()) != self.n_s_esc:
            raise ValueError(f"malformed packed stream: {int(esc.sum())} escape codes, {self.n_s_esc} escapes")
        b = self.code_table[np.minimum(codes, len(self.code_table) - 1)].astype(np.uint32)
        b[esc] = self.s_esc[:self.n_s_esc]
        if (b == 0xFFFFFFFF).any():
            raise ValueError("malformed packed stream: a code no concept holds")
        return b

    def bytes(self) -> int:
        """Bytes that crossed PCIe: values (or codes + escapes), links, runs."""
        vb = 2 * self.n_facts + 4 * self.n_s_esc if self.packed else 4 * self.n_facts
        return vb + 4 * self.n_links + 8 * (self.n_s_runs + self.n_l_runs)

    def fact_rows(self) -> Tuple[np.ndarray, np.ndarray]:
        """(x, b) per fact, in commit order."""
        return self._rows(self.s_run, self.n_s_runs, self.n_facts), self.values()

    def link_rows(self) -> Tuple[np.ndarray, np.ndarray]:
        """(x, pid) per link, in commit order."""
        return self._rows(self.l_run, self.n_l_runs, self.n_links), self.l_p[:self.n_links].copy()

    def facts(self, n_user: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        """(x, a) pairs sorted by (x, a); rows >= n_user (ELK range fillers) dropped when given."""
        x, a = self.fact_rows()
        if n_user is not None:
            keep = x < n_user
            x, a = x[keep], a[keep]
        o = np.lexsort((a, x))
        return x[o], a[o]

    def digest(self, pid_role: np.ndarray, pid_filler: np.ndarray, n_user: int) -> str:
        """Order-independent digest (distel_amd.result.set_digest) of the streamed closure over
        the caller's rows (< n_user): decoded from the runs and hashed per entry, no sort."""
        from .result import set_digest
        x, b = self.fact_rows()
        lx, lp = self.link_rows()
        if n_user is not None:
            k = x < n_user
            x, b = x[k], b[k]
            k = lx < n_user
            lx, lp = lx[k], lp[k]
        return set_digest(x, b, lx, pid_role[lp], pid_filler[lp])


class Stats(dict):
    @staticmethod
    def from_c(s: _ElStats) -> "Stats":
        return Stats(supersteps=s.supersteps, s_facts=s.s_facts, s_init=s.s_init, links=s.links, derived=s.derived,
                     activations=s.activations, propagations=s.propagations, bytes=s.bytes, ms=s.ms,
                     exchange_bytes=s.exchange_bytes)


class Partition:
    """Row partition of one engine: this rank owns S(X) for X in
    [row_lo, row_hi) (0, 0 = the equal split) and all-gathers its deltas each superstep.
    allgather (EL_XCHG_HOST): fn(send: bytes-like, recv: writable, size × len(send)) that
    all-gathers this rank's block over the caller's transport (e.g. ``gloo_allgather()``)."""

    def __init__(self, rank: int, count: int, exchange: int, group: "Optional[LocalGroup]" = None,
                 rccl_id: Optional[bytes] = None, rows: Tuple[int, int] = (0, 0),
                 allgather: Optional[Callable[[memoryview, memoryview], None]] = None):
        self.rank, self.count, self.exchange, self.group, self.rccl_id, self.rows = (
            rank, count, exchange, group, rccl_id, rows)
        self.allgather = allgather
        self.error: Optional[BaseException] = None  # the transport's last exception
        self._cfn = None
        if allgather is not None:
            def trampoline(_user, send, recv, nbytes):
                try:
                    allgather(memoryview((C.c_uint8 * nbytes).from_address(send)).cast("B"),
                              memoryview((C.c_uint8 * (nbytes * count)).from_address(recv)).cast("B"))
                    return 0
                except Exception as exc:  # noqa: BLE001 - reported through the C return code
                    self.error = exc
                    return 1
            self._cfn = _ALLGATHER(trampoline)  # kept alive as long as the partition


def gloo_allgather(group=None) -> Callable[[memoryview, memoryview], None]:
    """EL_XCHG_HOST transport over torch.distributed (any backend with CPU all_gather, e.g.
    gloo): the per-superstep delta all-gather of SURVEY.md §8(e) staged through host memory."""
    import torch
    import torch.distributed as dist

    def fn(send: memoryview, recv: memoryview) -> None:
        n = len(send)
        world = dist.get_world_size(group)
        src = torch.from_numpy(np.frombuffer(send, dtype=np.uint8).copy())
        out = [torch.empty(n, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(out, src, group=group)
        dst = np.frombuffer(recv, dtype=np.uint8)
        for q, t in enumerate(out):
            dst[q * n:(q + 1) * n] = t.numpy()
    return fn


class LocalGroup:
    """In-process exchange group (EL_XCHG_LOCAL): n engines driven by n threads."""

    def __init__(self, n: int):
        self._lib = load_library()
        self.ptr = C.c_void_p()
        rc = self._lib.el_group_create(C.byref(self.ptr), int(n))
        if rc != EL_OK:
            raise ElError(rc, "el_group_create failed")
        self.n = n

    def close(self) -> None:
        if self.ptr:
            self._lib.el_group_destroy(self.ptr)
            self.ptr = C.c_void_p()


def rccl_unique_id() -> bytes:
    """ncclUniqueId for EL_XCHG_RCCL (rank 0 makes it; the launcher broadcasts it)."""
    lib = load_library()
    buf = (C.c_uint8 * 128)()
    rc = lib.el_rccl_unique_id(C.byref(buf))
    if rc != EL_OK:
        raise ElError(rc, "el_rccl_unique_id failed (RCCL unavailable)")
    return bytes(buf)


class Engine:
    """One GPU saturation context (one DistEL rule cluster), on one device."""

    def __init__(self, device: int = 0, profile: bool = False, partition: Optional[Partition] = None,
                 compat_chain: bool = False, compat_range: bool = False):
        """compat_chain: EL_FLAG_COMPAT_DISTEL_CHAIN, DistEL's CR6 join that ignores s (hazard H2,
        Type5AxiomProcessorBase.java:115-154); default the complete EL+ closure.
        compat_range: EL_FLAG_COMPAT_DISTEL_RANGE, DistEL's range rule (hazard H1,
        RolePairHandler.java:471-479); default ELK's reading of ranges."""
        self._lib = load_library()
        self._ctx = C.c_void_p()
        flags = (EL_FLAG_COMPAT_DISTEL_CHAIN if compat_chain else 0) | (EL_FLAG_COMPAT_DISTEL_RANGE if compat_range else 0)
        cfg = _ElConfig(device, 1 if profile else 0, flags)
        if partition is not None:
            cfg.exchange = partition.exchange
            cfg.part_rank, cfg.part_count = partition.rank, partition.count
            cfg.row_lo, cfg.row_hi = partition.rows
            if partition.group is not None:
                cfg.group = partition.group.ptr
            if partition.rccl_id is not None:
                C.memmove(cfg.rccl_id, partition.rccl_id, 128)
            if partition._cfn is not None:
                cfg.host_allgather = C.cast(partition._cfn, C.c_void_p)
        rc = self._lib.el_create(C.byref(self._ctx), C.byref(cfg))
        if rc != EL_OK:
            raise ElError(rc, f"el_create(device={device}) failed: no usable HIP device or bad partition")
        self.partition = partition
        self.ax = None  # the loaded ontology (old ∪ increments; see the property)
        self._last: Optional[Stats] = None   # the last saturation's stats
        self._streamed = None  # (Stream, release) of the last streamed result until result_wait
        self._codes_for = None  # (the axioms a packed stream's code table was read for)
        self._stream: Optional[Stream] = None  # a streamed result armed for the next saturate()

    @property
    def ax(self) -> Optional[Axioms]:
        """The loaded axioms, increments included.  add_axioms() leaves the merge to the first
        reader: it is host bookkeeping (G3: ≈140 ms of array concatenation) that sat between the
        increment and the next saturate(), the GPU idle meanwhile."""
        if self._inc:
            for inc in self._inc:
                self._ax = merge_axioms(self._ax, inc) if self._ax is not None else inc
            self._inc = []
        return self._ax

    @ax.setter
    def ax(self, v: Optional[Axioms]) -> None:
        self._ax = v
        self._inc: List[Axioms] = []

    def _check(self, rc: int, what: str) -> None:
        cause = None
        if self.partition is not None:  # the transport's exception of THIS call, if any
            cause, self.partition.error = self.partition.error, None
        if rc != EL_OK:
            msg = self._lib.el_last_error(self._ctx)
            raise ElError(rc, f"{what}: {msg.decode() if msg else ''}") from cause

    def close(self) -> None:
        if self._ctx:
            self._lib.el_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ lifecycle
    def load(self, ax: Axioms) -> None:
        view = AxiomsView(ax)
        self._check(self._lib.el_load(self._ctx, C.byref(view.struct)), "el_load")
        self.ax = ax
        self._last = None  # (its counts size streamed results of this ontology only)

    def init(self) -> None:
        self._check(self._lib.el_init(self._ctx), "el_init")

    def add_axioms(self, inc: Axioms) -> None:
        """Incremental classification: the loaded ontology becomes old ∪ inc (same id spaces,
        possibly extended); a saturated state is kept and the next saturate() continues."""
        view = AxiomsView(inc)
        self._check(self._lib.el_add_axioms(self._ctx, C.byref(view.struct)), "el_add_axioms")
        self._inc.append(inc)
        self._last = None

    def increment_info(self) -> Dict:
        """The last add_axioms: host index build / upload / state migration ms, and the logged
        facts and links the next saturate() re-triggers first (el_increment_info)."""
        ms = (C.c_double * 3)()
        rt = (C.c_uint64 * 2)()
        self._check(self._lib.el_increment_info(self._ctx, ms, rt), "el_increment_info")
        return {"index_ms": ms[0], "upload_ms": ms[1], "migrate_ms": ms[2], "retrigger_facts": int(rt[0]),
                "retrigger_links": int(rt[1])}

    def step(self, rule: int) -> bool:
        ch = C.c_int(0)
        self._check(self._lib.el_step(self._ctx, int(rule), C.byref(ch)), "el_step")
        return bool(ch.value)

    def saturate(self) -> Stats:
        s = _ElStats()
        self._check(self._lib.el_saturate(self._ctx, C.byref(s)), "el_saturate")
        self._last = Stats.from_c(s)
        if self._stream is not None:  # (a streamed result: its counts are known now)
            st = self._stream._st
            self._stream.n_facts, self._stream.n_links = int(st.n_facts), int(st.n_links)
            self._stream.n_s_runs, self._stream.n_l_runs = int(st.n_s_runs), int(st.n_l_runs)
            self._stream.n_s_esc = int(st.n_s_esc)
            self._stream = None
        return self._last

    def stats(self) -> Stats:
        s = _ElStats()
        self._check(self._lib.el_get_stats(self._ctx, C.byref(s)), "el_get_stats")
        return Stats.from_c(s)

    def set_profile(self, on: bool) -> None:
        """Per-kernel HIP-event timing from the next launch on (el_set_profile)."""
        self._check(self._lib.el_set_profile(self._ctx, 1 if on else 0), "el_set_profile")

    def kernel_stats(self) -> List[Dict]:
        arr = (_ElKernelStat * NUM_KERNELS)()
        self._check(self._lib.el_kernel_stats(self._ctx, arr, NUM_KERNELS), "el_kernel_stats")
        out = []
        for k in range(NUM_KERNELS):
            s = arr[k]
            out.append(dict(kernel=KERNEL_NAMES[k], launches=int(s.launches), bytes=int(s.bytes), ms=float(s.ms),
                            group=KERNEL_NAMES[int(s.group)],
                            events={EVENT_NAMES[e]: int(s.events[e]) for e in range(NUM_EVENTS)}))
        return out

    def events(self) -> np.ndarray:
        """(kernels, events) uint64 matrix of algorithmic event counts."""
        ks = self.kernel_stats()
        return np.array([[k["events"][e] for e in EVENT_NAMES] for k in ks], dtype=np.uint64)

    def trace(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        n = C.c_size_t(0)
        rc = self._lib.el_superstep_trace(self._ctx, None, None, None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_superstep_trace")
        m = n.value
        a, b, c = (np.zeros(m, dtype=np.uint64) for _ in range(3))
        p = lambda x: x.ctypes.data_as(C.POINTER(C.c_uint64))
        self._check(self._lib.el_superstep_trace(self._ctx, p(a), p(b), p(c), m, C.byref(n)), "el_superstep_trace")
        return a, b, c

    # ------------------------------------------------------------ results
    def subsumers(self, x: int) -> np.ndarray:
        n = C.c_size_t(0)
        rc = self._lib.el_get_subsumers(self._ctx, int(x), None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_get_subsumers")
        out = np.zeros(n.value, dtype=np.uint32)
        self._check(self._lib.el_get_subsumers(self._ctx, int(x), _ptr(out), out.size, C.byref(n)),
                    "el_get_subsumers")
        return out

    def facts(self) -> Tuple[np.ndarray, np.ndarray]:
        """All (x, a) with a ∈ S(x), sorted by (x, a)."""
        n = C.c_size_t(0)
        rc = self._lib.el_copy_facts(self._ctx, None, None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_copy_facts")
        x = np.zeros(n.value, dtype=np.uint32)
        a = np.zeros(n.value, dtype=np.uint32)
        self._check(self._lib.el_copy_facts(self._ctx, _ptr(x), _ptr(a), x.size, C.byref(n)), "el_copy_facts")
        return x, a

    def links(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """All (x, r, y) with (x, y) ∈ R(r), sorted by (x, r, y)."""
        n = C.c_size_t(0)
        rc = self._lib.el_copy_links(self._ctx, None, None, None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_copy_links")
        x, r, y = (np.zeros(n.value, dtype=np.uint32) for _ in range(3))
        self._check(self._lib.el_copy_links(self._ctx, _ptr(x), _ptr(r), _ptr(y), x.size, C.byref(n)),
                    "el_copy_links")
        return x, r, y

    def result_info(self) -> _ElResult:
        r = _ElResult()
        self._check(self._lib.el_result_info(self._ctx, C.byref(r)), "el_result_info")
        return r

    def copy_result(self, out: Optional[Result] = None, pinned: bool = True, facts: bool = True,
                    links: bool = True, release: bool = False, wait: bool = True) -> Result:
        """Result copy-back into ``out`` (reused across calls; page-locked buffers by default).
        release: EL_RESULT_RELEASE — the next init()'s reset runs behind the copy-back; the engine
        has no state until init().  wait=False (with release): EL_RESULT_ASYNC — returns once the
        copy is enqueued; ``out`` is complete after result_wait() (or any later call on this engine)."""
        if not wait and not release:
            raise ValueError("an asynchronous copy-back releases the state (release=True)")
        info = self.result_info()
        out = out or Result()
        out._fit(info.row_hi - info.row_lo, info.n_facts if facts else 0, info.n_links if links else 0, pinned)
        r = _ElResult()
        r.flags = (EL_RESULT_RELEASE if release else 0) | (0 if wait else EL_RESULT_ASYNC)
        if facts:
            r.s_ptr = out.s_ptr.ctypes.data_as(C.POINTER(C.c_uint64))
            r.s_val = out.s_val.ctypes.data_as(_u32p)
            r.s_cap = out.s_val.size
        if links:
            r.l_ptr = out.l_ptr.ctypes.data_as(C.POINTER(C.c_uint64))
            r.l_pair = out.l_pair.ctypes.data_as(_u32p)
            r.l_cap = out.l_pair.size
        self._check(self._lib.el_copy_result(self._ctx, C.byref(r)), "el_copy_result")
        out.row_lo, out.row_hi, out.n_facts, out.n_links, out.n_pairs = (r.row_lo, r.row_hi, r.n_facts, r.n_links,
                                                                         r.n_pairs)
        return out

    def stream_result(self, out: Stream, release: bool = False, n_facts: int = 0, n_links: int = 0) -> Stream:
        """Arm the next saturate() to stream its result into ``out`` while it runs; complete after
        result_wait().  Buffers fit max(n_facts / n_links, the last saturation's counts), or
        64 entries per concept when neither is known for the loaded ontology (result_wait raises
        EL_ERANGE if short)."""
        last = self._last
        nf = max(n_facts, last["s_facts"] if last else 0) or 64 * max(self.ax.n_concepts if self.ax else 1, 1)
        nl = max(n_links, last["links"] if last else 0) or 64 * max(self.ax.n_concepts if self.ax else 1, 1)
        out.fit(nf, nl, out.n_s_runs, out.n_l_runs, out.n_s_esc)
        s = out._st
        s.flags = (EL_RESULT_RELEASE if release else 0) | (EL_STREAM_PACKED if out.packed else 0)
        if out.packed:
            if out.code_table is None or self._codes_for is not self.ax:
                out.code_table = self.stream_codes()
                self._codes_for = self.ax
            s.s_b = None
            s.s_code = out.s_code.ctypes.data_as(C.POINTER(C.c_uint16))
            s.s_cap = out.s_code.size
            s.s_esc = out.s_esc.ctypes.data_as(_u32p)
            s.s_esc_cap = out.s_esc.size
        else:
            s.s_b = out.s_b.ctypes.data_as(_u32p)
            s.s_cap = out.s_b.size
            s.s_code = None
            s.s_esc = None
            s.s_esc_cap = 0
        s.s_run = out.s_run.ctypes.data_as(_u32p)
        s.s_run_cap = out.s_run.shape[0]
        s.l_p = out.l_p.ctypes.data_as(_u32p)
        s.l_cap = out.l_p.size
        s.l_run = out.l_run.ctypes.data_as(_u32p)
        s.l_run_cap = out.l_run.shape[0]
        self._check(self._lib.el_stream_result(self._ctx, C.byref(s)), "el_stream_result")
        self._stream = out
        self._streamed = (out, release)
        return out

    def stream_codes(self) -> np.ndarray:
        """code -> concept of a packed stream (el_stream_codes; 0xFFFFFFFF: no concept)."""
        n = C.c_size_t(0)
        rc = self._lib.el_stream_codes(self._ctx, None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_stream_codes")
        t = np.zeros(n.value, np.uint32)
        self._check(self._lib.el_stream_codes(self._ctx, _ptr(t), n.value, C.byref(n)), "el_stream_codes")
        return t

    def pid_table(self) -> Tuple[np.ndarray, np.ndarray]:
        """pair id -> (role, filler), in pid order (the ids streamed links carry)."""
        n = C.c_size_t(0)
        rc = self._lib.el_pid_table(self._ctx, None, None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_pid_table")
        role = np.zeros(n.value, np.uint32)
        filler = np.zeros(n.value, np.uint32)
        self._check(self._lib.el_pid_table(self._ctx, _ptr(role), _ptr(filler), n.value, C.byref(n)), "el_pid_table")
        return role, filler

    def result_wait(self) -> None:
        """Block until an asynchronous copy-back (copy_result(wait=False)) or a streamed result
        has landed.  A streamed result whose buffers were short (EL_ERANGE: the state was kept)
        is streamed again at the fixpoint into buffers fitted to its counts."""
        rc = self._lib.el_result_wait(self._ctx)
        streamed, self._streamed = self._streamed, None
        if rc == EL_ERANGE and streamed is not None:
            out, release = streamed
            last = self._last
            self.stream_result(out, release, out.n_facts, out.n_links)
            self.saturate()  # (no superstep: the whole logs stream)
            self._last = last
            self._streamed = None
            rc = self._lib.el_result_wait(self._ctx)
        self._check(rc, "el_result_wait")

    def fresh_fillers(self) -> Tuple[np.ndarray, np.ndarray]:
        """ELK range fillers: concept n_concepts + i = filler[i] ⊓ ranges*(role[i])."""
        n = C.c_size_t(0)
        rc = self._lib.el_fresh_fillers(self._ctx, None, None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_fresh_fillers")
        b = np.zeros(n.value, np.uint32)
        r = np.zeros(n.value, np.uint32)
        self._check(self._lib.el_fresh_fillers(self._ctx, _ptr(b), _ptr(r), n.value, C.byref(n)), "el_fresh_fillers")
        return b, r

    def pair_table(self) -> Tuple[np.ndarray, np.ndarray]:
        """pair q -> (role, filler), ascending in (role, filler)."""
        n = C.c_size_t(0)
        rc = self._lib.el_pair_table(self._ctx, None, None, 0, C.byref(n))
        if rc not in (EL_OK, EL_ERANGE):
            self._check(rc, "el_pair_table")
        role = np.zeros(n.value, np.uint32)
        filler = np.zeros(n.value, np.uint32)
        self._check(self._lib.el_pair_table(self._ctx, _ptr(role), _ptr(filler), n.value, C.byref(n)),
                    "el_pair_table")
        return role, filler

    def export_result(self, layout: int = LAYOUT_X_TO_B) -> Tuple[np.ndarray, np.ndarray]:
        """Stream the result node through the C sink; returns (keys, values)."""
        ks: List[np.ndarray] = []
        vs: List[np.ndarray] = []

        def sink(_user, k, v, n):
            ks.append(np.ctypeslib.as_array(k, shape=(n,)).copy())
            vs.append(np.ctypeslib.as_array(v, shape=(n,)).copy())
            return 0
        cb = _SINK(sink)
        self._check(self._lib.el_export_result(self._ctx, int(layout), cb, None), "el_export_result")
        if not ks:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint32)
        return np.concatenate(ks), np.concatenate(vs)


def merge_axioms(a: Axioms, b: Axioms) -> Axioms:
    """old ∪ increment as one Axioms (b's id spaces extend a's)."""
    n = max(a.n_concepts, b.n_concepts)
    kind = np.zeros(n, np.uint8)
    kind[:b.n_concepts] = b.kind
    kind[:a.n_concepts] = a.kind
    cat = lambda x, y: np.concatenate([x, y]).astype(np.uint32)
    conj = [(a.conj_ops[a.conj_ptr[i]:a.conj_ptr[i + 1]].tolist(), int(a.conj_b[i])) for i in range(a.n_conj)] + \
           [(b.conj_ops[b.conj_ptr[i]:b.conj_ptr[i + 1]].tolist(), int(b.conj_b[i])) for i in range(b.n_conj)]
    return Axioms.build(n, max(a.n_roles, b.n_roles), kind=kind, sub=cat(a.sub, b.sub), conj=conj,
                        ex_rhs=cat(a.ex_rhs, b.ex_rhs), ex_lhs=cat(a.ex_lhs, b.ex_lhs),
                        subrole=cat(a.subrole, b.subrole), chain=cat(a.chain, b.chain),
                        domain=cat(a.domain, b.domain), range=cat(a.range, b.range))


def classify_partitioned(ax: Axioms, parts: int, devices: Optional[List[int]] = None,
                         rows: Optional[List[Tuple[int, int]]] = None,
                         compat_range: bool = False) -> Tuple[List[Engine], List[Stats]]:
    """Row-partitioned classification in ONE process: ``parts`` engines (one per thread,
    on ``devices`` round-robin, default all on device 0) exchanging their deltas through an
    in-process group (EL_XCHG_LOCAL).  The union of the engines' rows is the closure."""
    import threading
    devices = devices or [0]
    group = LocalGroup(parts)
    engs = [Engine(device=devices[q % len(devices)], compat_range=compat_range,
                   partition=Partition(q, parts, XCHG_LOCAL, group=group, rows=rows[q] if rows else (0, 0)))
            for q in range(parts)]
    engs[0]._group = group  # keep the group alive as long as the engines
    for e in engs:
        e.load(ax)
    stats: List[Optional[Stats]] = [None] * parts
    errs: List[BaseException] = []

    def run(q: int) -> None:
        try:
            engs[q].init()
            stats[q] = engs[q].saturate()
        except BaseException as exc:  # noqa: BLE001 — re-raised below
            errs.append(exc)
    th = [threading.Thread(target=run, args=(q,)) for q in range(parts)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return engs, stats  # type: ignore[return-value]


def merge_facts(engs: List[Engine]) -> Tuple[np.ndarray, np.ndarray]:
    """Union of the partitions' S facts, sorted by (x, a)."""
    parts = [e.facts() for e in engs]
    x = np.concatenate([p[0] for p in parts])
    a = np.concatenate([p[1] for p in parts])
    o = np.lexsort((a, x))
    return x[o], a[o]


def merge_links(engs: List[Engine]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    parts = [e.links() for e in engs]
    x, r, y = (np.concatenate([p[i] for p in parts]) for i in range(3))
    o = np.lexsort((y, r, x))
    return x[o], r[o], y[o]


def classify(ax: Axioms, device: int = 0, profile: bool = False,
             compat_chain: bool = False, compat_range: bool = False) -> Tuple[Engine, Stats]:
    """Load + init + saturate in one call (ELClassifier.classify() over all rule types)."""
    eng = Engine(device=device, profile=profile, compat_chain=compat_chain, compat_range=compat_range)
    eng.load(ax)
    eng.init()
    st = eng.saturate()
    return eng, st
