#!/usr/bin/env python3
"""Benchmark: EL+ classification (DistEL hot path) on MI355X.

One "step" = one full classification of the workload as SURVEY.md §8(d) defines the
metric: from the typed axioms resident in HBM (IR-in-HBM: the told axiom rows el_load
uploads, AxiomLoader's layout) to the fixpoint PLUS the result copy-back — el_init (the told
closure, its exr*/exl* rows, S(X) = {X, ⊤} ∪ told*(X), base links: all derived on the device
inside the step) + el_saturate + el_copy_result (the result rows X -> {B} and the role links
X -> {(r, Y)} as CSR into page-locked host buffers).  Nothing derived is carried from one
step to the next.  ``value`` = derived axioms per second over all ranks (D = Σ|S(X)| − init
facts + Σ|R(r)|).  Default workload: G3, the SNOMED-shaped generator = BASELINE.json
configs[2], the largest config that fits one GPU.  Steps run one at a time, so
``ms_per_step`` = ``classification_wall_s`` = the wall-clock of one classification, copy-back
included (``init_ms`` + ``saturate_ms`` + ``copyback_ms`` split it).  ``throughput_inflight2``
is a separately named figure: two engines (each with its own state and result buffers)
alternate, one's copy-back (EL_RESULT_ASYNC) crossing PCIe while the other classifies.

Multi-GPU (``torch.distributed.run``): weak scaling over the OntologyMultiplier ×N ontology
(BASELINE configs[3]: SNOMED×8 on 8 GPUs).  Two legs, both on the same ×N workload:
  exchange  every rank loads the ×N ontology and runs the row-partitioned engine, rank i owning
            copy i's rows, with the per-superstep RCCL delta all-gather and the delta-count sum
            as the termination test (CommunicationHandler.java:49-84 is the
            barrier it replaces).  This is the headline ``value`` at N > 1.
  copies    rank i classifies only its own copy (the copies share no concepts, so no data-path
            collective: barrier + max-over-ranks only) — reported as ``copies``.
A watchdog bounds the exchange leg: if it fails or has not finished in --exchange-timeout
seconds, rank 0 prints the line with the copies leg as ``value`` and the failure named.

Extra objects on the JSON line:
  roofline      dominant kernel (largest Σ time in a profiled classification):
                algorithmic bytes per launch (all work phases the launch carries) ÷
                average launch time (HIP events on the engine's stream), against the
                8 TB/s HBM peak
  cpu_baseline  the CPU oracle (oracle/el_oracle.c, 1 thread, same Jacobi
                algorithm) on the same workload; the Java/Redis reference cannot run
                on this image (no JVM, no redis-server)
"""
from __future__ import annotations

import argparse
import subprocess
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Two engines in flight use 8 HIP streams; with HIP's default of 4 hardware queues, streams of
# different engines would share a queue and one engine's DMAs would hold up the other's kernels.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "12")
# Load the system ROCm HIP runtime — the one libel_gpu.so is built against — before torch brings
# its bundled copy under the same soname (whichever loads first serves the whole process).  With
# torch's runtime the streamed result's D2H copies into page-locked memory run as blit kernels on
# the CUs (scripts/micro/d2h_py.py: __amd_rocclr_copyBuffer in the trace, ≈14 ms of CU time per G3
# classification beside the supersteps); with the system runtime they go to an SDMA engine.  Every
# world size does this (round 5): the ranks' barrier and reductions run over gloo (dist.py), and the
# data path's RCCL is opened by the engine itself, so torch's RCCL and CUDA process groups are not
# used.  A runtime whose major version differs from the one torch was built for is not preloaded.
# EL_HIP_RUNTIME=torch keeps torch's runtime.
HIP_RUNTIME = {"loaded": "torch", "path": None, "version": None}


def _preload_system_hip():
    path = "/opt/rocm/lib/libamdhip64.so.7"
    if os.environ.get("EL_HIP_RUNTIME", "system") != "system" or "torch" in sys.modules or not os.path.exists(path):
        return
    import ctypes
    import importlib.util
    import re
    real = os.path.realpath(path)  # libamdhip64.so.7.2.70200: the version is in the file name
    m = re.search(r"\.so\.(\d+)\.(\d+)\.(\d+)$", real)
    have = int(m.group(1)) if m else None
    want = None
    try:  # torch.version.hip without importing torch (torch/version.py: hip = '7.0.51831')
        spec = importlib.util.find_spec("torch")
        with open(os.path.join(os.path.dirname(spec.origin), "version.py")) as f:
            m = re.search(r"^hip\b[^=]*=\s*'(\d+)\.", f.read(), re.M)
        want = int(m.group(1)) if m else None
    except (OSError, AttributeError, TypeError):
        pass
    HIP_RUNTIME.update(path=real, version=real.rsplit(".so.", 1)[-1], torch_hip_major=want)
    if have is None or (want is not None and have != want):
        HIP_RUNTIME["loaded"] = f"torch (system runtime major {have} vs torch's {want})"
        return
    ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    HIP_RUNTIME["loaded"] = "system"


_preload_system_hip()
if int(os.environ.get("WORLD_SIZE", "1")) > 1:
    os.environ.setdefault("EL_DIST_BACKEND", "gloo")  # barrier + reductions; the engine opens RCCL itself

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOAD_DESC = {
    "g1": "G1 GO-like synthetic (20k classes, 8 roles, part_of transitive, 1 chain)",
    "g2": "G2 NCI-like synthetic (70k classes, 60 roles, tree-like, no chains) — BASELINE configs[1]",
    "g3": "G3 SNOMED-shaped synthetic (300k classes, 60 roles, 0.3N definitions, 2 chains + 3 transitive) "
          "— BASELINE configs[2]",
    "g3x": "G3X = G3 + 1% sibling disjointness (⊥), domains on 8 roles, ranges on 3",
    "g3e": "G3E = G3 + 1% named equivalences near the roots (told cycles, Normalizer.java:277-279)",
    "g5": "G5 role-heavy synthetic (100k classes, 200 roles, depth-20 chains, hub fillers) — BASELINE configs[4]",
}


class _stdout_to_stderr:
    """Route fd 1 to fd 2 for a block (native libraries write to fd 1 directly): the
    bench's stdout carries exactly one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def source_sha256() -> str:
    """SHA-256 over every file the engine library is compiled from — the HIP / C++ sources and
    their headers, the list __graft_entry__ uses for rebuild detection — so two lines from
    different kernels never share a hash (the kernel table and the PMC summaries name it)."""
    import hashlib
    import __graft_entry__ as ge
    h = hashlib.sha256()
    for f in ge.lib_inputs():
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def pmc_traffic(workload: str, kernel: str):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this workload
    (profiles/pmc/rNN_pmc_<workload>.json, written by scripts/pmc_summary.py from separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected as MI355X_MICROARCH.md
    prescribes).  Used only when the summary was taken on this exact kernel source; else None."""
    import glob
    import hashlib
    try:
        with open(os.path.join(ROOT, "distel_amd", "csrc", "el_gpu.hip"), "rb") as f:
            digest = hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc", f"r*_pmc_{workload}.json")), reverse=True):
        try:
            with open(path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            continue
        if pmc.get("source_sha256") != digest:
            continue
        k = pmc.get("kernels", {}).get(kernel)
        return None if not k or k.get("hbm_bytes_per_dispatch") is None else int(k["hbm_bytes_per_dispatch"])
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="g3", choices=sorted(WORKLOAD_DESC))
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--no-profile", action="store_true", help="skip the profiled roofline pass")
    ap.add_argument("--cpu-procs", type=int, default=16, help="host cores for the cpu_baseline leg (at most 16)")
    ap.add_argument("--no-cpu-full", action="store_true",
                    help="skip the whole-workload one-core oracle run beside the cpu_baseline sample")
    ap.add_argument("--cpu-scale", type=float, default=0.0,
                    help="workload scale of the cpu_baseline sample (default: --scale, capped at ~100 k concepts)")
    ap.add_argument("--partition", default="auto", choices=["auto", "copies", "exchange"],
                    help="N > 1: copies = one disjoint copy per rank, no collective; exchange = row-partitioned "
                         "engine over the ×N ontology with the RCCL delta all-gather; auto (default) = both, "
                         "exchange as the headline")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="exchange leg's all-gather: rccl = ncclAllGather over xGMI on the engine stream; host = "
                         "EL_XCHG_HOST through a gloo group (a rehearsal of N ranks on one GPU)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1 headline: weak = the OntologyMultiplier ×N ontology row-partitioned (configs[3]); "
                         "strong = ONE ontology (the workload itself) row-partitioned over the N ranks, balanced by "
                         "told edges (configs[2] on 1..8 GPUs, the shape DistEL runs).  --partition auto runs both "
                         "at N > 1 and reports the other one beside the headline")
    ap.add_argument("--exchange-timeout", type=float, default=180.0,
                    help="seconds the exchange leg may take before rank 0 reports the copies leg alone")
    ap.add_argument("--inflight", type=int, default=1, choices=[1, 2],
                    help="classifications in flight in the timed loop: 1 = one at a time (the default: "
                         "ms_per_step is one classification's wall-clock); 2 = two engines alternate, one's "
                         "result copy-back (EL_RESULT_ASYNC) rides over PCIe under the other's classification")
    ap.add_argument("--copyback", default="auto", choices=["auto", "packed", "stream", "rows"],
                    help="packed / stream: the result node's facts and links cross PCIe as the supersteps commit "
                         "them (el_stream_result; commit order, row-run encoded; packed = EL_STREAM_PACKED, each "
                         "fact's value a 16-bit column code, escapes for values outside the coded columns); auto: "
                         "stream or packed, whichever classified faster in two untimed probes of each before the "
                         "warmup (max over ranks); rows: after the fixpoint, as sorted CSR rows X -> {B} "
                         "(el_copy_result)")
    ap.add_argument("--no-throughput2", action="store_true",
                    help="skip the separately reported two-in-flight throughput loop")
    ap.add_argument("--increment", type=float, default=0.0,
                    help="N = 1: also time an incremental classification — a random FRAC of every axiom family "
                         "arrives as an increment (el_add_axioms) after the rest is classified; reported as "
                         "`increment` beside the headline (0 = off)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def bind_gpu_numa(dev: int):
    """Pin every thread of this process (the HIP runtime's and torch's worker threads included:
    each thread has its own affinity mask, so all of /proc/self/task are set), and the threads and
    children started later, to the CPUs of its GPU's NUMA node, before any page-locked buffer is
    allocated, so those buffers and the host threads that wait on the device sit next to the GPU's
    PCIe link.  Page-locked memory on the far node halves the D2H rate of the streamed result;
    which node a run lands on otherwise varies from run to run.  EL_NUMA_BIND=0 leaves the affinity
    alone.  Returns what was done (for the bench line)."""
    if os.environ.get("EL_NUMA_BIND", "1") == "0":
        return {"bound": False, "reason": "EL_NUMA_BIND=0"}
    try:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so.7")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, int(dev)) != 0:
            return {"bound": False, "reason": "hipDeviceGetPCIBusId failed"}
        bus = buf.value.decode().lower()
        with open(f"/sys/bus/pci/devices/{bus}/numa_node") as f:
            node = int(f.read())
        if node < 0:
            return {"bound": False, "pci": bus, "node": node}
        cpus = set()
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
        use = cpus & os.sched_getaffinity(0)
        if not use:
            return {"bound": False, "pci": bus, "node": node, "reason": "no allowed CPU on the node"}
        threads = 0
        for tid in os.listdir("/proc/self/task"):
            try:
                os.sched_setaffinity(int(tid), use)
                threads += 1
            except OSError:  # (a thread that ended meanwhile)
                pass
        os.sched_setaffinity(0, use)
        return {"bound": True, "pci": bus, "node": node, "cpus": len(use), "threads": threads}
    except (OSError, ValueError, AttributeError) as e:
        return {"bound": False, "reason": str(e)[:80]}


def d2h_probe(mb: int = 64, reps: int = 4):
    """This process's device -> page-locked host copy rate right now (GB/s): 4 × 64 MB on a
    stream of its own, timed on the host, through the HIP runtime directly (ctypes; every buffer
    and the stream freed after — a torch tensor here would leave torch's streams and caches
    behind, and streams beyond the process's hardware queues share them with the engine's).  The
    streamed result needs the rate: G3's 0.64 GB cross PCIe during ≈18.5 ms of supersteps, and the
    rate measured on the GPU boxes is bimodal — 56 GB/s, or 30 GB/s in some processes and periods
    (scripts/micro/d2h_streams.hip: the same binary in consecutive processes on one box, buffer
    near or far) — so a slow period leaves a copy-back tail.  Reported in the line so a
    tail can be read against it."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so.7")
        n = mb << 20
        d, h, s = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        if hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(n)) != 0:
            return None
        ok = hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(n), 0) == 0
        ok = ok and hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
        gbs = None
        if ok:
            cp = lambda: hip.hipMemcpyAsync(h, d, ctypes.c_size_t(n), 2, s)  # hipMemcpyDeviceToHost
            cp()
            hip.hipStreamSynchronize(s)
            t0 = time.perf_counter()
            for _ in range(reps):
                cp()
            hip.hipStreamSynchronize(s)
            gbs = round(reps * n / (time.perf_counter() - t0) / 1e9, 1)
        if s.value:
            hip.hipStreamDestroy(s)
        if h.value:
            hip.hipHostFree(h)
        hip.hipFree(d)
        return gbs
    except OSError:
        return None


def main():
    args = parse()
    import threading

    import torch

    from distel_amd import dist as D
    from distel_amd import engine, generators, ir

    rk = D.init_from_env()
    world, rank, local = rk.world, rk.rank, rk.local
    has_cuda = torch.cuda.is_available()
    dev = local if has_cuda else 0
    numa = bind_gpu_numa(dev) if has_cuda else None

    t0 = time.time()
    ax = generators.workload(args.workload, args.scale)   # this rank's copy (×world disjoint copies)
    gen_s = time.time() - t0
    run_copies = args.partition != "exchange"
    run_exchange = args.partition == "exchange" or (world > 1 and args.partition == "auto")
    run_strong = args.scaling == "strong" or (world > 1 and args.partition == "auto")

    def timed(engines, steps, warmup):
        """K classifications between barriers.  One engine: each step runs init + saturate +
        copy-back to the end before the next starts.  Two engines: they alternate; a helper
        thread enqueues one engine's copy-back (EL_RESULT_ASYNC; it waits ~1 ms on the device for
        the row counts) while this thread starts the other's classification (ctypes drops the
        GIL inside the library, and the two threads never share an engine); drain() waits for
        the last copy-backs inside the timed region."""
        stream = args.copyback != "rows"
        modes = ["stream", "packed"] if args.copyback == "auto" else [args.copyback]
        results = [{m: engine.Stream(packed=m == "packed") for m in modes} if stream else engine.Result()
                   for _ in engines]  # page-locked, reused
        cur = [modes[0]]  # page-locked, reused
        split = []  # (init, saturate, copy-back) seconds per step; the last `steps` are the timed ones
        turn = [0]
        pool = ThreadPoolExecutor(max_workers=1) if len(engines) == 2 else None
        copying = [None] * len(engines)

        def classify():
            i = turn[0] % len(engines)
            turn[0] += 1
            e, res = engines[i], (results[i][cur[0]] if stream else results[i])
            if copying[i] is not None:
                copying[i].result()  # (the enqueue finished long ago; errors surface here)
                copying[i] = None
            t0 = time.perf_counter()
            e.init()
            t1 = time.perf_counter()
            if stream:  # the result crosses PCIe while the supersteps run
                e.stream_result(res, release=True)
            st = e.saturate()
            t2 = time.perf_counter()
            if stream:
                if pool is None:
                    e.result_wait()  # (two in flight: the next turn of this engine, or drain(), waits)
            elif pool is None:
                e.copy_result(res, release=True)
            else:
                copying[i] = pool.submit(e.copy_result, res, release=True, wait=False)
            split.append((t1 - t0, t2 - t1, time.perf_counter() - t2))
            return st

        def drain():
            for i, e in enumerate(engines):
                if copying[i] is not None:
                    copying[i].result()
                    copying[i] = None
                e.result_wait()

        probe = None
        if len(modes) > 1:  # auto: two untimed classifications with each encoding, the faster kept
            probe = {m: [] for m in modes}
            for _ in range(2):
                for m in modes:
                    cur[0] = m
                    t0 = time.perf_counter()
                    classify()
                    drain()
                    probe[m].append(time.perf_counter() - t0)
            probe = {m: 1e3 * D.allreduce(rk, min(v), "max") for m, v in probe.items()}
            cur[0] = min(modes, key=lambda m: probe[m])
        split.clear()
        t_max, derived_all, st = D.run_weak(rk, classify, steps, warmup, drain=drain)
        if pool is not None:
            pool.shutdown()
        results = [r[cur[0]] if stream else r for r in results]
        for r in results:
            assert (r.n_facts, r.n_links) == (st["s_facts"], st["links"]) or (len(ax.range) and not stream) or \
                engines[0].partition is not None, "copy-back lost facts"
        res = results[(turn[0] - 1) % len(engines)]
        copy_bytes = (res.bytes() if stream else
                      8 * 2 * (res.row_hi - res.row_lo + 1) + 4 * (res.n_facts + res.n_links))
        sp = split[-steps:]
        return {"t_max": t_max, "derived": derived_all, "st": st, "ms_per_step": 1e3 * t_max / steps,
                "value": derived_all * steps / t_max, "copy_bytes": int(copy_bytes),
                "init_ms": 1e3 * sum(t[0] for t in sp) / len(sp), "saturate_ms": 1e3 * sum(t[1] for t in sp) / len(sp),
                "copyback_ms": 1e3 * sum(t[2] for t in sp) / len(sp), "inflight": len(engines),
                "encoding": cur[0] if stream else "rows", "probe_ms": probe}

    # (diagnostic, EL_D2H_PROBE=1: this process's D2H rate before any engine exists)
    d2h = {"before": d2h_probe()} if has_cuda and rank == 0 and os.environ.get("EL_D2H_PROBE") == "1" else None
    legs = {}
    if run_copies:
        # whole ontology (N = 1) / this rank's own copy (N > 1): no data-path collective
        eng = engine.Engine(device=dev)
        t0 = time.time()
        eng.load(ax)  # host index build + upload: AxiomLoader's part, reported separately
        load_s = time.time() - t0
        engines = [eng]
        if args.inflight == 2:
            eng2 = engine.Engine(device=dev)
            eng2.load(ax)
            engines.append(eng2)
        legs["copies"] = timed(engines, args.steps, args.warmup)
        legs["copies"]["load_s"] = load_s
        if len(engines) == 1 and world == 1 and not args.no_throughput2:
            eng2 = engine.Engine(device=dev)
            eng2.load(ax)
            t2 = timed([eng, eng2], args.steps, args.warmup)
            eng2.close()
            legs["copies"]["throughput2"] = {
                "value": round(t2["value"], 1), "unit": "axioms/s",
                "ms_per_classification": round(t2["ms_per_step"], 4), "steps": args.steps,
                "schedule": "two engines alternate; one's result copy-back (EL_RESULT_ASYNC) overlaps "
                            "the other's classification"}
        for e in engines:
            e.close()

    def increment_leg():
        """the base classified (untimed), then el_add_axioms(increment) +
        el_saturate timed — the delta the reference's currInc-scored first iteration processes
        (Type1_1AxiomProcessor.java:138-141); K repetitions, each from a freshly classified base."""
        base, inc = ir.split_increment(ax, args.increment, seed=11)
        e = engine.Engine(device=dev)
        rows = []
        for k in range(args.warmup + args.steps):
            e.load(base)
            e.init()
            e.saturate()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e.add_axioms(inc)
            t1 = time.perf_counter()
            st = e.saturate()
            t2 = time.perf_counter()
            if k >= args.warmup:
                rows.append((t1 - t0, t2 - t1, st, e.increment_info()))
        e.close()
        add_ms = 1e3 * sum(r[0] for r in rows) / len(rows)
        sat_ms = 1e3 * sum(r[1] for r in rows) / len(rows)
        avg = lambda k: sum(r[3][k] for r in rows) / len(rows)
        st, info = rows[-1][2], rows[-1][3]
        # the classification part of an increment: the device state carried over (the told
        # closure of the new index, CSRs, sets, re-trigger lists) + the saturation; the host index
        # build and its upload are AxiomLoader's part, reported apart as for el_load
        cls_ms = avg("migrate_ms") + sat_ms
        return {"frac": args.increment, "axioms": inc.counts(), "add_axioms_ms": round(add_ms, 4),
                "index_ms": round(avg("index_ms"), 4), "upload_ms": round(avg("upload_ms"), 4),
                "migrate_ms": round(avg("migrate_ms"), 4), "saturate_ms": round(sat_ms, 4),
                "classification_ms": round(cls_ms, 4), "ms": round(add_ms + sat_ms, 4),
                "supersteps": st["supersteps"],
                "retrigger": [info["retrigger_facts"], info["retrigger_links"]],
                "facts_after": st["s_facts"], "links_after": st["links"], "derived_after": st["derived"],
                "schedule": "el_add_axioms (indexes rebuilt, state carried over, re-trigger lists of the facts and "
                            "links the new axioms reach) + el_saturate (first superstep over those lists, then "
                            "semi-naive); no result copy-back"}

    def profile_once(peng, workload, pmc, encoding):
        """One classification of an engine already loaded, in the timed schedule (streamed copy-back
        armed), with HIP events around every launch on its engine stream: the dominant kernel
        (largest Σ time; phases sharing a launch add their algorithmic bytes) as `roofline`, and
        the whole table.  A partitioned engine runs it on every rank together (collectives)."""
        peng.init()
        if encoding != "rows":
            peng.stream_result(engine.Stream(packed=encoding == "packed"))  # (not released: counters read after)
        pst = peng.saturate()
        if encoding != "rows":
            peng.result_wait()
        ks = peng.kernel_stats()
        launches = {}
        for k in ks:
            g = launches.setdefault(k["group"], {"kernel": k["group"].split(":")[0], "launches": 0, "ms": 0.0,
                                                 "bytes": 0})
            g["bytes"] += k["bytes"]
            if k["kernel"] == k["group"]:
                g["launches"], g["ms"] = k["launches"], k["ms"]
        prof = [g for g in launches.values() if g["launches"] and g["ms"] > 0]
        dom = max(prof, key=lambda g: g["ms"])
        per_launch_bytes = dom["bytes"] / dom["launches"]
        avg_ms = dom["ms"] / dom["launches"]
        achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": pmc_traffic(workload, dom["kernel"]) if pmc else None,
                "kernel": dom["kernel"], "bytes_per_launch": int(per_launch_bytes),
                "avg_launch_us": round(avg_ms * 1e3, 3), "launches": dom["launches"],
                "profiled_ms": round(pst["ms"], 3),
                "source": "HIP events around every launch on the engine stream of one profiled classification "
                          "in the timed schedule; the whole table is this line's `kernels` "
                          "(launches, ms, algorithmic bytes per kernel)"}
        table = {g["kernel"]: {"launches": g["launches"], "ms": round(g["ms"], 4), "bytes": g["bytes"]}
                 for g in launches.values() if g["launches"]}
        return roof, table

    def exchange_leg(strong=False):
        """weak: the ×N ontology, rank i owning copy i's rows; strong: the workload itself, the
        rows balanced by told edges (ir.balanced_rows) — one ontology's concept space sharded
        over the ranks, every R(r) link into another rank's rows crossing the exchange."""
        if strong:
            full = ax
            rows = ir.balanced_rows(ax, world)[rank] if world > 1 else (0, ax.n_concepts)
        else:
            full = ir.replicate(ax, world) if world > 1 else ax
            rows = ir.copy_slice(ax, world, rank) if world > 1 else (0, ax.n_concepts)
            if rank == 0:
                rows = (0, rows[1])  # ⊥ and ⊤ live on rank 0
        if args.transport == "host":
            group = rk.dist.new_group(backend="gloo") if world > 1 else None
            part = engine.Partition(rank, world, engine.XCHG_HOST, rows=rows,
                                    allgather=engine.gloo_allgather(group) if world > 1 else
                                    (lambda send, recv: recv.__setitem__(slice(None), send)))
        else:
            uid = engine.rccl_unique_id() if rank == 0 else None
            if world > 1:
                box = [uid]
                rk.dist.broadcast_object_list(box, src=0)
                uid = box[0]
            part = engine.Partition(rank, world, engine.XCHG_RCCL, rccl_id=uid, rows=rows)
        with _stdout_to_stderr():  # RCCL prints its version banner on stdout at communicator init
            xeng = engine.Engine(device=dev, partition=part)
        t0 = time.time()
        xeng.load(full)
        load_s = time.time() - t0
        leg = timed([xeng], args.steps, args.warmup)
        leg["load_s"] = load_s
        leg["rows"] = rows
        if not args.no_profile:
            # per-rank roofline (round-5 verdict #1): one more classification of the partitioned
            # context with HIP events on, every rank together; the line carries the slowest rank's
            # dominant kernel (PMC traffic is measured on the N = 1 schedule only: null here)
            xeng.set_profile(True)
            roof, table = profile_once(xeng, args.workload, pmc=False, encoding=leg["encoding"])
            xeng.set_profile(False)
            allr = D.gather_objects(rk, (roof, table))
            slow = max(range(len(allr)), key=lambda i: allr[i][0]["profiled_ms"])
            roof = dict(allr[slow][0])
            roof["rank"] = slow
            roof["per_rank"] = [{"rank": i, "kernel": r[0]["kernel"], "frac": r[0]["frac"],
                                 "avg_launch_us": r[0]["avg_launch_us"], "profiled_ms": r[0]["profiled_ms"]}
                                for i, r in enumerate(allr)]
            roof["source"] = ("HIP events around every launch on each rank's engine stream, one profiled "
                              "classification of the partitioned context in the timed schedule (all ranks "
                              "together); the slowest rank's dominant kernel; `kernels` is that rank's table")
            leg["profile"] = {"roofline": roof, "kernels": allr[slow][1]}
        xeng.close()
        return leg

    def build_line(head, head_name, extra):
        st = head["st"]
        copies = legs.get("copies")
        return {
            "metric": "derived_axioms_per_sec (EL+ classification, SURVEY.md §8(d))",
            "value": round(head["value"], 1),
            "unit": "axioms/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "strong" if head_name == "strong" else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": WORKLOAD_DESC[args.workload] + (f" ×scale {args.scale}" if args.scale != 1 else "")
                       + (f", OntologyMultiplier ×{world}" if world > 1 and head_name != "strong" else ""),
                       "concepts_per_rank": ax.n_concepts, "roles": ax.n_roles, "axioms": ax.counts(),
                       "parallelism": (f"row partition of the ×{world} ontology over {world} GPUs (rank i owns copy "
                                       f"i's rows), {'RCCL' if args.transport == 'rccl' else 'host-staged gloo'} "
                                       f"delta all-gather + delta-count sum per superstep"
                                       if head_name == "exchange" else
                                       f"row partition of ONE ontology over {world} GPUs (rows balanced by told "
                                       f"edges), {'RCCL' if args.transport == 'rccl' else 'host-staged gloo'} "
                                       f"delta all-gather + delta-count sum per superstep"
                                       if head_name == "strong" else
                                       f"{world} disjoint copies, one per GPU, no data-path collective"
                                       if world > 1 else "one GPU, whole ontology"),
                       "schedule": ("two classifications in flight per GPU: one's result copy-back "
                                    "(EL_RESULT_ASYNC) overlaps the other's classification"
                                    if head["inflight"] == 2 else "one classification at a time, copy-back included")},
            "classification_wall_s": round(head["ms_per_step"] / 1e3, 6) if head["inflight"] == 1 else None,
            "derived_axioms": head["derived"],
            "s_facts_per_rank": st["s_facts"],
            "links_per_rank": st["links"],
            "supersteps": st["supersteps"],
            "load_s": round(head["load_s"], 3),
            "generate_s": round(gen_s, 3),
            "inflight": head["inflight"],
            "init_ms": round(head["init_ms"], 4),
            "saturate_ms": round(head["saturate_ms"], 4),
            "copyback_ms": round(head["copyback_ms"], 4),
            "latency_ms": round(head["ms_per_step"], 4) if head["inflight"] == 1 else None,
            "copyback": ("streamed: the result node's facts and links in commit order, row-run encoded "
                         "(B / pair id per entry + (X, end) per run), crossing PCIe as the supersteps commit "
                         "them (el_stream_result)" + ("; packed: B as a 16-bit column code, escapes for B outside "
                                                      "the coded columns (EL_STREAM_PACKED)"
                                                      if head["encoding"] == "packed" else "")
                         if args.copyback != "rows" else
                         "rows: S(X) and links as sorted CSR rows after the fixpoint (el_copy_result)"),
            "copyback_bytes": head["copy_bytes"],
            "copyback_encoding": head["encoding"],
            "copyback_probe_ms": ({m: round(v, 3) for m, v in head["probe_ms"].items()} if head["probe_ms"] else None),
            "copyback_gbs": (round(head["copy_bytes"] / (head["copyback_ms"] * 1e-3) / 1e9, 2)
                             if head["copyback_ms"] > 0 and args.copyback == "rows" else None),
            "throughput_inflight2": copies.get("throughput2") if copies else None,
            **extra,
        }

    def leg_summary(leg):
        xb = leg["st"].get("exchange_bytes", 0)
        return {"value": round(leg["value"], 1), "ms_per_step": round(leg["ms_per_step"], 4),
                "derived_axioms": leg["derived"], "supersteps": leg["st"]["supersteps"],
                "init_ms": round(leg["init_ms"], 4), "saturate_ms": round(leg["saturate_ms"], 4),
                "copyback_ms": round(leg["copyback_ms"], 4), "load_s": round(leg["load_s"], 3), "rows_rank0": leg.get("rows"),
                "exchange_bytes_per_rank": xb,
                "exchange_bytes_per_superstep": round(xb / max(leg["st"]["supersteps"], 1), 1)}

    def pick_head():
        order = (["strong", "exchange"] if args.scaling == "strong" else ["exchange", "strong"]) + ["copies"]
        for name in order:
            if name in legs:
                return name
        return None

    if args.increment > 0 and world == 1:
        legs["increment"] = increment_leg()
    xlegs = ([("exchange", False)] if run_exchange else []) + ([("strong", True)] if run_strong else [])
    if xlegs:
        done = threading.Event()

        def fallback(err):
            """A partitioned leg failed or hangs: rank 0 prints the line from the legs that finished."""
            name = pick_head()
            if rank == 0 and name is not None:
                extra = {"roofline": None, "cpu_baseline": None, "errors": err}
                for n in ("copies", "exchange", "strong"):
                    extra[n] = leg_summary(legs[n]) if n in legs else None
                print(json.dumps(build_line(legs[name], name, extra)), flush=True)
            os._exit(0 if name is not None else 1)

        def watchdog():
            if not done.wait(args.exchange_timeout * len(xlegs)):
                fallback({"timeout": f"partitioned legs unfinished after {args.exchange_timeout * len(xlegs):.0f} s"})
        threading.Thread(target=watchdog, daemon=True).start()
        for name, strong in xlegs:
            try:
                legs[name] = exchange_leg(strong)
            except Exception as exc:  # noqa: BLE001 — reported on the line; the other ranks' watchdogs end them
                err = f"{type(exc).__name__}: {exc}"
                print(f"rank {rank}: {name} leg failed: {err}", file=sys.stderr, flush=True)
                fallback({name: err})
        done.set()
    head_name = pick_head()
    head = legs[head_name]
    st = head["st"]

    roofline = None
    kernels = None
    head_prof = head.get("profile")
    if head_prof is not None:  # N > 1: the partitioned leg profiled on every rank, the slowest rank's
        roofline, kernels = head_prof["roofline"], head_prof["kernels"]
    elif rank == 0 and not args.no_profile:
        # profiled classification in the timed step's schedule (the streamed copy-back beside the
        # supersteps): HIP events bracket every launch on the engine stream
        peng = engine.Engine(device=dev, profile=True)
        peng.load(ax)
        roofline, kernels = profile_once(peng, args.workload, pmc=True, encoding=head["encoding"])
        peng.close()

    cpu = None
    if rank == 0 and not args.no_cpu:
        # cpu_baseline leg: the CPU oracle, timed in a child process that never touches the GPU
        # (oracle/cpu_baseline.py): one classification alone (1 core) and P concurrent ones,
        # one per host core (P = the box's CPU share, at most 16).  Reported value: P cores.
        # the oracle keeps an N²-bit matrix per classification: stay within ~160 GB of host memory
        # (the GPU box allows 270 GiB per command)
        # bounded sample: the same generator at a scale of at most ~100 k concepts (one oracle
        # classification ≈ 15-20 s; full G3 takes the oracle ≈ 216 s, and its rate per axiom is
        # lower there, so the sample flatters the CPU)
        cpu_scale = args.scale if args.cpu_scale <= 0 else args.cpu_scale
        cpu_scale = min(cpu_scale, args.scale * 100_000 / ax.n_concepts)
        n_cpu = int(ax.n_concepts * cpu_scale / args.scale)
        per_run = 1.5 * n_cpu * n_cpu / 8
        procs = max(1, min(16, os.cpu_count() or 1, args.cpu_procs, int(160e9 // per_run)))
        try:
            out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), args.workload,
                                  str(cpu_scale), str(procs)], check=True, capture_output=True, text=True).stdout
            cb = json.loads(out.strip().splitlines()[-1])
        except (subprocess.SubprocessError, OSError, ValueError, IndexError) as exc:
            cb = {"error": f"{type(exc).__name__}: {str(exc)[:200]}"}
    if rank == 0 and cpu is None and not args.no_cpu and "error" in cb:
        cpu = {"value": None, "unit": "axioms/s", "cores": procs, "kind": "port", "sample": None, "error": cb["error"]}
    elif rank == 0 and not args.no_cpu:
        cpu = {"value": round(cb["derived"] / cb["wall_s"], 1), "unit": "axioms/s", "cores": procs, "kind": "port",
               "sample": f"{procs} concurrent classifications of {args.workload} at scale {cpu_scale:.4g} "
                         f"(≈{n_cpu} concepts, {cb['single_derived']} derived axioms each) by the CPU oracle "
                         f"(semi-naive Jacobi, 1 thread each, one per core): {cb['wall_s']:.3f} s wall; "
                         f"one alone: {cb['single_s']:.3f} s",
               "value_1core": round(cb["single_derived"] / cb["single_s"], 1),
               "classification_s": round(cb["single_s"], 4),
               # the span the GPU step times: the told closure and its rows (elo_create's index
               # build; el_init on the GPU) + init + saturation
               "closure_index_s": round(cb["single_create_s"], 4),
               "init_saturate_s": round(cb["single_s"] - cb["single_create_s"], 4)}
        if cpu_scale == args.scale and world == 1:
            cpu["parity_derived_equal"] = cb["single_derived"] == st["derived"]
        if world == 1 and cpu_scale < args.scale and not args.no_cpu_full:
            # beside the sample: the whole workload classified by the oracle on one host core
            # (G3: ≈15 s, 19 GB of host memory for its bit matrix); a failure (e.g. the child
            # killed for memory) is reported in the line instead of losing the measured GPU result
            try:
                out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), args.workload,
                                      str(args.scale), "1"], check=True, capture_output=True, text=True).stdout
                fb = json.loads(out.strip().splitlines()[-1])
                cpu["full_1core"] = {"value": round(fb["single_derived"] / fb["single_s"], 1), "unit": "axioms/s",
                                     "classification_s": round(fb["single_s"], 4),
                                     "closure_index_s": round(fb["single_create_s"], 4),
                                     "derived": fb["single_derived"],
                                     "parity_derived_equal": fb["single_derived"] == st["derived"],
                                     "sample": f"the whole {args.workload} workload, one classification by the CPU "
                                               f"oracle on one core"}
            except (subprocess.SubprocessError, OSError, ValueError, KeyError, IndexError) as exc:
                cpu["full_1core"] = {"error": f"{type(exc).__name__}: {str(exc)[:200]}"}

    if rank == 0:
        extra = {}
        if world > 1 or "exchange" in legs or "strong" in legs:
            for n in ("copies", "exchange", "strong"):
                extra[n] = leg_summary(legs[n]) if n in legs else None
        if "increment" in legs:
            inc = dict(legs["increment"])
            inc["vs_full_classification"] = round(inc["classification_ms"] / head["ms_per_step"], 4)
            inc["with_index_vs_full"] = round(inc["ms"] / head["ms_per_step"], 4)
            extra["increment"] = inc
        extra["roofline"] = roofline
        extra["cpu_baseline"] = cpu
        extra["numa"] = numa
        extra["hip_runtime"] = HIP_RUNTIME
        if d2h is not None:
            extra["d2h_gbs"] = d2h
        extra["lib"] = os.path.relpath(engine.load_library()._name, ROOT)
        line = build_line(head, head_name, extra)
        if kernels:  # the record roofline is computed from (HIP events, the profiled classification)
            line["kernels"] = kernels
            line["source_sha256"] = source_sha256()
        print(json.dumps(line), flush=True)
    D.shutdown(rk)


if __name__ == "__main__":
    main()
