"""Cross-process row partition: one process per rank, deltas all-gathered
every superstep through the caller's transport (EL_XCHG_HOST over gloo).

CPU: the transport callback as the library calls it (a C function pointer through ctypes) at
world size 2.  GPU: two child processes, each with its own partitioned context on the one
GPU of the lease, classify an OntologyMultiplier ×2 ontology (and an unaligned equal split);
the union of their rows must be bit-exactly the oracle's closure and their supersteps agree."""
import ctypes as C
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cb_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from distel_amd import engine
    dist.init_process_group(backend="gloo")
    part = engine.Partition(rank, world, engine.XCHG_HOST, allgather=engine.gloo_allgather())
    fn = C.cast(part._cfn, C.c_void_p).value
    call = engine._ALLGATHER(fn)  # as the library calls it: a plain C function pointer
    ok = True
    for n in (1, 7, 4096, 300_001):
        send = (C.c_uint8 * n)(*([(rank * 31 + i) % 251 for i in range(n)] if n < 5000 else []))
        if n >= 5000:
            C.memset(send, 17 + rank, n)
        recv = (C.c_uint8 * (n * world))()
        rc = call(None, C.addressof(send), C.addressof(recv), n)
        got = np.frombuffer(recv, dtype=np.uint8).reshape(world, n)
        for r in range(world):
            exp = (np.array([(r * 31 + i) % 251 for i in range(n)], dtype=np.uint8) if n < 5000 else
                   np.full(n, 17 + r, dtype=np.uint8))
            ok &= rc == 0 and np.array_equal(got[r], exp)
    # a transport that raises returns nonzero to the library, the exception kept for the caller
    bad = engine.Partition(rank, world, engine.XCHG_HOST, allgather=lambda s, r: 1 / 0)
    rc = engine._ALLGATHER(C.cast(bad._cfn, C.c_void_p).value)(None, C.addressof(send), C.addressof(recv), 1)
    ok &= rc == 1 and isinstance(bad.error, ZeroDivisionError)
    q.put((rank, bool(ok)))
    dist.destroy_process_group()


def test_host_allgather_callback_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cb_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == [(0, True), (1, True)]


def _run_ranks(tmp_path, name, scale, copies, world=2, timeout=300):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_RANK="0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "xproc_worker.py"), name,
                                       str(scale), str(copies), str(tmp_path)], env=env))
    try:
        for p in procs:
            assert p.wait(timeout=timeout) == 0, "a rank failed"
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    parts = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    stats = [json.load(open(os.path.join(tmp_path, f"rank{r}.json"))) for r in range(world)]
    x = np.concatenate([p["x"] for p in parts])
    a = np.concatenate([p["a"] for p in parts])
    o = np.lexsort((a, x))
    lx, lr, ly = (np.concatenate([p[k] for p in parts]) for k in ("lx", "lr", "ly"))
    ol = np.lexsort((ly, lr, lx))
    return (x[o], a[o]), (lx[ol], lr[ol], ly[ol]), stats


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale,copies", [("g3", 0.02, 2), ("g3x", 0.02, 2), ("g5", 0.02, 1)])
def test_two_processes_host_exchange(tmp_path, name, scale, copies, oracle_lib):
    from distel_amd import generators, ir
    (fx, fa), links, stats = _run_ranks(tmp_path, name, scale, copies)
    base = generators.workload(name, scale)
    ax = ir.replicate(base, copies) if copies > 1 else base
    o = oracle_lib.saturate(ax, 0)
    ox, oa = o.facts()
    assert np.array_equal(fx, ox) and np.array_equal(fa, oa), "S(X) differs from the oracle"
    for g, c in zip(links, o.links()):
        assert np.array_equal(g, c), "R(r) differs from the oracle"
    assert sum(s["derived"] for s in stats) == o.stats()["derived"]
    assert len({s["supersteps"] for s in stats}) == 1  # lock-step supersteps across processes
