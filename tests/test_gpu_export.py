"""GPU result export and copy-back against the CPU oracle.

The result node X -> {B} (ResultRearranger DB1, ResultRearranger.java:57-105) and the role
links come back through el_copy_result (CSR rows built on the device, el_rows.hip),
el_export_result (B_TO_X = result node DB0, X_TO_B = DB1), el_get_subsumers and the
el_copy_facts / el_copy_links triples.  Every path is compared with the oracle's closure —
bit-exact, rows ascending — including rows on each of the row-sort paths (≤ 64 entries:
register sort; ≤ 4096: LDS sort; longer: bit-matrix read-out for S rows, global sort for link
rows).
"""
import os

import numpy as np
import pytest

import kat
from distel_amd import engine, generators, ir

pytestmark = pytest.mark.gpu


def _oracle_rows(o, n):
    ox, oa = o.facts()
    ptr = np.zeros(n + 1, np.uint64)
    np.add.at(ptr, ox.astype(np.int64) + 1, 1)
    return np.cumsum(ptr).astype(np.uint64), oa


def _check_result(eng, o, ax, pinned=True):
    res = eng.copy_result(pinned=pinned)
    assert (res.row_lo, res.row_hi) == (0, ax.n_concepts)
    # the caller's rows (the oracle's stats count ELK range fillers' rows too, like el_stats)
    assert res.n_facts == len(o.facts()[0]) and res.n_links == len(o.links()[0])
    ptr, oa = _oracle_rows(o, ax.n_concepts)
    assert np.array_equal(res.s_ptr, ptr)
    assert np.array_equal(res.s_val[:res.n_facts], oa)
    # links: pair q -> (role, filler); rows ascending in q = ascending in (role, filler)
    role, filler = eng.pair_table()
    assert res.n_pairs == role.size
    key = role.astype(np.uint64) << np.uint64(32) | filler.astype(np.uint64)
    assert np.all(np.diff(key.astype(np.int64)) > 0)
    lx, lr, ly = o.links()
    lptr = np.zeros(ax.n_concepts + 1, np.uint64)
    np.add.at(lptr, lx.astype(np.int64) + 1, 1)
    assert np.array_equal(res.l_ptr, np.cumsum(lptr).astype(np.uint64))
    q = res.l_pair[:res.n_links]
    assert np.array_equal(role[q], lr) and np.array_equal(filler[q], ly)
    return res


def test_copy_result_g2(oracle_lib):
    ax = generators.workload("g2")
    eng, _ = engine.classify(ax, device=0)
    o = oracle_lib.saturate(ax, 0)
    _check_result(eng, o, ax, pinned=True)
    _check_result(eng, o, ax, pinned=False)  # pageable buffers: staged by the runtime
    # a second classification into the same (reused) buffers
    res = engine.Result()
    eng.init()
    eng.saturate()
    eng.copy_result(res)
    eng.init()
    eng.saturate()
    eng.copy_result(res)
    x, a = res.facts()
    ox, oa = o.facts()
    assert np.array_equal(x, ox) and np.array_equal(a, oa)
    eng.close()


@pytest.mark.parametrize("path", kat.kat_files(), ids=lambda p: os.path.basename(p))
def test_copy_result_kat(path, oracle_lib):
    ax, _ = kat.load_kat(path)
    eng, _ = engine.classify(ax, device=0)
    _check_result(eng, oracle_lib.saturate(ax, 0), ax)
    eng.close()


def _long_rows_ontology():
    """One concept with 5,000 told subsumers (a long S row: bit-matrix read-out), one with
    6,000 existentials (a long link row: global sort), one with 300 of each (LDS sort)."""
    n = 2 + 3 + 6000
    big_s, big_l, mid = 2, 3, 4
    fill = list(range(5, n))
    rng = np.random.default_rng(3)
    sub = [(big_s, int(b)) for b in rng.permutation(fill)[:5000]]
    sub += [(mid, int(b)) for b in rng.permutation(fill)[:300]]
    ex = [(big_l, int(rng.integers(0, 3)), int(b)) for b in rng.permutation(fill)[:6000]]
    ex += [(mid, int(rng.integers(0, 3)), int(b)) for b in rng.permutation(fill)[:300]]
    return ir.Axioms.build(n, 3, sub=sub, ex_rhs=ex)


def test_copy_result_long_rows(oracle_lib):
    ax = _long_rows_ontology()
    eng, _ = engine.classify(ax, device=0)
    o = oracle_lib.saturate(ax, 0)
    res = _check_result(eng, o, ax)
    assert int(res.s_ptr[3] - res.s_ptr[2]) > 4096 and int(res.l_ptr[4] - res.l_ptr[3]) > 4096
    eng.close()


def test_export_and_subsumers_g2(oracle_lib):
    """el_export_result (both layouts) and el_get_subsumers against the oracle, after the
    result node's filter (no ⊥ row, no datatype rows; ResultRearranger.java:57-105)."""
    ax = generators.workload("g2", scale=0.3)
    eng, _ = engine.classify(ax, device=0)
    o = oracle_lib.saturate(ax, 0)
    ox, oa = o.facts()
    keep = (ox != 0) & (ax.kind[ox] != 3)
    k, v = eng.export_result(engine.LAYOUT_X_TO_B)
    assert np.array_equal(k, ox[keep]) and np.array_equal(v, oa[keep])
    kb, vb = eng.export_result(engine.LAYOUT_B_TO_X)
    o2 = np.lexsort((ox[keep], oa[keep]))
    assert np.array_equal(kb, oa[keep][o2]) and np.array_equal(vb, ox[keep][o2])
    rng = np.random.default_rng(5)
    for x in rng.integers(0, ax.n_concepts, 200).tolist() + [0, 1, ax.n_concepts - 1]:
        assert np.array_equal(eng.subsumers(x), oa[ox == x])
    gx, ga = eng.facts()
    assert np.array_equal(gx, ox) and np.array_equal(ga, oa)
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c)
    eng.close()


def test_copy_result_small_buffers():
    ax = generators.workload("g1", scale=0.05)
    eng, st = engine.classify(ax, device=0)
    import ctypes as C
    r = engine._ElResult()
    small = np.zeros(4, np.uint32)
    r.s_val = small.ctypes.data_as(C.POINTER(C.c_uint32))
    r.s_cap = small.size
    assert eng._lib.el_copy_result(eng._ctx, C.byref(r)) == engine.EL_ERANGE
    assert r.n_facts == st["s_facts"]
    eng.close()


def test_copy_result_empty():
    ax = ir.Axioms.build(2, 0)
    eng, _ = engine.classify(ax, device=0)
    res = eng.copy_result()
    assert res.n_facts == 2 and res.n_links == 0
    assert res.s_ptr.tolist() == [0, 1, 2] and res.s_val[:2].tolist() == [0, 1]
    eng.close()


def test_copy_result_release(oracle_lib):
    """EL_RESULT_RELEASE: the copy is the closure, the engine then has no state until init(),
    and the reset done behind the copy-back leaves a clean start (same closure again)."""
    ax = generators.workload("g1", scale=0.3)
    o = oracle_lib.saturate(ax, 0)
    eng = engine.Engine(device=0)
    eng.load(ax)
    res = engine.Result()
    for _ in range(3):
        eng.init()
        eng.saturate()
        eng.copy_result(res, release=True)
        x, a = res.facts()
        ox, oa = o.facts()
        assert np.array_equal(x, ox) and np.array_equal(a, oa)
        with pytest.raises(engine.ElError):
            eng.subsumers(2)
        with pytest.raises(engine.ElError):
            eng.saturate()
    eng.init()
    eng.saturate()
    _check_result(eng, o, ax)
    eng.close()


def _result_digest(res, role, filler):
    """SHA-256 of a copy-back in the pinned digests' format (tests/golden/closure_digests.txt):
    facts (x, a) then links (x, r, y), each lexicographically sorted."""
    import hashlib
    x, a = res.facts()
    n = res.row_hi - res.row_lo
    lx = np.repeat(np.arange(res.row_lo, res.row_hi, dtype=np.uint32), np.diff(res.l_ptr[:n + 1]).astype(np.int64))
    q = res.l_pair[:res.n_links]
    h = hashlib.sha256()
    for arr in (x, a, lx, role[q], filler[q]):
        h.update(np.ascontiguousarray(arr, dtype=np.uint32).tobytes())
    return h.hexdigest()


def test_copy_result_release_g3_pinned():
    """The bench's step at full G3 — init, saturate, copy-back with release (S rows by bit-matrix
    read-out, the next reset beside it) — twice, each copy hashing to the closure digest the
    oracle and the independent worklist saturator agreed on."""
    want = None
    for line in open(os.path.join(os.path.dirname(__file__), "golden", "closure_digests.txt")):
        f = line.split()
        if len(f) == 4 and f[0] == "g3" and float(f[1]) == 1.0:
            want = f[3]
    assert want
    ax = generators.workload("g3")
    eng = engine.Engine(device=0)
    eng.load(ax)
    role, filler = eng.pair_table()
    res = engine.Result()
    for _ in range(2):
        eng.init()
        eng.saturate()
        eng.copy_result(res, release=True)
        assert _result_digest(res, role, filler) == want
    eng.close()


def _g3_digest():
    for line in open(os.path.join(os.path.dirname(__file__), "golden", "closure_digests.txt")):
        f = line.split()
        if len(f) == 4 and f[0] == "g3" and float(f[1]) == 1.0:
            return f[3]
    raise AssertionError("no pinned G3 digest")


def test_copy_result_async_two_engines_g3():
    """The bench's pipelined schedule at full G3: two engines alternate, each copy-back enqueued
    with EL_RESULT_ASYNC so it lands while the other engine saturates.  Every copy — read after
    result_wait(), or after the engine's next call waited for it — hashes to the pinned digest."""
    want = _g3_digest()
    ax = generators.workload("g3")
    engs = [engine.Engine(device=0) for _ in range(2)]
    for e in engs:
        e.load(ax)
    role, filler = engs[0].pair_table()
    results = [engine.Result(), engine.Result()]
    for i in range(5):
        e, res = engs[i % 2], results[i % 2]
        e.init()  # (waits for this engine's previous copy-back)
        e.saturate()
        e.copy_result(res, release=True, wait=False)
        if i >= 1:  # the other engine's copy-back landed behind this saturation
            o = engs[(i + 1) % 2]
            o.result_wait()
            assert _result_digest(results[(i + 1) % 2], role, filler) == want
    engs[0].result_wait()
    assert _result_digest(results[0], role, filler) == want
    with pytest.raises(ValueError):
        engs[1].copy_result(results[1], wait=False)  # asynchronous needs release
    for e in engs:
        e.close()


def test_copy_result_async_g2_close_in_flight(oracle_lib):
    """An async copy-back still in flight when the engine is closed or re-initialised."""
    ax = generators.workload("g2", scale=0.3)
    o = oracle_lib.saturate(ax, 0)
    ox, oa = o.facts()
    eng = engine.Engine(device=0)
    eng.load(ax)
    res = engine.Result()
    for _ in range(2):
        eng.init()
        eng.saturate()
        eng.copy_result(res, release=True, wait=False)
    eng.init()  # waits for the copy-back
    x, a = res.facts()
    assert np.array_equal(x, ox) and np.array_equal(a, oa)
    eng.saturate()
    eng.copy_result(res, release=True, wait=False)
    eng.close()  # drains it


def test_release_then_step_or_increment(oracle_lib):
    """A releasing copy-back enqueues the next classification's base links and propagations
    behind its reset.  A next state that is not a fresh saturation must not see them: per-rule
    stepping (el_step) after el_init, and an increment (el_add_axioms) after el_init, both reach
    the oracle's closure; a plain saturation after them is exact again."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_incremental import _split
    ax = generators.workload("g1", scale=0.2)
    o = oracle_lib.saturate(ax, 0)
    ox, oa = o.facts()
    res = engine.Result()
    eng = engine.Engine(device=0)
    eng.load(ax)
    eng.init()
    eng.saturate()
    eng.copy_result(res, release=True)
    eng.init()  # per-rule stepping on the state the release prepared
    for _ in range(200):
        if not any([eng.step(r) for r in range(8)]):
            break
    gx, ga = eng.facts()
    assert np.array_equal(gx, ox) and np.array_equal(ga, oa)
    for g, c in zip(eng.links(), o.links()):
        assert np.array_equal(g, c)
    eng.copy_result(res, release=True, wait=False)
    eng.init()
    eng.saturate()
    x, a = eng.facts()
    assert np.array_equal(x, ox) and np.array_equal(a, oa)
    eng.close()
    # an increment after el_init on a released state
    pieces = _split(ax, 2, 11, grow=False)
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(pieces[0])
    eng.init()
    eng.saturate()
    eng.copy_result(res, release=True)
    eng.init()
    eng.add_axioms(pieces[1])
    eng.saturate()
    o2 = oracle_lib.saturate(ax, 0, compat_range=True)
    gx, ga = eng.facts()
    ox2, oa2 = o2.facts()
    assert np.array_equal(gx, ox2) and np.array_equal(ga, oa2)
    for g, c in zip(eng.links(), o2.links()):
        assert np.array_equal(g, c)
    eng.close()


@pytest.mark.parametrize("release", [False, True])
def test_readout_block_summary(release, oracle_lib, monkeypatch):
    """S rows by the bit-matrix read-out over the block summary (forced for small results with
    EL_READOUT_MIN=0): KATs, a long-row ontology, G2, and an increment (the summary rebuilt
    from the re-laid-out matrix), each copy against the oracle; with release, twice in a row
    (the reset clears the summary with the matrix)."""
    monkeypatch.setenv("EL_READOUT_MIN", "0")
    cases = [kat.load_kat(p)[0] for p in kat.kat_files()[:6]]
    cases += [_long_rows_ontology(), generators.workload("g2", scale=0.5)]
    for ax in cases:
        o = oracle_lib.saturate(ax, 0)
        ptr, oa = _oracle_rows(o, ax.n_concepts)
        eng = engine.Engine(device=0)
        eng.load(ax)
        res = engine.Result()
        for _ in range(2 if release else 1):
            eng.init()
            eng.saturate()
            eng.copy_result(res, release=release)
            assert np.array_equal(res.s_ptr, ptr) and np.array_equal(res.s_val[:res.n_facts], oa)
        eng.close()
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_gpu_incremental import _split
    ax = generators.workload("g1", scale=0.3)
    pieces = _split(ax, 3, 5, grow=True)
    eng = engine.Engine(device=0, compat_range=True)
    eng.load(pieces[0])
    eng.init()
    eng.saturate()
    for inc in pieces[1:]:
        eng.add_axioms(inc)
        eng.saturate()
    res = eng.copy_result(release=release)
    o = oracle_lib.saturate(ax, 0, compat_range=True)
    ptr, oa = _oracle_rows(o, ax.n_concepts)
    assert np.array_equal(res.s_ptr, ptr) and np.array_equal(res.s_val[:res.n_facts], oa)
    eng.close()


# ---- streamed result (el_stream_result): the result node's writes in commit order, DMA'd while
# the supersteps run

def _stream_sets(eng, strm, n_user):
    """S facts sorted by (x, a) and links (x, r, y) sorted, from a streamed result."""
    x, a = strm.facts(n_user)
    role, filler = eng.pid_table()
    lx, lp = strm.link_rows()
    keep = lx < n_user
    lx, lr, ly = lx[keep], role[lp[keep]], filler[lp[keep]]
    o = np.lexsort((ly, lr, lx))
    return x, a, lx[o], lr[o], ly[o]


def _assert_stream_matches(eng, strm, o, n_user):
    x, a, lx, lr, ly = _stream_sets(eng, strm, n_user)
    ox, oa = o.facts()
    assert np.array_equal(x, ox) and np.array_equal(a, oa)
    for g, c in zip((lx, lr, ly), o.links()):
        assert np.array_equal(g, c)


@pytest.mark.parametrize("packed", [False, True], ids=["values", "packed"])
@pytest.mark.parametrize("path", kat.kat_files()[:12], ids=lambda p: os.path.basename(p))
def test_stream_result_kat(path, packed, oracle_lib):
    ax, _ = kat.load_kat(path)
    eng = engine.Engine(device=0)
    eng.load(ax)
    eng.init()
    strm = eng.stream_result(engine.Stream(packed=packed))
    st = eng.saturate()
    eng.result_wait()
    # every logged fact / link streamed once (the ELK range fillers' rows included)
    assert (strm.n_facts, strm.n_links) == (st["s_facts"], st["links"])
    _assert_stream_matches(eng, strm, oracle_lib.saturate(ax, 0), ax.n_concepts)
    eng.close()


@pytest.mark.parametrize("packed", [False, True], ids=["values", "packed"])
def test_stream_result_fuzz_release(packed, oracle_lib):
    """Random ontologies (told cycles included), streamed with release, one engine reused."""
    eng = engine.Engine(device=0)
    strm = engine.Stream(packed=packed)
    for seed in range(60):
        ax = generators.random_small(4400 + seed, n=8 + seed % 50, n_roles=1 + seed % 4)
        eng.load(ax)
        eng.init()
        eng.stream_result(strm, release=True)
        eng.saturate()
        eng.result_wait()
        _assert_stream_matches(eng, strm, oracle_lib.saturate(ax, 0), ax.n_concepts)
    eng.close()


def test_stream_result_small_buffers_erange():
    ax = generators.workload("g1", 0.05)
    eng = engine.Engine(device=0)
    eng.load(ax)
    eng.init()
    st = eng.saturate()
    eng.init()
    strm = engine.Stream()
    strm.fit(16, 16, 16, 16)
    eng._last = None
    for short in ("values", "runs"):
        eng.init()
        s = engine._ElStream()  # arm by hand with buffers far too small
        s.s_b = strm.s_b.ctypes.data_as(engine._u32p)
        s.s_cap = 16 if short == "values" else strm.s_b.size
        s.s_run = strm.s_run.ctypes.data_as(engine._u32p)
        s.s_run_cap = 16 if short == "runs" else strm.s_run.shape[0]
        s.l_p = strm.l_p.ctypes.data_as(engine._u32p)
        s.l_cap = 16 if short == "values" else strm.l_p.size
        s.l_run = strm.l_run.ctypes.data_as(engine._u32p)
        s.l_run_cap = 16 if short == "runs" else strm.l_run.shape[0]
        s.flags = engine.EL_RESULT_RELEASE  # (a short buffer keeps the state all the same)
        if short == "runs":  # values fit, only the runs are short
            strm.fit(st["s_facts"], st["links"], 16, 16)
            s.s_b, s.s_cap = strm.s_b.ctypes.data_as(engine._u32p), strm.s_b.size
            s.l_p, s.l_cap = strm.l_p.ctypes.data_as(engine._u32p), strm.l_p.size
        assert eng._lib.el_stream_result(eng._ctx, engine.C.byref(s)) == engine.EL_OK
        eng._lib.el_saturate(eng._ctx, None)
        assert s.n_facts == st["s_facts"] and s.n_links == st["links"]
        assert s.n_s_runs > 16 and s.n_l_runs > 16
        assert eng._lib.el_result_wait(eng._ctx) == engine.EL_ERANGE
        # the state was kept: streamed again at the fixpoint into buffers of the counts
        strm.n_facts, strm.n_links, strm.n_s_runs, strm.n_l_runs = s.n_facts, s.n_links, s.n_s_runs, s.n_l_runs
        eng.stream_result(strm, release=True, n_facts=s.n_facts, n_links=s.n_links)
        st2 = eng.saturate()
        eng.result_wait()
        assert st2["supersteps"] == 0 or st2["derived"] == st["derived"]
        assert (strm.n_facts, strm.n_links) == (st["s_facts"], st["links"])
    # pageable run buffers are refused (the device writes them)
    eng.init()
    s = engine._ElStream()
    pageable = np.zeros(64, np.uint32)
    s.s_run, s.s_run_cap = pageable.ctypes.data_as(engine._u32p), 32
    assert eng._lib.el_stream_result(eng._ctx, engine.C.byref(s)) == engine.EL_EINVAL
    eng.close()


def test_stream_packed_short_escapes_erange(oracle_lib):
    """EL_STREAM_PACKED with an escape buffer far too short: EL_ERANGE with the state kept and
    the escape count reported; re-armed with it, the fixpoint streams the whole log again.
    (78,002 concepts: more than the 65,535 coded columns, so some facts escape.)"""
    ax = generators.workload("g3", 0.2)
    eng = engine.Engine(device=0)
    eng.load(ax)
    eng.init()
    st = eng.saturate()
    eng.init()
    strm = engine.Stream(packed=True)
    strm.fit(st["s_facts"], st["links"], st["s_facts"], st["links"], 16)
    s = engine._ElStream()
    s.flags = engine.EL_RESULT_RELEASE | engine.EL_STREAM_PACKED
    s.s_code = strm.s_code.ctypes.data_as(engine.C.POINTER(engine.C.c_uint16))
    s.s_cap = strm.s_code.size
    s.s_esc, s.s_esc_cap = strm.s_esc.ctypes.data_as(engine._u32p), 4
    s.s_run, s.s_run_cap = strm.s_run.ctypes.data_as(engine._u32p), strm.s_run.shape[0]
    s.l_p, s.l_cap = strm.l_p.ctypes.data_as(engine._u32p), strm.l_p.size
    s.l_run, s.l_run_cap = strm.l_run.ctypes.data_as(engine._u32p), strm.l_run.shape[0]
    assert eng._lib.el_stream_result(eng._ctx, engine.C.byref(s)) == engine.EL_OK
    eng._lib.el_saturate(eng._ctx, None)
    assert s.n_s_esc > 4
    assert eng._lib.el_result_wait(eng._ctx) == engine.EL_ERANGE
    strm.n_facts, strm.n_links, strm.n_s_runs, strm.n_l_runs = s.n_facts, s.n_links, s.n_s_runs, s.n_l_runs
    strm.n_s_esc = s.n_s_esc
    eng.stream_result(strm, release=True, n_facts=s.n_facts, n_links=s.n_links)
    eng.saturate()
    eng.result_wait()
    _assert_stream_matches(eng, strm, oracle_lib.saturate(ax, 0), ax.n_concepts)
    eng.close()


def _set_digest(name, scale):
    """Pinned order-independent closure digest (tests/golden/set_digests.txt: the oracle's closure,
    cross-checked against its SHA-256 pin by make_set_digests.py)."""
    for line in open(os.path.join(os.path.dirname(__file__), "golden", "set_digests.txt")):
        f = line.split()
        if len(f) == 4 and f[0] == name and float(f[1]) == scale:
            return f[3]
    raise AssertionError(f"no pinned set digest for {name} {scale}")


@pytest.mark.parametrize("packed", [False, True], ids=["values", "packed"])
def test_stream_result_g3_digest_two_engines(packed):
    """The bench's schedule at full G3 with the streamed copy-back: one engine serial, then two
    alternating (one's DMA tail beside the other's classification); every result hashes to the
    pinned closure digest.  The digest is order-independent (a sum of per-entry hashes,
    distel_amd.result.set_digest), so the commit-order stream is decoded and hashed without a
    sort of its 137 M entries."""
    want = _set_digest("g3", 1.0)
    ax = generators.workload("g3")
    engs = [engine.Engine(device=0) for _ in range(2)]
    for e in engs:
        e.load(ax)
    strms = [engine.Stream(packed=packed), engine.Stream(packed=packed)]
    role, filler = engs[0].pid_table()

    def digest(e, s):
        return s.digest(role, filler, ax.n_concepts)

    for i in range(4):
        e, s = engs[i % 2] if i >= 2 else engs[0], strms[i % 2] if i >= 2 else strms[0]
        e.init()
        e.stream_result(s, release=True)
        e.saturate()
        if i < 2:
            e.result_wait()
            assert digest(e, s) == want
        elif i == 3:
            engs[0].result_wait()  # (landed behind engine 1's classification)
            assert digest(engs[0], strms[0]) == want
            engs[1].result_wait()
            assert digest(engs[1], strms[1]) == want
    for e in engs:
        e.close()
