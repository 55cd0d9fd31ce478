"""GPU parity under the host concurrency the bench (and a multi-client deployment) uses: several
handles driven at once from host threads, every result checked against the CPU oracle.

- Six LocalBundleAdjustment handles on six threads (bench.py's LBA leg: one solver per LocalMapping
  client), each handle's window count growing between its calls (4 -> 8 -> 24 -> 6 windows: the
  handle's planning pool gains workers between calls, and its buffers grow) for several rounds.
  Every window must give the oracle's iteration / trial counts and outlier set, and poses / points
  within 1e-5 (BASELINE.json north_star), exactly as a lone solve does (tests/test_gpu_lba.py).
- Two ORBmatcher handles running SearchByProjection batches at once from two threads, each batch
  large enough for the threaded pinned staging (matcher.hip staged_upload), bit-exact vs the oracle.
"""
import threading

import numpy as np
import pytest

import oracle_bind as ob
import scenes
from slamhot import synth

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _same(g, o):
    assert g["iterations"] == o["iterations"], (g["iterations"], o["iterations"])
    assert g["trials"] == o["trials"]
    np.testing.assert_allclose(g["chi2_final"], o["chi2_final"], rtol=1e-8)
    assert np.array_equal(g["edge_outlier"], o["edge_outlier"])
    assert np.abs(g["kf_Tcw"].astype(np.float64) - o["kf_Tcw"]).max() <= TOL
    assert np.abs(g["pt_pos"].astype(np.float64) - o["pt_pos"]).max() <= TOL


def _run_threads(fns, timeout=100):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append(e)
    ths = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
        assert not t.is_alive(), "a handle's thread did not finish"
    if errs:
        raise errs[0]


def test_six_lba_handles_concurrent_growing_batches():
    import slamhot
    # 12 distinct windows (mono, stereo, a fixed-KF-heavy one), oracle once per window
    pool = [synth.lba_window(s) for s in range(300, 308)] + [synth.lba_window(s, stereo_frac=0.3)
                                                              for s in range(308, 312)]
    want = [ob.lba_solve(w) for w in pool]
    counts = [4, 8, 24, 6]
    nh = 6
    handles = [slamhot.LocalBundleAdjustment() for _ in range(nh)]
    got = [[] for _ in range(nh)]

    def worker(h):
        def f():
            for rnd in range(2):
                for c in counts:
                    idx = [(h * 5 + rnd * 7 + k) % len(pool) for k in range(c)]
                    res = handles[h].solve([pool[i] for i in idx])
                    got[h].append((idx, res))
        return f
    try:
        _run_threads([worker(h) for h in range(nh)])
    finally:
        for s in handles:
            s.close()
    n = 0
    for h in range(nh):
        assert len(got[h]) == 2 * len(counts)
        for idx, res in got[h]:
            for i, r in zip(idx, res):
                _same(r, want[i])
                n += 1
    assert n == nh * 2 * sum(counts)


def test_six_lba_prepared_runs_concurrent():
    """bench.py's exact driving pattern: prepare() once per handle, then run() repeatedly from six
    threads at once (the C call only); the last run's results equal the oracle."""
    import slamhot
    pool = [synth.lba_window(s) for s in range(320, 326)]
    want = [ob.lba_solve(w) for w in pool]
    nh = 6
    handles = [slamhot.LocalBundleAdjustment() for _ in range(nh)]
    wins = [[pool[(h + k) % len(pool)] for k in range(16)] for h in range(nh)]
    runs = [handles[h].prepare(wins[h]) for h in range(nh)]
    iters = [[] for _ in range(nh)]

    def worker(h):
        def f():
            for _ in range(4):
                iters[h].append(runs[h]())
        return f
    try:
        _run_threads([worker(h) for h in range(nh)])
        for h in range(nh):
            assert len(set(iters[h])) == 1, iters[h]  # the same windows give the same LM iteration total
            for k, r in enumerate(runs[h].results()):
                _same(r, want[(h + k) % len(pool)])
    finally:
        for s in handles:
            s.close()


@pytest.mark.parametrize("kind", ["last", "local"])
def test_two_matcher_batches_concurrent(kind):
    import slamhot
    nfr = 32
    sets = []
    for b in range(2):
        views, others, descs = [], [], []
        for i in range(nfr):
            S = scenes.scene(500 + 100 * b + i)
            fv, keep = scenes.frame_view(S)
            views.append(fv)
            if kind == "last":
                lf, lkeep = scenes.last_frame(S, mono=False, motion=(0.02, 0.2)[i % 2])
                others.append((lf, lkeep, keep))
            else:
                geom, desc = scenes.local_map_geom(S, n_extra=300)
                others.append((geom, keep))
                descs.append(desc)
        sets.append((views, others, descs))
    ms = [slamhot.ORBmatcher(0.9, True) if kind == "last" else slamhot.ORBmatcher(0.8) for _ in range(2)]
    outs = [[None] * 3 for _ in range(2)]

    def worker(b):
        def f():
            views, others, descs = sets[b]
            for r in range(3):
                if kind == "last":
                    outs[b][r] = ms[b].SearchByProjection_last_batch(views, [o[0] for o in others], 7.0, False)
                else:
                    outs[b][r] = ms[b].SearchLocalPoints_batch(views, [o[0] for o in others], descs, 1.0, False, 20.0)
        return f
    try:
        _run_threads([worker(0), worker(1)])
    finally:
        for m in ms:
            m.close()
    for b in range(2):
        views, others, descs = sets[b]
        for i in range(nfr):
            if kind == "last":
                no, fo = ob.search_by_projection_last(views[i], others[i][0], 0.9, True, 7.0, False)
                for r in range(3):
                    nm, fm = outs[b][r][i]
                    assert nm == no and np.array_equal(fm, fo), (b, r, i)
            else:
                nto, tro = ob.is_in_frustum(views[i], others[i][0], 0.5)
                no, fo = ob.search_by_projection_local(views[i], tro, descs[i], 0.8, 1.0, False, 20.0)
                for r in range(3):
                    nm, fm, nt = outs[b][r][i]
                    assert nt == nto and nm == no and np.array_equal(fm, fo), (b, r, i)
