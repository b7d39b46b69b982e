"""Handles on several host threads at once (include/tsm_adcensus.h: one handle per thread;
handles run concurrently).  Two threads, each with its own handle on the same device,
compute different pairs in different modes at the same time -- the first launches of
every kernel variant in the process included, where the per-(kernel, device) LDS-limit
setup runs (engine.cpp ensure_lds_limit) -- and every disparity must equal the bits the
same handle settings give on one thread.  ctypes releases the GIL around library calls,
so the two threads' pipelines really do overlap on the host and on the GPU.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (seed, H, W, labels, model, omp threads): RGB and HSI, short and long label axes
# (split streamer with label slices, 8-vector scanline), the emulated race
CASES = [
    (7001, 120, 331, 65, 0, 0),
    (7002, 96, 250, 300, 0, 0),
    (7003, 120, 331, 65, 1, 0),
    (7004, 80, 400, 193, 0, 5),
    (7005, 64, 900, 449, 1, 0),
    (7006, 130, 300, 129, 0, 0),
]


def _run(tsm, case, pair):
    seed, H, W, L, model, omp = case
    m = tsm.ADCensus(0)
    try:
        m.setMatchingStrategy(tsm.ColorModel(model))
        m.setMinMaxDisparity(0, L - 1)
        if omp:
            m.setOmpEmulation(omp)
        return m.compute(pair[0], pair[1])
    finally:
        m.close()


def test_two_handles_on_two_threads():
    import tea_stereo_matching_amd as tsm

    if tsm.device_count() == 0:
        pytest.fail("no HIP device visible to a -m gpu test")
    pairs = [tsm.synthetic.make_scene(s, H, W, L)[:2] for (s, H, W, L, _, _) in CASES]

    # both threads start together (a barrier), each walks the cases in a different order
    got = [[None] * len(CASES) for _ in range(2)]
    errors = []
    start = threading.Barrier(2)

    def worker(t):
        try:
            order = list(range(len(CASES)))
            if t == 1:
                order.reverse()
            start.wait()
            for rep in range(2):
                for i in order:
                    out = _run(tsm, CASES[i], pairs[i])
                    if got[t][i] is None:
                        got[t][i] = out
                    elif not np.array_equal(got[t][i], out):
                        errors.append(f"thread {t} case {i}: repeat differs")
        except Exception as e:  # surfaced below, with the thread's name
            errors.append(f"thread {t}: {e!r}")

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts), "a worker thread did not finish"
    assert not errors, errors

    # the same settings on one thread, after the concurrent phase
    for i, case in enumerate(CASES):
        want = _run(tsm, case, pairs[i])
        for t in range(2):
            assert np.array_equal(got[t][i], want), (t, case)

    # and the first case against the oracle (RGB, serial scanline)
    from conftest import host_threads
    from oracle import oracle as O
    seed, H, W, L, model, omp = CASES[0]
    ref, _ = O.compute(pairs[0][0], pairs[0][1], O.default_params(O.RGB, 0, L - 1, num_threads=host_threads()))
    assert np.array_equal(got[0][0], ref)
