"""TSM_TRACE=1 runs the descriptor-checked aggregation streamer (k_agg_split<..., CHK>):
every meta-ring descriptor a wave consumes is range-checked, and a protocol slip sets a
device flag that the per-launch trace reports ("PROTOCOL CHECK FAILED") instead of
addressing outside the arena.  A clean run reports nothing and computes the same maps as
the unchecked product path, for one label slice, two label slices and a group of pairs."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import tea_stereo_matching_amd as tsm
out = []
for (H, W, D, n) in ((96, 160, 48, 1), (64, 200, 299, 1), (48, 120, 32, 3)):
    m = tsm.ADCensus(0)
    m.setMatchingStrategy(tsm.ColorModel.RGB, False, False)
    m.setMinMaxDisparity(0, D)
    pairs = [tsm.synthetic.make_scene(500 + i, H, W, D + 1)[:2] for i in range(n)]
    if n == 1:
        out.append(m.compute(*pairs[0]))
    else:
        m.setConcurrency(n)
        out.extend(m.compute_batch([p[0] for p in pairs], [p[1] for p in pairs]))
    m.close()
np.save(sys.argv[2], np.concatenate([o.ravel() for o in out]))
"""


def _run(tmp_path, trace):
    env = dict(os.environ)
    env.pop("TSM_TRACE", None)
    if trace:
        env["TSM_TRACE"] = "1"
    out = str(tmp_path / f"out_{int(trace)}.npy")
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT, out], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    return np.load(out), r.stderr


def test_trace_checked_streamer_clean_and_identical(tmp_path):
    plain, _ = _run(tmp_path, False)
    traced, log = _run(tmp_path, True)
    assert "k_agg_split" in log  # the checked streamer ran, once per launch
    assert "PROTOCOL CHECK FAILED" not in log, [l for l in log.splitlines() if "FAILED" in l][:5]
    assert "sync=no error" in log and "launch=no error" in log
    assert np.array_equal(plain, traced)
