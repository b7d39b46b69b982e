#!/usr/bin/env python3
"""Single-frame latency on the GPU box: one config-B pair at a time through (a) the
device-resident call, (b) the host call (ADCensus.compute), with the stage split."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tea_stereo_matching_amd as T  # noqa: E402

H, W, D = 375, 1242, 192
l, r, _ = T.synthetic.make_scene(1000, H, W, D + 1)
dev = torch.device("cuda", 0)
dl, dr = torch.from_numpy(l).to(dev), torch.from_numpy(r).to(dev)
out = torch.empty((H, W), dtype=torch.float32, device=dev)
m = T.ADCensus(0)
m.setMatchingStrategy(T.ColorModel.RGB, False, False)
m.setMinMaxDisparity(0, D)
m.setConcurrency(int(sys.argv[1]) if len(sys.argv) > 1 else 1)


def dev_call():
    m.compute_device_ptr(dl.data_ptr(), dr.data_ptr(), H, W, W * 3, out.data_ptr(), W * 4)
    m.synchronize()


for name, fn in (("device", dev_call), ("host", lambda: m.compute(l, r))):
    for _ in range(3):
        fn()
    t0 = time.perf_counter()
    for _ in range(20):
        fn()
    print(f"{name}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/frame")
m.setProfiling(True)
m.resetStageTimes()
for _ in range(10):
    dev_call()
m.setProfiling(False)
st = m.stageTimes()
print({k: round(v[0] / max(1, v[1]), 4) for k, v in st.items()}, "sum", round(sum(v[0] / max(1, v[1]) for v in st.values()), 3))
m.close()
