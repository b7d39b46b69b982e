#!/usr/bin/env python3
"""Golden hashes for SURVEY §8 configs C and E at full size (test infrastructure).

Runs the oracle (oracle/, the C restatement of source/ADCensus.cpp) on the synthetic
config C pair (1500x1000, setMinMaxDisparity(0, 256)) and config E pair (2048x1536 grey
replicated to BGR, setMinMaxDisparity(0, 320)), serial scanline semantics, RGB model,
and records the SHA-256 of the fp32 disparity bytes plus a few statistics in
tests/golden/config_hashes.json.  The GPU test compares its own output's hash: a
bit-exact check at sizes whose oracle run takes minutes (too long for the GPU suite).

    python tests/golden/make_config_hashes.py [--threads N]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import tea_stereo_matching_amd.synthetic as syn  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    out = {}
    for name, gen, D in (("C", syn.config_c, 256), ("E", syn.config_e, 320)):
        left, right, _ = gen()
        t0 = time.time()
        d, _ = O.compute(left, right, O.default_params(O.RGB, 0, D, num_threads=args.threads))
        d = np.ascontiguousarray(d, dtype=np.float32)
        out[name] = {
            "shape": list(d.shape), "max_disparity": D,
            "sha256": hashlib.sha256(d.tobytes()).hexdigest(),
            "valid_fraction": float((d >= 0).mean()),
            "sum_valid": float(d[d >= 0].astype(np.float64).sum()),
            "oracle_seconds": round(time.time() - t0, 1), "oracle_threads": args.threads,
        }
        print(name, out[name], flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "config_hashes.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
