#!/usr/bin/env python3
"""North-star parity figure (BASELINE.json: "within +-0.5 px on >= 99 % of valid pixels"),
measured on the CPU with the oracle.

The product's default scanline semantics are serial (the reference's intended algorithm);
the reference's shipped binaries ran a racy OpenMP schedule whose outcome the oracle
reproduces exactly at T = 20 (tests/test_oracle_fixtures.py: both demo PNGs pixel for
pixel).  Since the GPU path is bit-exact with the oracle in both modes (tests/), the
figure compares oracle-serial (= the GPU default) against oracle-T20 (= the reference's own
output) on the reference's two demo pairs and on config B's first pair.

    python tools/parity_figure.py [--threads N] > profiles/r03_parity_figure.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import load_bgr  # noqa: E402
from oracle import oracle as O  # noqa: E402
import tea_stereo_matching_amd.synthetic as syn  # noqa: E402


def figure(left, right, D, threads):
    serial, _ = O.compute(left, right, O.default_params(O.RGB, 0, D, num_threads=threads))
    ref, _ = O.compute(left, right, O.default_params(O.RGB, 0, D, num_threads=threads, scan_emulate_threads=20))
    valid = ref >= 0
    both = valid & (serial >= 0)
    close = np.abs(serial - ref) <= 0.5
    return {
        "valid_pixels_ref": int(valid.sum()),
        "frac_within_0.5px_of_valid_ref": round(float((close & valid).sum() / valid.sum()), 5),
        "frac_within_0.5px_where_both_valid": round(float((close & both).sum() / both.sum()), 5),
        "frac_identical_all_pixels": round(float((serial == ref).mean()), 5),
        "frac_validity_agrees": round(float(((serial >= 0) == valid).mean()), 5),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    d = os.path.join(ROOT, "tests", "golden", "demo")
    out = {"what": "oracle serial semantics (the GPU default) vs oracle with the T=20 race emulation "
                   "(reproduces the reference's demo outputs exactly), RGB, D=[0,192]"}
    for name in ("0600", "0045"):
        l, r = load_bgr(os.path.join(d, f"{name}-Left.png")), load_bgr(os.path.join(d, f"{name}-Right.png"))
        out[name] = figure(l, r, 192, args.threads)
        print(name, out[name], file=sys.stderr, flush=True)
    l, r, _ = syn.config_b(1000)
    out["config_b_seed1000"] = figure(l, r, 192, args.threads)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
