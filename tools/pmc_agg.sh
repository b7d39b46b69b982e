#!/bin/bash
# GPU box: HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes) of the fused aggregation
# launches (k_agg_split) over a short bench of single-pair groups -> gpurun_out/agg_pmc.json
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
RX=k_agg_split
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ops --batch 2 --concurrency 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_agg_fetch -o run -- $B > gpurun_out/pmc_agg_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_agg_fetch.log; exit $rc; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_agg_write -o run -- $B > gpurun_out/pmc_agg_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_agg_write.log; exit $rc; }
python3 - <<'PY'
import collections, csv, json
def per(path, c):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == c:
            d[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(d.values())
f = per("gpurun_out/pmc_agg_fetch/run_counter_collection.csv", "FETCH_SIZE")
w = per("gpurun_out/pmc_agg_write/run_counter_collection.csv", "WRITE_SIZE")
fb = 2 * sum(f) / len(f) * 1024
wb = sum(w) / len(w) * 1024
alg = 2 * (2 * 193 * 1242 * 375 * 4)
out = {"kernel": "k_agg_split<true,49,false> (config B, one pair, fused pass pair: one read + one write of the two-view volume)",
       "dispatches": [len(f), len(w)], "fetch_bytes_corrected": fb, "write_bytes": wb,
       "hbm_bytes_per_launch": fb + wb, "algorithmic_bytes_per_launch": alg, "ratio": (fb + wb) / alg,
       "note": "FETCH_SIZE doubled (gfx950: 64 B tallied per 128-B request), separate passes"}
json.dump(out, open("gpurun_out/agg_pmc.json", "w"), indent=1)
print(json.dumps(out))
PY
