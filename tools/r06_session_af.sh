#!/bin/bash
# round-6 session af: address-translation counters of the aggregation streamer over 6 fresh
# handles (their speeds differ by handle, deterministically per process)
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/xcc_probe.py --handles 6 2>&1 | grep -v "WARNING\|amdgpu.ids" | tee gpurun_out/r06af_speed.txt || exit 1
timeout -s KILL 400 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum --kernel-include-regex "k_agg_split|k_scan_line" --output-format csv -d gpurun_out/af_pmc -o run -- python3 tools/xcc_probe.py --handles 6 --batches 1 > gpurun_out/af_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -8 gpurun_out/af_pmc.log
