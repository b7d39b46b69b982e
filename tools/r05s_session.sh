set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/remap_probe.py 4 8 || exit 1
export TSM_REMAP_MI=4
TAG=rmb4 bash tools/pmc_kernel.sh k_remap_fixed_buf tools/remap_probe.py 4 || exit 1
i=10
for set in "FETCH_SIZE" "WRITE_SIZE" "TA_TA_BUSY_sum TD_TD_BUSY_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex k_remap_fixed_buf --output-format csv -d gpurun_out/pk_rmb4_$i -o run -- python3 tools/remap_probe.py 4 > gpurun_out/pk_rmb4_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pk_rmb4_$i.log; exit $rc; }
done
python3 tools/pmc_sum.py gpurun_out/pk_rmb4_*/run_counter_collection.csv
