set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stereo_ops.py tests/test_gpu_cpp_api.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r05m_tests.log 2>&1; rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r05m_tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/r05m_tests.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-configs --no-cpu-baseline > gpurun_out/r05m_bench.log 2>&1; echo "bench rc=$?"
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05m_bench.log') if l.startswith('{')][-1])
print(json.dumps(d['next_rows']))"
