#!/bin/bash
# GPU box: two bench ranks on the one GPU over gloo (RCCL refuses two ranks on one device):
# the multi-rank bookkeeping (barriers, max-over-ranks timing, per-rank verification), first
# without the gather, then with it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 --concurrency 16 --no-cpu-baseline --no-ops"
TSM_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 $A --no-gather > gpurun_out/reh_nogather.log 2>&1
rc=$?; echo "no-gather rc=$rc"; grep '^{' gpurun_out/reh_nogather.log | cut -c1-300; [ $rc -ne 0 ] && { tail -20 gpurun_out/reh_nogather.log; exit $rc; }
TSM_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 $A > gpurun_out/reh_gather.log 2>&1
rc=$?; echo "gather rc=$rc"; grep '^{' gpurun_out/reh_gather.log | cut -c1-300; [ $rc -ne 0 ] && tail -20 gpurun_out/reh_gather.log; exit $rc
