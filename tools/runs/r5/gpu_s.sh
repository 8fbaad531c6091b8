#!/bin/bash
# Split-K XCD remap: numerics, dW probe A/B (interleaved), headline bench A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5s2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm" > gpurun_out/r5s2/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5s2/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/gemm_dw_probe.py > gpurun_out/r5s2/dw_on_$i.txt 2>&1 || exit 1
  MIPIPE_G3_SPLIT_REMAP=0 timeout -k 10 120 python tools/gemm_dw_probe.py > gpurun_out/r5s2/dw_off_$i.txt 2>&1 || exit 1
done
grep -v "^{\|amdgpu" gpurun_out/r5s2/dw_on_2.txt gpurun_out/r5s2/dw_off_2.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --schedules none --ref-fp32 0 > gpurun_out/r5s2/bench_on_$i.log 2>&1 || exit 1
  MIPIPE_G3_SPLIT_REMAP=0 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --schedules none --ref-fp32 0 > gpurun_out/r5s2/bench_off_$i.log 2>&1 || exit 1
done
for f in gpurun_out/r5s2/bench_*.log; do echo "$f $(grep '^{' $f | cut -c150-185)"; done
