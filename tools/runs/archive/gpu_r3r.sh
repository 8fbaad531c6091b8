#!/bin/bash
# gemm3 balanced-read schedule (A/B build _C_g3b.so, -D MP_G3_SCHED=2) vs default:
# GEMM numerics on the variant, GEMM microbench (interleaved), bench.py (interleaved).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MIPIPE_EXT_VARIANT=g3b timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or linear" --timeout 120 --timeout-method thread > gpurun_out/g3b_test.log 2>&1
rc=$?; tail -2 gpurun_out/g3b_test.log; [ $rc -ne 0 ] && exit $rc
for v in "" g3b "" g3b; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 200 python -u tools/bench_kernels.py --only _ > gpurun_out/g3b_bk_${v:-def}.log 2>&1 || exit 1
  echo "== ${v:-default}"; grep -E "^(fwd|dx|dw)_" gpurun_out/g3b_bk_${v:-def}.log | python3 -c "
import sys,ast
for l in sys.stdin:
    k,d=l.split(' ',1); d=ast.literal_eval(d.strip()); print(k, d['ours_tflops'], d['lib_tflops'])"
done > gpurun_out/g3b_bk_ab.txt
: > gpurun_out/g3b_bench_ab.txt
for v in "" g3b "" g3b; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/g3b_bench_${v:-def}.log 2>&1 || exit 1
  echo "${v:-default} $(tail -1 gpurun_out/g3b_bench_${v:-def}.log | cut -c150-260)" >> gpurun_out/g3b_bench_ab.txt
done
cat gpurun_out/g3b_bench_ab.txt
