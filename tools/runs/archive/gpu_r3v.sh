#!/bin/bash
# f32 GEMM: XCD-aware column-major raster (A/B build _C_f32r.so, -D MP_F32_RASTER=1) vs
# default: f32 GEMM tests on the variant, split-K sweep (interleaved), fp32 L8H8 trainer.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MIPIPE_EXT_VARIANT=f32r timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_reference_parity.py tests/test_native_gpu.py -x -q -m gpu -k "f32" --timeout 120 --timeout-method thread > gpurun_out/f32r_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f32r_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "" f32r "" f32r; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 200 python -u tools/f32_gemm_sweep.py --json gpurun_out/f32r_sweep_${v:-def}.json > gpurun_out/f32r_sweep_${v:-def}.log 2>&1 || exit 1
  cp gpurun_out/f32r_sweep_${v:-def}.json gpurun_out/f32r_sweep_${v:-def}_$RANDOM.json
done
: > gpurun_out/f32r_trainer_ab.txt
for v in "" f32r "" f32r; do
  MIPIPE_EXT_VARIANT=$v timeout -k 10 200 python -u tools/ref_table_gpu.py --engine trainer --fwd-bwd --precision fp32 --only 8x8,4x12 > gpurun_out/f32r_tr_${v:-def}.log 2>&1 || exit 1
  echo "${v:-default} $(grep tokens_per_s gpurun_out/f32r_tr_${v:-def}.log | cut -c1-100 | tr '\n' ' ')" >> gpurun_out/f32r_trainer_ab.txt
done
cat gpurun_out/f32r_trainer_ab.txt
