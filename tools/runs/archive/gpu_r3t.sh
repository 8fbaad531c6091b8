#!/bin/bash
# bench.py N=1 (m = 4): microbatch lanes 2 (auto) vs 4, interleaved; f32-linear GPU tests.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_reference_parity.py tests/test_kernels_gpu.py -x -q -m gpu -k "f32" --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1
rc=$?; tail -2 gpurun_out/f32_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/lanes_m4_ab.txt
for l in 2 4 2 4; do
  MIPIPE_LANES=$l timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/lanes_m4_$l.log 2>&1 || exit 1
  echo "lanes=$l $(tail -1 gpurun_out/lanes_m4_$l.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["microbatch_lanes"], d["hbm_peak_gb_per_gpu"])')" >> gpurun_out/lanes_m4_ab.txt
done
cat gpurun_out/lanes_m4_ab.txt
