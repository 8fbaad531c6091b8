# selective recompute: GPU tests + Llama-3 8B one-GPU A/B (GPipe m = 4 does not fit without recompute)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_native_runner_gpu.py -x -q --timeout 200 --timeout-method thread -k "selective" > gpurun_out/r6_selective_tests.log 2>&1 || exit 1
for rc in 1 auto; do
  timeout -k 10 400 python -u tools/llama8b_step.py --schedule GPipe --m 4 --steps 3 --recompute $rc > gpurun_out/r6_llama_rc_$rc.log 2>&1 || exit 1
done
