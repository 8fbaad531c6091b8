set -o pipefail
cd "$GRAFT_REPO_ROOT"
run2() {
  timeout -k 10 200 python -u bench.py "$@" --steps 30 --warmup 5 --no-bubble > gpurun_out/c1.log 2>&1 &
  p1=$!
  timeout -k 10 200 python -u bench.py "$@" --steps 30 --warmup 5 --no-bubble > gpurun_out/c2.log 2>&1 &
  p2=$!
  wait $p1; r1=$?; wait $p2; r2=$?
  echo "pair rc $r1 $r2: $(grep -o '"value": [0-9.]*' gpurun_out/c1.log) $(grep -o '"value": [0-9.]*' gpurun_out/c2.log)"
  [ $r1 -eq 0 ] && [ $r2 -eq 0 ]
}
timeout -k 10 200 python -u bench.py --model reference --mbs 8 --seq 128 --microbatches 4 --steps 30 --warmup 5 --no-bubble > gpurun_out/c0.log 2>&1 && echo "ref single $(grep -o '"value": [0-9.]*' gpurun_out/c0.log)" && \
run2 --model reference --mbs 8 --seq 128 --microbatches 4 && \
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-bubble > gpurun_out/c0.log 2>&1 && echo "gpt2 single $(grep -o '"value": [0-9.]*' gpurun_out/c0.log)" && \
run2
