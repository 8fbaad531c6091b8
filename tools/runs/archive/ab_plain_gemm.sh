#!/bin/bash
# Plain-GEMM backend A/B on one MI355X: MIPIPE_GEMM=hip (our engines for every GEMM) vs
# auto (per-shape timed choice between our engine and hipBLASLt for plain fwd / dX GEMMs).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_plain_gemm.log
: > $out
for rep in 1 2; do
  for pol in hip auto; do
    echo "== MIPIPE_GEMM=$pol gpt2-small rep $rep" >> $out
    MIPIPE_GEMM=$pol timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-bubble 2>/dev/null | tail -1 >> $out || exit 1
  done
done
for pol in hip auto; do
  echo "== MIPIPE_GEMM=$pol reference L8H8" >> $out
  MIPIPE_GEMM=$pol timeout -k 10 200 python bench.py --model reference --mbs 8 --seq 128 --microbatches 4 --steps 20 --warmup 5 --no-bubble 2>/dev/null | tail -1 >> $out || exit 1
done
