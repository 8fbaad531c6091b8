#!/bin/bash
# GPT-2 small, global batch 32 x 1024 on one GPU: microbatch size x lanes
set -o pipefail
for rep in 1 2; do
  echo "mbs16 m2 lanes2 $(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-bubble 2>/dev/null | tail -1 | cut -c80-125)"
  echo "mbs8 m4 lanes2 $(MIPIPE_LANES=2 timeout -k 10 200 python bench.py --mbs 8 --microbatches 4 --steps 20 --warmup 5 --no-bubble 2>/dev/null | tail -1 | cut -c80-125)"
  echo "mbs8 m4 lanes4 $(MIPIPE_LANES=4 timeout -k 10 200 python bench.py --mbs 8 --microbatches 4 --steps 20 --warmup 5 --no-bubble 2>/dev/null | tail -1 | cut -c80-125)"
done
