#!/bin/bash
# dW split-K cap A/B (MIPIPE_DW_MAXSPLIT) on the GPT-2 small bench (lanes on): fewer
# splits = less f32 slab + reduce traffic, fewer workgroups per dW GEMM
set -o pipefail
for rep in 1 2; do for c in 32 8 4; do
  echo "MAXSPLIT=$c $(MIPIPE_DW_MAXSPLIT=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-bubble 2>/dev/null | tail -1 | cut -c80-125)"
done; done
