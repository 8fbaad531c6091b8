#!/bin/bash
# Reference model L8H8 (batch 32 x 128, m = 4, lanes): in_proj bias grads as colsum jobs
# (kept) vs fused into the attention backward kernels (dbias=) -- run against a build where
# models/native.py._mha_bwd passes dbias=gb when MIPIPE_AB_DBIAS=1.  Recorded result (one
# MI355X, 2 interleaved runs each): fused 573.6K / 579.3K tok/s, colsum jobs 609.0K / 610.1K.
for rep in 1 2; do for v in 1 0; do echo "DBIAS=$v"; MIPIPE_AB_DBIAS=$v timeout -k 10 200 python bench.py --model reference --mbs 8 --seq 128 --microbatches 4 --steps 20 --warmup 5 --no-bubble 2>/dev/null | tail -1; done; done
