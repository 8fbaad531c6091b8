#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tape
timeout -k 10 200 python -u tools/r5/tape_dump.py > gpurun_out/tape/1f1b.txt 2>&1
