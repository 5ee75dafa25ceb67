#!/bin/bash
# BASELINE cfg 4 (hard 22x22) and cfg 5 (FOMAML) tiers
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py --fomaml --steps 2 --warmup 1 2>&1 | tee gpurun_out/bench_fomaml.log || exit $?
timeout -k 10 600 python bench.py --difficulty hard --size 22 --steps 1 --warmup 1 --no-cpu-baseline 2>&1 | tee gpurun_out/bench_hard22.log
