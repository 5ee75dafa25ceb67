#!/bin/bash
# driver-settings bench (all tiers) then the rocprofv3 trace + PMC passes of scripts/gpu_prof_r03.sh
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_driver.log
TAG=${TAG:-r03b} PMC=1 bash scripts/gpu_prof_r03.sh
