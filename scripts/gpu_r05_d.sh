#!/bin/bash
# round 5 (d): the driver-settings bench line (all tiers, CPU baseline), then the kernel trace + PMC passes of the
# same command over the timed iterations (scripts/gpu_prof_r05.sh), summaries under gpurun_out/summary/
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG:-r05c}_bench_driver.log 2>&1 || exit $?
tail -c 300 gpurun_out/${TAG:-r05c}_bench_driver.log
PMC=1 TAG=${TAG:-r05c} bash scripts/gpu_prof_r05.sh
