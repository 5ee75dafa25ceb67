#!/bin/bash
# round 6 (final, part 2): the driver-settings bench under rocprofv3 (kernel trace + FETCH_SIZE / WRITE_SIZE passes,
# step sequence, busy union), then the driver-settings line with every tier and the CPU baseline
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
TAG=r06zf PMC=1 bash scripts/gpu_profile_bench.sh > gpurun_out/r06zf_prof.log 2>&1; rc=$?
tail -2 gpurun_out/r06zf_prof.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06zf_bench_driver.log 2>&1; rc=$?
grep -o '"value": [0-9.]*\|"phases_ms": {[^}]*}\|"fomaml": {[^}]*}' gpurun_out/r06zf_bench_driver.log | head -5; exit $rc
