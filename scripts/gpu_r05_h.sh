#!/bin/bash
# round 5 (h): the in-process A/B with per-kernel HIP-event times
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/ab_update.py 2 5 ${AB:-fast_timers4,fast_noa3p_timers4,fast_nodzp_timers4} > gpurun_out/${LOG:-r05h_ab}.log 2>&1
rc=$?; tail -70 gpurun_out/${LOG:-r05h_ab}.log; exit $rc
