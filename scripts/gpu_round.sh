#!/bin/bash
# tests + smoke + bench + rocprofv3 trace/PMC passes, all bounded; stops at the first crash/timeout
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
BENCH_ARGS="${BENCH_ARGS:---steps 2 --warmup 1}" bash scripts/gpu_check.sh || exit $?
STEPS=1 PMC=1 bash scripts/gpu_profile.sh
