#!/bin/bash
# kernel trace of a short bench run, then the GPU busy/idle split of the update phases (scripts/busy_union.py)
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/busy"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/busy" -o run -- \
    python "$R/bench.py" ${BENCH_ARGS:---steps 4 --warmup 6 --no-cpu-baseline --no-tiers} > "$R/gpurun_out/busy/log" 2>&1 || exit $?
python "$R/scripts/busy_union.py" "$R/gpurun_out/busy/run_kernel_trace.csv" | tee "$R/gpurun_out/busy/summary.txt"
rm -f "$R/gpurun_out/busy/run_kernel_trace.csv"
