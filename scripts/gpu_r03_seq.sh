#!/bin/bash
# kernel trace of the driver-settings bench: per-kernel stats + one optimizer step's sequence (prof_summary.py) and
# the GPU busy / idle split of the update phases (busy_union.py)
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/prof_trace" -o run -- \
    python "$R/bench.py" ${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --no-tiers} > "$R/gpurun_out/prof_trace.log" 2>&1 || exit $?
cd "$R" && python scripts/busy_union.py gpurun_out/prof_trace/run_kernel_trace.csv | tee gpurun_out/busy_union.txt
python scripts/prof_summary.py "${TAG:-r03}" gpurun_out/summary || exit $?
cp gpurun_out/busy_union.txt gpurun_out/summary/${TAG:-r03}_busy_union.txt
rm -f gpurun_out/prof_trace/run_kernel_trace.csv
