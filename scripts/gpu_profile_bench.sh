#!/bin/bash
# rocprofv3 kernel trace of the bench at the driver's settings (20 timed steps after 5 warmups), untruncated
# kernel names (template arguments tell the x6 GEMM roles and the segmented-sum passes apart), then separate
# PMC passes (FETCH_SIZE, WRITE_SIZE) over the SAME command; the summaries keep only each kernel's launches of the
# timed iterations (PMC_TIMED_FRAC = steps / (steps + warmup)), so kernel times and bytes per launch describe the
# training state the bench line measures; summaries written on the box.
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --no-tiers}"
PMC_ARGS="${PMC_ARGS:-$ARGS}"
export PMC_TIMED_FRAC="${PMC_TIMED_FRAC:-0.8}"
timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/prof_trace" -o run -- \
    python "$R/bench.py" $ARGS > "$R/gpurun_out/prof_trace.log" 2>&1 || exit $?
tail -c 400 "$R/gpurun_out/prof_trace.log"
if [ -n "$PMC" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 420 rocprofv3 --pmc $C --kernel-include-regex "${PMC_RE:-k_}" -f csv \
        -d "$R/gpurun_out/prof_pmc_$C" -o run -- python "$R/bench.py" $PMC_ARGS \
        > "$R/gpurun_out/prof_pmc_$C.log" 2>&1 || exit $?
    echo "pmc $C done"
  done
fi
cd "$R" && python scripts/prof_summary.py "${TAG:-r06}" gpurun_out/summary || exit $?
python scripts/busy_union.py gpurun_out/prof_trace/run_kernel_trace.csv > gpurun_out/summary/${TAG:-r06}_busy_union.txt
python scripts/kernel_sequence.py gpurun_out/prof_trace/run_kernel_trace.csv \
    gpurun_out/summary/${TAG:-r06}_step_sequence.md || true
cp gpurun_out/prof_trace.log gpurun_out/summary/ 2>/dev/null
rm -f gpurun_out/prof_*/run_kernel_trace.csv gpurun_out/prof_*/run_counter_collection.csv
