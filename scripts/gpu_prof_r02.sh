#!/bin/bash
# rocprofv3 kernel trace + stats of the bench at the driver's settings (20 timed steps after 5
# warmups), then separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the same command.
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --no-tiers}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d "$R/gpurun_out/prof_trace" -o run -- \
    python "$R/bench.py" $ARGS > "$R/gpurun_out/prof_trace.log" 2>&1 || exit $?
tail -c 600 "$R/gpurun_out/prof_trace.log"
if [ -n "$PMC" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "${PMC_RE:-k_}" -f csv \
        -d "$R/gpurun_out/prof_pmc_$C" -o run -- python "$R/bench.py" $ARGS \
        > "$R/gpurun_out/prof_pmc_$C.log" 2>&1 || exit $?
    echo "pmc $C done"
  done
  for C in FETCH_SIZE WRITE_SIZE; do  # the HBM-scale env tier alone (2M envs) -> k_env_step_large
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_step" -T -f csv \
        -d "$R/gpurun_out/prof_pmcenv_$C" -o run -- python "$R/bench.py" --env-tier-only \
        > "$R/gpurun_out/prof_pmcenv_$C.log" 2>&1 || exit $?
    echo "pmc env $C done"
  done
fi
# summaries on the box (the raw per-launch CSVs exceed what gpurun copies back), then drop the raw files
cd "$R" && python scripts/prof_summary.py "${TAG:-r02}" gpurun_out/summary || exit $?
cp gpurun_out/prof_trace.log gpurun_out/summary/ 2>/dev/null
rm -f gpurun_out/prof_*/run_kernel_trace.csv gpurun_out/prof_*/run_counter_collection.csv
