#!/bin/bash
# rocprofv3 kernel trace of the FOMAML tier (BASELINE cfg 5: 32 tasks x 256 support + 256 query steps per meta
# step), summarised on the box under gpurun_out/summary/<TAG>_fomaml_*.
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/summary"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/prof_fomaml" -o run -- \
    python "$R/bench.py" --fomaml --steps ${STEPS:-3} --warmup 2 > "$R/gpurun_out/prof_fomaml.log" 2>&1 || exit $?
tail -c 600 "$R/gpurun_out/prof_fomaml.log"
cd "$R" && PROF_TRACE_DIR=prof_fomaml python scripts/prof_summary.py "${TAG:-r05}_fomaml" gpurun_out/summary || exit $?
python scripts/busy_union.py gpurun_out/prof_fomaml/run_kernel_trace.csv > gpurun_out/summary/${TAG:-r05}_fomaml_busy_union.txt 2>&1 || true
cp gpurun_out/prof_fomaml.log gpurun_out/summary/${TAG:-r05}_fomaml_bench.log
rm -f gpurun_out/prof_fomaml/run_kernel_trace.csv
