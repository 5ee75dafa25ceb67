#!/bin/bash
# round 6 (e): the reference-gradient tests; where a FOMAML meta step's time goes (phases, kernel trace)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_update_grad.py \
    > gpurun_out/r06e_grad.log 2>&1; rc=$?
grep -E "reference|PASS|FAIL|Error|passed|failed" gpurun_out/r06e_grad.log | tail -28; crash $rc && exit $rc
timeout -k 10 300 python -u scripts/probe_fomaml.py 4 > gpurun_out/r06e_fomaml_phases.log 2>&1 \
    || { tail -20 gpurun_out/r06e_fomaml_phases.log; exit 1; }
cat gpurun_out/r06e_fomaml_phases.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_fm" -o run -- \
    python3 -u "$R/bench.py" --fomaml --steps 5 --warmup 2 > "$R/gpurun_out/r06e_fomaml_trace.log" 2>&1; rc=$?
cd "$R"; tail -3 gpurun_out/r06e_fomaml_trace.log
PROF_TRACE_DIR=prof_fm python3 scripts/prof_summary.py r06e_fomaml gpurun_out/r06e_fm > /dev/null 2>&1
head -30 gpurun_out/r06e_fm/r06e_fomaml_kernel_stats.md
python3 scripts/busy_union.py gpurun_out/prof_fm/run_kernel_trace.csv > gpurun_out/r06e_fm/busy.txt 2>&1; tail -5 gpurun_out/r06e_fm/busy.txt
rm -f gpurun_out/prof_fm/run_kernel_trace.csv
exit $rc
