#!/bin/bash
# round 5 (s): in-process A/B (the same update replayed under each setting): wall clock, then a kernel trace of
# the same alternation with per-setting step timelines
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
S=${AB:-fast,fast_noa3p,fast_nodzp}
L=${LOG:-r05s}
timeout -k 10 500 python -u scripts/ab_update.py ${REP:-3} 5 $S > gpurun_out/${L}_ab.log 2>&1 || exit $?
grep "ms/update" gpurun_out/${L}_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/prof_$L" -o run -- \
    python3 -u "$R/scripts/ab_update.py" 1 5 $S > "$R/gpurun_out/${L}_trace.log" 2>&1 || exit $?
TOPK=80 python3 "$R/scripts/update_timeline.py" "$R/gpurun_out/prof_$L/run_kernel_trace.csv" $S > "$R/gpurun_out/${L}_timeline.txt" 2>&1
gzip -c "$R/gpurun_out/prof_$L/run_kernel_trace.csv" > "$R/gpurun_out/${L}_trace.csv.gz"; rm -rf "$R/gpurun_out/prof_$L"
grep -A3 "^==" "$R/gpurun_out/${L}_timeline.txt"
