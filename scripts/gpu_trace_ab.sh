#!/bin/bash
# kernel trace of one A/B setting (per-kernel times by template instance)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
L=${LOG:-r06t}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_$L" -o run -- \
    python3 -u "$R/scripts/ab_update.py" 1 5 ${AB:-fast} > "$R/gpurun_out/$L.log" 2>&1
rc=$?; cd "$R"; tail -5 gpurun_out/$L.log
PROF_TRACE_DIR=prof_$L python3 scripts/prof_summary.py $L gpurun_out/${L}_prof > /dev/null 2>&1
head -45 gpurun_out/${L}_prof/${L}_kernel_stats.md
rm -rf gpurun_out/prof_$L
exit $rc
