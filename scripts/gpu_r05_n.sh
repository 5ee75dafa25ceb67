#!/bin/bash
# round 5 (n): per-step timelines of the update under one setting per process (kernel trace)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for s in ${AB:-fast fast_noa3p}; do
  timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/prof_n_$s" -o run -- \
      python3 -u "$R/scripts/ab_update.py" 2 5 $s > "$R/gpurun_out/r05n_$s.log" 2>&1 || exit $?
  python3 "$R/scripts/update_timeline.py" "$R/gpurun_out/prof_n_$s/run_kernel_trace.csv" > "$R/gpurun_out/r05n_${s}_timeline.txt" 2>&1
  rm -rf "$R/gpurun_out/prof_n_$s"
  echo "== $s"; head -32 "$R/gpurun_out/r05n_${s}_timeline.txt"
done
