#!/bin/bash
# round 5 (m): one A/B setting per process (no allocator / cache sharing between settings)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for s in ${AB:-fast fast_nodzp fast_noa3p fast}; do
  timeout -k 10 300 python -u scripts/ab_update.py 3 5 $s > gpurun_out/r05m_$s.log 2>&1 || exit $?
  grep "ms/update" gpurun_out/r05m_$s.log
done
