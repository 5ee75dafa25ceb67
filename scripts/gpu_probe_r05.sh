#!/bin/bash
# round 5 probes: one python probe under a time limit, log under gpurun_out/
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 ${TLIM:-300} python -u $PROBE > gpurun_out/${LOG:-probe}.log 2>&1
rc=$?; tail -40 gpurun_out/${LOG:-probe}.log; exit $rc
