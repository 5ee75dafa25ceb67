#!/bin/bash
# a list of GPU test files (TESTS), stop on the first failure; log under gpurun_out/
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
LOG=gpurun_out/${LOG:-pytest_sel}.log
timeout -k 10 ${TLIM:-600} python -u -m pytest ${TESTS:-tests} -v -m gpu -x --timeout ${PER:-150} --timeout-method thread > $LOG 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" $LOG | tail -40; tail -5 $LOG; exit $rc
