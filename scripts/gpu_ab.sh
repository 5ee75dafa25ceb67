#!/bin/bash
# in-process A/B of update switches (scripts/ab_update.py), after the selected GPU tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/pytest_sel.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_sel.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u scripts/ab_update.py ${AB_ARGS:-3 4 deferred,torch_opt} > gpurun_out/ab.log 2>&1; rc=$?
tail -5 gpurun_out/ab.log; exit $rc
