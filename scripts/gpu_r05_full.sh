#!/bin/bash
# round 5: the full -m gpu suite (one process), log under gpurun_out/
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 ${TLIM:-1080} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/${LOG:-r05_pytest_gpu}.log 2>&1
rc=$?; grep -E "FAIL|ERROR" gpurun_out/${LOG:-r05_pytest_gpu}.log | head -20; tail -3 gpurun_out/${LOG:-r05_pytest_gpu}.log; exit $rc
