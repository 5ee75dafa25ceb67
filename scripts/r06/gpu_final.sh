#!/bin/bash
# round 6 (final): the whole -m gpu suite and smoke() on the final tree, then the driver-settings bench under rocprofv3
# (kernel trace + FETCH_SIZE / WRITE_SIZE passes, step sequence, busy union), then the driver-settings line with every
# tier and the CPU baseline
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 800 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r06zf_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r06zf_pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/r06zf_pytest_gpu.log | head -10
crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zf_smoke.log 2>&1; rc=$?
tail -1 gpurun_out/r06zf_smoke.log; crash $rc && exit $rc
exit 0
