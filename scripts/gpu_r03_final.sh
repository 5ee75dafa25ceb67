#!/bin/bash
# full -m gpu suite + smoke (stop on failure), then the rocprofv3 trace + PMC profile of the driver-settings bench
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
[ -n "$NO_PROF" ] && exit 0
TAG=${TAG:-r03j} PMC=1 bash scripts/gpu_prof_r03.sh || exit $?
