#!/bin/bash
# full -m gpu suite + smoke (stop on failure), then the driver-settings bench (all tiers) -> gpurun_out/
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench_driver.log 2>&1 || exit $?
tail -c 1500 gpurun_out/bench_driver.log
