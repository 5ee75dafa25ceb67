#!/bin/bash
# round-2 GPU check: parity tests (bounded), then the bench at the driver's settings
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/bench.log 2>&1
rc=$?; tail -c 3000 gpurun_out/bench.log; exit $rc
