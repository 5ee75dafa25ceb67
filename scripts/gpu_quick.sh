#!/bin/bash
# subset of GPU tests + a short bench (development loop)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${TESTS:-tests} -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-tiers} 2>&1 | tee gpurun_out/bench.log
exit ${PIPESTATUS[0]}
