#!/bin/bash
# round 6 (j): the tree after the session restart -- the full GPU suite and smoke(), then the driver-settings bench
# with every tier (FOMAML with its captured inner / outer steps)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 150 python -u scripts/probe_one_acc.py 111000 20 > gpurun_out/r06j_one_acc.log 2>&1; rc=$?
cat gpurun_out/r06j_one_acc.log; crash $rc && exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r06j_pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r06j_pytest_gpu.log; grep -E "FAIL|Error" gpurun_out/r06j_pytest_gpu.log | head -20
crash $rc && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06j_smoke.log 2>&1; rc=$?
tail -3 gpurun_out/r06j_smoke.log; crash $rc && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06j_bench_driver.log 2>&1; rc=$?
tail -c 2500 gpurun_out/r06j_bench_driver.log; exit $rc
