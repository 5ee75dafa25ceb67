#!/bin/bash
# round 6 (final, part 3): the whole -m gpu suite and smoke() on the tree after the late probes (product code as in
# r06zf), then the driver-settings line with every tier and the CPU baseline (env-tier traffic now from r06zf_pmc.json)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 800 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r06zg_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r06zg_pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/r06zg_pytest_gpu.log | head -10
crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zg_smoke.log 2>&1; rc=$?
tail -1 gpurun_out/r06zg_smoke.log; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06zg_bench_driver.log 2>&1; rc=$?
grep -o '"value": [0-9.]*\|"phases_ms": {[^}]*}' gpurun_out/r06zg_bench_driver.log | head -3; exit $rc
