#!/bin/bash
# round 5 (c): FOMAML's fused acting step + the compact acting table: tests, the FOMAML bench, its kernel trace
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_grouped_policy.py tests/test_gpu_fomaml.py tests/test_gpu_cli.py::test_fomaml_cli_smoke tests/test_gpu_rollout_graph.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r05_c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/r05_c_tests.log | tail -30; tail -3 gpurun_out/r05_c_tests.log
[ "$rc" -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --fomaml --steps 5 --warmup 2 > gpurun_out/r05_fomaml_bench.log 2>&1 || exit $?
tail -2 gpurun_out/r05_fomaml_bench.log
TAG=r05b bash scripts/gpu_prof_fomaml.sh || exit $?
bash scripts/gpu_pmc_gemm_r05.sh
exit $rc
