#!/bin/bash
# round 5: the new / changed GPU tests, then a short bench line; logs under gpurun_out/
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
T="tests/test_gpu_capture_safety.py tests/test_gpu_cli.py::test_fomaml_cli_smoke tests/test_gpu_h3.py::test_gemm_nt_dynamic_range tests/test_gpu_h3.py::test_gemm_tn_dynamic_range tests/test_gpu_windows.py::test_window_conv3_patch_reuse_bitwise tests/test_gpu_fast_step.py::test_patch_reuse_partial_rows_never_read_directly tests/test_gpu_dp.py::test_eight_rank_ppo_equals_one_process_over_concatenated_envs tests/test_gpu_bench_dp.py tests/test_gpu_act_step.py tests/test_gpu_rollout_graph.py ${EXTRA}"
timeout -k 10 900 python -u -m pytest $T -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r05_check.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/r05_check.log | tail -40; tail -3 gpurun_out/r05_check.log
[ "$rc" -le 1 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-tiers --no-cpu-baseline > gpurun_out/r05_bench.log 2>&1 || exit $?
  tail -c 1500 gpurun_out/r05_bench.log
fi
exit $rc
