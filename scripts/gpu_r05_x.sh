#!/bin/bash
# round 5 (x): env parity after a kernel change (goldens, oracle, rollout graph), then the rollout's kernel stats
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
L=${LOG:-r05x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_env.py \
    tests/test_gpu_hard22.py tests/test_gpu_rollout_graph.py tests/test_gpu_act_step.py} > gpurun_out/${L}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${L}_pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
WARM=${WARM:-6} timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_$L" -o run -- \
    python3 -u "$R/scripts/probe_rollout.py" ${ROUNDS:-4} ${SET:-1} > "$R/gpurun_out/${L}_rollout.log" 2>&1 || exit $?
cat "$R/gpurun_out/${L}_rollout.log" | grep median
cp "$R/gpurun_out/prof_$L/run_kernel_stats.csv" "$R/gpurun_out/${L}_kernel_stats.csv"
python3 "$R/scripts/busy_union.py" "$R/gpurun_out/prof_$L/run_kernel_trace.csv" > "$R/gpurun_out/${L}_busy.txt" 2>&1
grep -E "refill|fallback|env_step|codes_conv3|k_h3_ntp" "$R/gpurun_out/${L}_kernel_stats.csv" | cut -c1-200
rm -rf "$R/gpurun_out/prof_$L"
