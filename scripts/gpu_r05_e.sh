#!/bin/bash
# round 5 (e): GEMM ablation probe, acting-path tests, a short bench (rollout phase)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
PROBE="scripts/probe_h3_ablate.py" LOG=probe_ablate bash scripts/gpu_probe_r05.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout_graph.py tests/test_gpu_act_step.py tests/test_gpu_hard22.py tests/test_gpu_grouped_policy.py::test_group_act_parts_match_per_task_models -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r05_e_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/r05_e_tests.log | tail -30; tail -3 gpurun_out/r05_e_tests.log
[ "$rc" -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-tiers --no-cpu-baseline > gpurun_out/r05_bench_e.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05_bench_e.log") if l.startswith("{")][-1])
print("value", d["value"], "phases", d["phases_ms"], "frames", d["distinct_frames_per_sample"])
PY
exit $rc
