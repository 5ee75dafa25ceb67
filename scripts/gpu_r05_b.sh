#!/bin/bash
# round 5 (b): the plane-GEMM probe, the acting-table / fused-step tests, a short bench, the FOMAML kernel trace
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
PROBE="scripts/probe_h3_planes.py" LOG=probe_planes2 bash scripts/gpu_probe_r05.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout_graph.py tests/test_gpu_act_step.py tests/test_gpu_hard22.py tests/test_gpu_eval.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r05_b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/r05_b_tests.log | tail -30; tail -3 gpurun_out/r05_b_tests.log
[ "$rc" -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-tiers --no-cpu-baseline > gpurun_out/r05_bench_b.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05_bench_b.log") if l.startswith("{")][-1])
print("value", d["value"], "phases", d["phases_ms"], "frames", d["distinct_frames_per_sample"])
PY
bash scripts/gpu_prof_fomaml.sh
