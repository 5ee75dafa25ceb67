#!/bin/bash
# round 6 (af): k_env_step with the block's wall rows read as one coalesced run (LDS transpose) against the per-lane
# 16-B pieces (lib/libmerlin_hip_base.so): env / rollout tests on the new kernel, then the 2M-env tier and the rollout
# at the bench state, alternating libraries (one process each)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
crash() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_env.py \
    tests/test_gpu_rollout_graph.py > gpurun_out/r06af_tests.log 2>&1; rc=$?
echo "tests: $(tail -1 gpurun_out/r06af_tests.log)"; crash $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
BASE="$R/ppo-2dgrid_amd/lib/libmerlin_hip_base.so"
for L in new base new base; do
  if [ $L = base ]; then export MERLIN_HIP_LIB="$BASE"; else unset MERLIN_HIP_LIB; fi
  timeout -k 10 180 python -u bench.py --env-tier-only > gpurun_out/r06af_env_$L.log 2>&1; rc=$?
  echo "env $L: $(tail -1 gpurun_out/r06af_env_$L.log | cut -c1-260)"; crash $rc && exit $rc
  WARM=6 timeout -k 10 300 python -u scripts/probe_rollout.py 5 1 > gpurun_out/r06af_roll_$L.log 2>&1; rc=$?
  echo "rollout $L: $(tail -1 gpurun_out/r06af_roll_$L.log)"; crash $rc && exit $rc
done
exit 0
