#!/bin/bash
# round 5 (z): rollout wall time per library variant (MERLIN_HIP_LIB), one process each, same seeds and warm-up
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
L=${LOG:-r05z}
: > gpurun_out/${L}.log
for v in ${VARIANTS:-v0 v3 v4}; do
    MERLIN_HIP_LIB="$R/ppo-2dgrid_amd/lib/libmerlin_$v.so" WARM=${WARM:-6} timeout -k 10 300 \
        python3 -u scripts/probe_rollout.py ${ROUNDS:-6} ${SET:-1} > gpurun_out/${L}_$v.log 2>&1 || exit $?
    echo "$v $(grep median gpurun_out/${L}_$v.log)" | tee -a gpurun_out/${L}.log
done
for v in ${STAGEVARS:-s0 v0 s2}; do
    MERLIN_HIP_LIB="$R/ppo-2dgrid_amd/lib/libmerlin_$v.so" timeout -k 10 120 python3 -u scripts/probe_stage.py 100 \
        > gpurun_out/${L}_stage_$v.log 2>&1 || exit $?
    echo "$v $(cat gpurun_out/${L}_stage_$v.log)" | tee -a gpurun_out/${L}.log
done
