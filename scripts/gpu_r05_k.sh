#!/bin/bash
# round 5 (k): refill / step kernel times per library variant (rocprofv3 kernel stats of scripts/probe_rollout.py)
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
L=${LOG:-r05k2}
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-x0 x1}; do
    MERLIN_HIP_LIB="$R/ppo-2dgrid_amd/lib/libmerlin_$v.so" WARM=${WARM:-12} timeout -k 10 300 rocprofv3 --kernel-trace \
        --stats -f csv -d "$R/gpurun_out/prof_${L}_$v" -o run -- python3 -u "$R/scripts/probe_rollout.py" 3 1 \
        > "$R/gpurun_out/${L}_$v.log" 2>&1 || exit $?
    echo "$v $(grep median "$R/gpurun_out/${L}_$v.log")"
    grep -E "k_env_refill<16, 16>|k_patch_maps<0>" "$R/gpurun_out/prof_${L}_$v/run_kernel_stats.csv" | cut -d, -f1-4
    rm -rf "$R/gpurun_out/prof_${L}_$v"
done
