#!/bin/bash
# rocprofv3 passes over the bench command (kernel trace + stats; then separate PMC passes
# for k_env_step's HBM bytes).  Outputs under gpurun_out/prof*.
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --no-tiers"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d "$R/gpurun_out/prof_trace" -o run -- \
    python "$R/bench.py" $ARGS > "$R/gpurun_out/prof_trace.log" 2>&1 || exit $?
tail -2 "$R/gpurun_out/prof_trace.log"
if [ -n "$PMC" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "k_env_step|k_conv|k_im2col3|k_col2im3|k_gae|k_adv|k_window|k_seg|k_bias_relu|k_relu_bwd|k_head" -T -f csv \
        -d "$R/gpurun_out/prof_pmc_$C" -o run -- python "$R/bench.py" $ARGS --no-graph \
        > "$R/gpurun_out/prof_pmc_$C.log" 2>&1 || exit $?
    echo "pmc $C done"
  done
  # the HBM-scale env tier alone (2M envs): k_env_step's per-launch HBM bytes -> k_env_step_large
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_env_step" -T -f csv \
        -d "$R/gpurun_out/prof_pmcenv_$C" -o run -- python "$R/bench.py" --env-tier-only \
        > "$R/gpurun_out/prof_pmcenv_$C.log" 2>&1 || exit $?
    echo "pmc env $C done"
  done
fi
find "$R/gpurun_out" -name "*.csv" | head -20
if [ -n "$LAYERS" ]; then
  timeout -k 10 400 python "$R/scripts/probe_layers.py" 2>&1 | tee "$R/gpurun_out/probe_layers.log"
fi
