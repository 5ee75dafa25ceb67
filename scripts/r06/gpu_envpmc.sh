#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over bench.py --env-tier-only (2M envs): the HBM bytes of k_env_step's roofline
# launches (the last 16, auto-reset off), merged into profiles/<TAG>_pmc.json as k_env_step_large.
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/summary"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 python "$R/bench.py" --env-tier-only > "$R/gpurun_out/envtier.log" 2>&1 || exit $?
cat "$R/gpurun_out/envtier.log"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex k_env_step -f csv \
      -d "$R/gpurun_out/prof_pmcenv_$C" -o run -- python "$R/bench.py" --env-tier-only \
      > "$R/gpurun_out/prof_pmcenv_$C.log" 2>&1 || exit $?
  echo "pmc $C done"
done
cd "$R" && cp profiles/${TAG}_pmc.json gpurun_out/summary/ && \
  PMC_MERGE_ENV=1 python scripts/prof_summary.py "$TAG" gpurun_out/summary || exit $?
python - <<PY
import json; d=json.load(open("gpurun_out/summary/${TAG}_pmc.json")); print(d.get("k_env_step_large"))
PY
rm -f gpurun_out/prof_pmcenv_*/run_counter_collection.csv
