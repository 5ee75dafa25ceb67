#!/bin/bash
# rocprofv3 HIP API trace + stats of a short bench run: which host calls block (syncs, mallocs)
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/hiptrace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-trace --stats -f csv -d "$R/gpurun_out/hiptrace" -o run -- \
    python "$R/bench.py" ${BENCH_ARGS:---steps 3 --warmup 3 --no-cpu-baseline --no-tiers} > "$R/gpurun_out/hiptrace/log" 2>&1 || exit $?
cd "$R/gpurun_out/hiptrace" && ls && head -40 run_hip_api_stats.csv
python - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("run_hip_api_trace.csv")))
print(len(rows), "hip api calls; columns", list(rows[0].keys()))
# long calls (> 200 us) by function
long = collections.Counter(); tot = collections.Counter()
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if d > 200:
        long[r["Function"]] += 1
        tot[r["Function"]] += d
for f, c in long.most_common(20):
    print(f"{f:40s} {c:6d} calls > 200us, {tot[f]/1e3:9.1f} ms")
PY
rm -f run_hip_api_trace.csv
