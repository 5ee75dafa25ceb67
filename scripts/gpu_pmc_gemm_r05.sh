#!/bin/bash
# PMC passes (one rocprofv3 run each, SQ counters) over one h3 NT GEMM configuration: where the waves' cycles go
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmc_r05"
cd /tmp && export TMPDIR=/tmp
for spec in ${CFGS:-42:1 13:0}; do
  cfg=${spec%%:*}; pl=${spec##*:}
  i=0
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "k_h3_nt" -f csv -d "$R/gpurun_out/pmc_r05/c${cfg}_p$i" -o run -- \
        python "$R/scripts/probe_gemm_one.py" $cfg 4 $pl > "$R/gpurun_out/pmc_r05/c${cfg}_p$i.log" 2>&1 || exit $?
  done
done
cd "$R" && python - <<'PY'
import csv, glob, os, collections
out = []
for d in sorted(glob.glob("gpurun_out/pmc_r05/c*_p*")):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "k_h3_nt" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out.append(os.path.basename(d) + " " + " ".join(f"{k}={sum(v)/len(v):.4g}" for k, v in sorted(acc.items())))
open("gpurun_out/pmc_r05/summary.txt", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
rm -f gpurun_out/pmc_r05/*/run_counter_collection.csv
