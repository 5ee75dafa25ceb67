#!/bin/bash
# PMC passes over the h3 GEMM probe (scripts/probe_h3.py): SQ counters of the k_h3_* kernels
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmc_h3"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/pmc_h3/counters.txt" 2>&1
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "k_h3_" -f csv -d "$R/gpurun_out/pmc_h3/p$i" -o run -- \
      python "$R/scripts/probe_h3.py" 111000 2 > "$R/gpurun_out/pmc_h3/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc_h3/p$i.log"; }
done
cd "$R" && python - <<'PY'
import csv, glob, collections, re
out = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/pmc_h3/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_h3_\w*<[^>]*>)", r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:60]
        out[k].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
with open("gpurun_out/pmc_h3/summary.txt", "w") as f:
    for k, d in out.items():
        f.write(k + "\n")
        for c, v in sorted(d.items()):
            f.write(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})\n")
print(open("gpurun_out/pmc_h3/summary.txt").read())
PY
rm -f gpurun_out/pmc_h3/p*/run_counter_collection.csv
