"""Turn rocprofv3 outputs under gpurun_out/ into the committed profiles/ summaries.

    python scripts/prof_summary.py <tag> [dest]
writes <dest, default profiles>/<tag>_kernel_stats.md (+ .csv copy) from the --kernel-trace --stats pass and
profiles/<tag>_pmc.json from the FETCH_SIZE / WRITE_SIZE passes: per kernel, the mean over
its largest-grid launches, HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950:
FETCH_SIZE counts half of a wide coalesced read stream, MI355X_MICROARCH.md §HBM).
"""
import csv
import re
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
DEST = os.path.join(REPO, "profiles")


def stats(tag):
    src = os.path.join(OUT, "prof_trace", "run_kernel_stats.csv")
    if not os.path.exists(src):
        return
    rows = list(csv.DictReader(open(src)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {tag}: rocprofv3 --kernel-trace --stats of `bench.py` (1 warmup + timed iterations)", "",
             f"total kernel time {tot / 1e6:.1f} ms", "",
             "| kernel | calls | total ms | % | avg us |", "|---|---|---|---|---|"]
    for r in rows[:40]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['Percentage']):.2f} | {float(r['AverageNs']) / 1e3:.2f} |")
    os.makedirs(DEST, exist_ok=True)
    open(os.path.join(DEST, f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    shutil.copy(src, os.path.join(DEST, f"{tag}_kernel_stats.csv"))


def pmc(tag):
    res = {}
    # prof_pmc_*: the bench loop; prof_pmcenv_*: bench.py --env-tier-only (2M envs), whose
    # k_env_step launches are keyed k_env_step_large (bench.py tiers.env_only_2M_envs)
    for pre, rename in (("prof_pmc_", {}), ("prof_pmcenv_", {"k_env_step": "k_env_step_large"})):
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            src = os.path.join(OUT, f"{pre}{counter}", "run_counter_collection.csv")
            if os.path.exists(src):
                collect(res, src, counter, rename)
    for k, d in res.items():
        if "fetch_size_kb" in d and "write_size_kb" in d:
            d["hbm_bytes_per_launch"] = int((2 * d["fetch_size_kb"] + d["write_size_kb"]) * 1024)
    if res:
        json.dump(res, open(os.path.join(DEST, f"{tag}_pmc.json"), "w"), indent=1)


def collect(res, src, counter, rename):
    per = {}
    for r in csv.DictReader(open(src)):
        raw = r["Kernel_Name"]
        m = re.search(r"::(k_\w+(?:<[^>]*>)?)\(", raw)  # untruncated merlin kernel: keep template args
        if m:
            name = m.group(1)
        else:
            name = raw.split("(")[0].split("<")[0].replace("void ", "").strip()
            name = name.split("::")[-1]
        name = rename.get(name, name)
        per.setdefault(name, []).append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    for k, vals in per.items():
        g = max(v[0] for v in vals)
        big = [v[1] for v in vals if v[0] == g]
        d = res.setdefault(k, {"grid": g, "launches": len(big)})
        d[counter.lower() + "_kb"] = sum(big) / len(big)


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    if len(sys.argv) > 2:
        DEST = os.path.abspath(sys.argv[2])
    stats(tag)
    pmc(tag)
    print("wrote profiles for", tag)
