"""Turn rocprofv3 outputs under gpurun_out/ into the committed profiles/ summaries.

    python scripts/prof_summary.py <tag> [dest]
writes <dest, default profiles>/<tag>_kernel_stats.md (+ .csv copy) from the --kernel-trace --stats pass and
profiles/<tag>_pmc.json from the FETCH_SIZE / WRITE_SIZE passes: per kernel, the mean over its launches,
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts half of a wide coalesced read
stream, MI355X_MICROARCH.md §HBM).
PMC_TIMED_FRAC (env, default 1): keep only the last fraction of each kernel's launches, in dispatch order -- with
the bench run as `--steps K --warmup W --no-tiers --no-cpu-baseline` that is K / (K + W), the launches of the timed
iterations, so the kernel times and PMC bytes describe the same training state as the bench line's HIP events
(the update's work grows with the distinct frames per minibatch as the policy trains).
"""
import csv
import re
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
TIMED_FRAC = float(os.environ.get("PMC_TIMED_FRAC", "1"))


def timed_tail(vals):
    """The last TIMED_FRAC of a kernel's launches (in dispatch order)."""
    import math

    k = max(1, math.ceil(len(vals) * TIMED_FRAC))
    return vals[-k:]


DEST = os.path.join(REPO, "profiles")


def kname(raw):
    """Kernel name for the tables: merlin kernels keep their template arguments (the x6 GEMM roles and
    the segmented-sum passes are template instantiations), others are cut to the function name."""
    m = re.search(r"::(k_\w+(?:<[^>]*>)?)\(", raw) or re.search(r"^(k_\w+(?:<[^>]*>)?)", raw)
    if m:
        return m.group(1)
    name = raw.split("(")[0].split("<")[0].replace("void ", "").strip()
    return name.split("::")[-1][:90]


def stats(tag):
    """Per-kernel table from the per-dispatch kernel trace (untruncated names), plus the ordered
    launches of one optimizer step (scripts/kernel_sequence.py)."""
    src = os.path.join(OUT, os.environ.get("PROF_TRACE_DIR", "prof_trace"), "run_kernel_trace.csv")
    if not os.path.exists(src):
        return
    per = {}
    for r in csv.DictReader(open(src)):
        per.setdefault(kname(r["Kernel_Name"]), []).append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    agg = {}
    for k, v in per.items():
        v = timed_tail(sorted(v))
        agg[k] = [len(v), sum(d for _, d in v)]
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for v in agg.values())
    scope = "every launch" if TIMED_FRAC >= 1 else f"the last {TIMED_FRAC:.3f} of each kernel's launches (timed iterations)"
    lines = [f"# {tag}: rocprofv3 --kernel-trace of `bench.py` (per-dispatch durations, untruncated names; {scope})", "",
             f"total kernel time {tot / 1e6:.1f} ms", "",
             "| kernel | calls | total ms | % | avg us |", "|---|---|---|---|---|"]
    os.makedirs(DEST, exist_ok=True)
    with open(os.path.join(DEST, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ns", "avg_ns"])
        for k, (c, ns) in rows:
            w.writerow([k, c, ns, ns // c])
    for k, (c, ns) in rows[:60]:
        lines.append(f"| `{k}` | {c} | {ns / 1e6:.2f} | {100 * ns / tot:.2f} | {ns / c / 1e3:.2f} |")
    os.makedirs(DEST, exist_ok=True)
    open(os.path.join(DEST, f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import kernel_sequence

    try:
        kernel_sequence.main(src, os.path.join(DEST, f"{tag}_step_sequence.md"))
    except SystemExit as e:
        print("no step sequence:", e)


def env_rename(name):
    """bench.py --env-tier-only (2M envs): every k_env_step instantiation is keyed k_env_step_large (bench.py
    env_large_tier's roofline.traffic).  Its other kernels are dropped: they would collide with the bench loop's
    entries of the same name."""
    return "k_env_step_large" if name.startswith("k_env_step") else None


# bench.py --env-tier-only launches k_env_step 1 + 16 (auto-reset on) + 16 (auto-reset off, the roofline timing)
# times: the last 16 in dispatch order are the roofline's launches
ENV_TIMED = 16


def pmc(tag, merge=False):
    out = os.path.join(DEST, f"{tag}_pmc.json")
    res = json.load(open(out)) if merge and os.path.exists(out) else {}
    # prof_pmc_*: the bench loop; prof_pmcenv_*: bench.py --env-tier-only
    for pre, rename, last in (("prof_pmc_", None, None), ("prof_pmcenv_", env_rename, ENV_TIMED)):
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            src = os.path.join(OUT, f"{pre}{counter}", "run_counter_collection.csv")
            if os.path.exists(src):
                collect(res, src, counter, rename, last)
    for k, d in res.items():
        if "fetch_size_kb" in d and "write_size_kb" in d:
            d["hbm_bytes_per_launch"] = int((2 * d["fetch_size_kb"] + d["write_size_kb"]) * 1024)
    if res:
        json.dump(res, open(out, "w"), indent=1)


def collect(res, src, counter, rename=None, last=None):
    per = {}
    for r in csv.DictReader(open(src)):
        name = kname(r["Kernel_Name"])
        name = rename(name) if rename else name
        if name is None:
            continue
        per.setdefault(name, []).append((int(r["Dispatch_Id"]), int(r["Grid_Size"]), float(r["Counter_Value"])))
    for k, vals in per.items():
        # dispatch order; the timed iterations' launches
        vals = sorted(vals)[-last:] if last else timed_tail(sorted(vals))
        d = res.setdefault(k, {"grid_max": max(v[1] for v in vals), "launches": len(vals),
                               "timed_frac": TIMED_FRAC if not last else round(len(vals) / len(per[k]), 4)})
        d[counter.lower() + "_kb"] = sum(v[2] for v in vals) / len(vals)


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    if len(sys.argv) > 2:
        DEST = os.path.abspath(sys.argv[2])
    if os.environ.get("PMC_MERGE_ENV"):  # add the --env-tier-only passes to an existing <tag>_pmc.json
        pmc(tag, merge=True)
        print("merged env-tier PMC into", tag)
        sys.exit(0)
    stats(tag)
    pmc(tag)
    print("wrote profiles for", tag)
