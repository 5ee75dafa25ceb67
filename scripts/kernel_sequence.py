"""Ordered kernel launches of one optimizer step from a rocprofv3 --kernel-trace CSV.

    python scripts/kernel_sequence.py <run_kernel_trace.csv> <out.md> [anchor=k_ppo_loss]

Takes the launches between the last two `anchor` launches (one per minibatch in the window path),
ordered by start time, and writes name / stream queue / duration / gap to the previous end, plus
a per-name total, so the small torch kernels between the hand-written ones can be attributed.
"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    if m:
        return m.group(1)
    return name.split("(")[0].split("<")[0][-60:]


def main(src, out, anchor="k_ppo_loss"):
    rows = []
    for r in csv.DictReader(open(src)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if short(r[2]).split("<")[0] == anchor]
    if len(marks) < 3:
        raise SystemExit(f"fewer than 3 {anchor} launches")
    a, b = marks[-3], marks[-2]
    seg = rows[a:b]
    lines = [f"# one optimizer step: {len(seg)} launches between two `{anchor}` launches", "",
             f"span {(seg[-1][1] - seg[0][0]) / 1e3:.1f} us", "",
             "| # | kernel | queue | us | gap us |", "|---|---|---|---|---|"]
    tot = collections.Counter()
    cnt = collections.Counter()
    prev_end = seg[0][0]
    for i, (s, e, n, q) in enumerate(seg):
        k = short(n)
        tot[k] += (e - s) / 1e3
        cnt[k] += 1
        lines.append(f"| {i} | `{k}` | {q} | {(e - s) / 1e3:.1f} | {(s - prev_end) / 1e3:.1f} |")
        prev_end = max(prev_end, e)
    lines += ["", "| kernel | launches | total us |", "|---|---|---|"]
    for k, v in tot.most_common():
        lines.append(f"| `{k}` | {cnt[k]} | {v:.1f} |")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
