"""GPU idle time from a rocprofv3 kernel trace: union of kernel intervals (all queues) vs wall span, over the
last N update phases (an update = the dispatches between two rollout graphs).  python scripts/busy_union.py <trace.csv>"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
# iteration boundaries: the rollout's k_env_step dispatches come in runs; an update = dispatches after the last
# k_env_step of a run until the next k_env_step
marks = [i for i, (_, _, k) in enumerate(rows) if "k_env_step" in k]
runs = []
start = marks[0]
for a, b in zip(marks, marks[1:]):
    if b - a > 200:  # a gap in env steps: the update in between
        runs.append((a + 1, b))
out = []
for a, b in runs[-6:]:
    seg = rows[a:b]
    t0, t1 = seg[0][0], max(e for _, e, _ in seg)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in seg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    out.append(((t1 - t0) / 1e6, busy / 1e6, len(seg)))
for w, bz, n in out:
    print(f"update: span {w:8.1f} ms, GPU busy (union) {bz:8.1f} ms, idle {w - bz:7.1f} ms ({(w - bz) / w * 100:.1f} %), {n} dispatches")
