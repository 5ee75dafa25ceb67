"""Per-optimizer-step timeline of the timed updates in a rocprofv3 kernel trace of scripts/ab_update.py (one
setting): the dispatches after the last rollout, cut into steps at each k_opt_adam.  Prints per step the span, the
GPU busy union and per queue the kernel time, medians over the steps; and the median duration of each kernel.
    python scripts/update_timeline.py <run_kernel_trace.csv>"""
import csv
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import kname  # noqa: E402

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "0")))
rows.sort()
last_env = max(i for i, r in enumerate(rows) if "k_env_step" in r[2])
rows = rows[last_env + 1:]
def report(steps):
    spans, busys, perq, kern = [], [], {}, {}
    for seg in steps:

        t0, t1 = seg[0][0], max(e for _, e, _, _ in seg)
        spans.append(t1 - t0)
        busy, cs, ce = 0, None, None
        for s, e, _, _ in seg:
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        busys.append(busy)
        q = {}
        for s, e, k, qid in seg:
            q[qid] = q.get(qid, 0) + e - s
            name = kname(k)
            kern.setdefault(f"q{qid} {name}", []).append(e - s)
        for qid, v in q.items():
            perq.setdefault(qid, []).append(v)
    print(f"steps {len(steps)}  span median {st.median(spans) / 1e3:.1f} us (mean {st.mean(spans) / 1e3:.1f})  busy median "
          f"{st.median(busys) / 1e3:.1f} us (mean {st.mean(busys) / 1e3:.1f})")
    for qid, v in sorted(perq.items()):
        print(f"  queue {qid}: kernel time median {st.median(v) / 1e3:.1f} us per step (mean {st.mean(v) / 1e3:.1f})")
    n = max(1, len(steps))
    for name, v in sorted(kern.items(), key=lambda kv: -sum(kv[1]))[:int(os.environ.get("TOPK", "26"))]:
        print(f"  {name[:70]:70s} {len(v) / n:5.2f}/step  median {st.median(v) / 1e3:8.1f} us  mean/step "
              f"{sum(v) / n / 1e3:8.1f} us")



cuts = [-1] + [i for i, r in enumerate(rows) if "k_opt_adam" in r[2]]
allsteps = [rows[a + 1:b + 1] for a, b in zip(cuts, cuts[1:])]
# scripts/ab_update.py alternates its settings update by update (80 optimizer steps each): with their names given,
# the steps are grouped per setting
names = sys.argv[2].split(",") if len(sys.argv) > 2 else [None]
SPU = int(os.environ.get("STEPS_PER_UPDATE", "80"))
for si, setting in enumerate(names):
    steps = [st_ for u in range(len(allsteps) // SPU) if u % len(names) == si
             for st_ in allsteps[u * SPU + 1:(u + 1) * SPU]] if setting else allsteps[1:]
    if setting:
        print(f"== {setting}")
    report(steps)
