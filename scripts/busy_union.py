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

# where the last update's idle time is: its largest gaps between the union's busy intervals, with the kernels either
# side (a host read drains the queue: the gap after it is the host's planning / queueing time)
if runs:
    a, b = runs[-1]
    seg = rows[a:b]
    gaps, cur_e, last_k = [], None, None
    for s, e, k in seg:
        if cur_e is not None and s > cur_e:
            gaps.append((s - cur_e, last_k, k, cur_e - seg[0][0]))
        if cur_e is None or e > cur_e:
            cur_e, last_k = e, k
    gaps.sort(reverse=True)
    tot = sum(g for g, *_ in gaps)
    print(f"last update: {len(gaps)} gaps, {tot / 1e6:.2f} ms; the largest:")
    for g, k0, k1, at in gaps[:12]:
        print(f"    {g / 1e3:8.1f} us at +{at / 1e6:7.2f} ms  after {k0[:48]:48s} before {k1[:48]}")


# rollout phases: from the first k_env_step of a run to the last one, plus the per-kernel means and the mean step
# period (k_env_step start to start), so the dispatch gaps of the captured rollout graph show
def union(seg):
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in seg:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return busy + (cur_e - cur_s if cur_e is not None else 0)


bounds = [marks[0]] + [b for a, b in zip(marks, marks[1:]) if b - a > 200]
ends = [a for a, b in zip(marks, marks[1:]) if b - a > 200] + [marks[-1]]
for a, b in list(zip(bounds, ends))[-3:]:
    seg = rows[a:b + 1]
    t0, t1 = seg[0][0], max(e for _, e, _ in seg)
    bz = union(seg)
    steps = [s for s, _, k in seg if "k_env_step" in k]
    per = (steps[-1] - steps[0]) / max(1, len(steps) - 1) / 1e3
    print(f"rollout: span {(t1 - t0) / 1e6:8.2f} ms, GPU busy (union) {bz / 1e6:8.2f} ms, {len(steps)} env steps, "
          f"step period {per:.1f} us, {len(seg)} dispatches")
    agg = {}
    for s, e, k in seg:
        n, tot = agg.get(k[:60], (0, 0))
        agg[k[:60]] = (n + 1, tot + e - s)
    for k, (n, tot) in sorted(agg.items(), key=lambda x: -x[1][1])[:8]:
        print(f"    {k:60s} {n:5d} x {tot / n / 1e3:7.1f} us")
