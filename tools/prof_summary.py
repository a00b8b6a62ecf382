"""Summarise a rocprofv3 kernel_trace.csv: per-kernel time in a window.

--after NAME : only dispatches after the LAST dispatch whose name contains NAME
--grid-x N   : only dispatches of kernels whose grid size ... (unused filter hook)
Prints the top kernels and the per-step total when --steps is given.
"""
import argparse
import csv
import collections

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--after", default=None)
ap.add_argument("--before", default=None, help="only dispatches before the FIRST dispatch containing this")
ap.add_argument("--steps", type=int, default=0)
ap.add_argument("--top", type=int, default=25)
ap.add_argument("--window-json", default=None, help="bench.py --json-out file: keep only its timed region")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if a.window_json:
    import json
    t0, t1 = json.load(open(a.window_json))["detail"]["timed_monotonic_ns"]
    rows = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
    print(f"timed window {(t1 - t0) / 1e6:.1f} ms")
if a.after:
    idx = max(i for i, r in enumerate(rows) if a.after in r["Kernel_Name"])
    rows = rows[idx + 1:]
if a.before:
    idx = min((i for i, r in enumerate(rows) if a.before in r["Kernel_Name"]), default=len(rows))
    rows = rows[:idx]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    k = r["Kernel_Name"][:90]
    agg[k][0] += 1
    agg[k][1] += d
tot = sum(v[1] for v in agg.values())
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3 if rows else 0
print(f"dispatches={len(rows)} busy={tot/1e3:.2f} ms span={span/1e3:.2f} ms")
if a.steps:
    print(f"per step: busy {tot/a.steps/1e3:.3f} ms, span {span/a.steps/1e3:.3f} ms")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
    extra = f" per-step {t/a.steps:8.1f}us" if a.steps else ""
    print(f"{t/1e3:9.3f} ms {100*t/tot:5.1f}% n={n:6d} avg={t/n:8.1f}us{extra}  {k}")

# ---- idle gaps (union of kernel intervals over all queues) ----
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows)
gaps, cur_end, prev_name = [], None, ""
busy_union = 0
for s, e, n in iv:
    if cur_end is None:
        busy_union += e - s
        cur_end, prev_name = e, n
        continue
    if s > cur_end:
        gaps.append((s - cur_end, prev_name, n))
        busy_union += e - s
        cur_end, prev_name = e, n
    elif e > cur_end:
        busy_union += e - cur_end
        cur_end, prev_name = e, n
idle = sum(g[0] for g in gaps)
print(f"union busy {busy_union/1e6:.2f} ms, idle {idle/1e6:.2f} ms in {len(gaps)} gaps "
      f"({sum(1 for g in gaps if g[0] > 1e5)} > 100 us, {sum(g[0] for g in gaps if g[0] > 1e5)/1e6:.2f} ms)")
for g, p, n in sorted(gaps, reverse=True)[:10]:
    print(f"  gap {g/1e3:10.1f} us after {p!r} before {n!r}")
