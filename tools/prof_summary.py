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
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
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
