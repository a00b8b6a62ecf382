"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel (short name),
mean of each counter over its dispatches, plus mean duration."""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--match", default="oamd", help="substring filter on the kernel name")
ap.add_argument("--grid", action="store_true", help="key kernels by name AND grid size (one template, many shapes)")
a = ap.parse_args()
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for r in csv.DictReader(open(a.csv)):
    name = r["Kernel_Name"]
    if not re.search(a.match, name):
        continue
    short = re.sub(r"\(.*", "", name)[:80]
    if a.grid:
        short += f" grid={r.get('Grid_Size') or r.get('Grid_Size_X', '?')}"
    agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[short][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, cs in agg.items():
    d = list(dur[k].values())
    print(k, f"dispatches={len(d)} mean_us={sum(d) / len(d):.1f}")
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):.4g}")
