"""Compare kernel traces of bench ranks that share one GPU (tools/gpu/prof_two_procs.sh):
per-kernel time per rank, the union of busy time, and how much of it overlaps."""
import argparse
import collections
import csv
import glob
import json

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+", help="rocprofv3 output dirs or kernel_trace.csv files, one per process")
ap.add_argument("--window-json", required=True)
ap.add_argument("--top", type=int, default=14)
a = ap.parse_args()
t0, t1 = json.load(open(a.window_json))["detail"]["timed_monotonic_ns"]
print(f"timed window {(t1 - t0) / 1e6:.1f} ms")
ivs = []
for d in a.dirs:
    f = d if d.endswith(".csv") else glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ivs.append((s, e))
        g = agg[r["Kernel_Name"][:70]]
        g[0] += 1
        g[1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values())
    print(f"== {d}: {len(rows)} dispatches, kernel time {tot:.1f} ms")
    for name, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {ms:9.1f} ms  n={n:6d} avg={ms / n * 1e3:8.1f} us  {name}")
ivs.sort()
union = 0
cur_s, cur_e = ivs[0]
for s, e in ivs[1:]:
    if s > cur_e:
        union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
total = sum(e - s for s, e in ivs)
print(f"union busy {union / 1e6:.1f} ms of {(t1 - t0) / 1e6:.1f} ms window; sum of kernel time {total / 1e6:.1f} ms "
      f"(overlap factor {total / max(union, 1):.2f})")
