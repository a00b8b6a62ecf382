"""GPU idle at decode-window boundaries of a flagship kernel trace.

A decode window ends with the D2H copy of its sampled tokens (``__amd_rocclr_copyBuffer``)
and the next one starts with its first bookkeeping kernel. For every idle gap that
follows a copy kernel inside the timed window this prints the size distribution and,
for a few gaps of median size, the kernels around it (start offset us, duration us).

  python tools/window_gaps.py run_kernel_trace.csv --window-json fl.json [--examples 4]
"""
import argparse
import csv
import gzip
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-json", required=True)
    ap.add_argument("--examples", type=int, default=4)
    ap.add_argument("--min-us", type=float, default=20.0)
    a = ap.parse_args()
    f = gzip.open(a.trace, "rt") if a.trace.endswith(".gz") else open(a.trace)
    line = [x for x in open(a.window_json) if x.startswith("{") and '"metric"' in x][-1]
    t0, t1 = json.loads(line)["detail"]["timed_monotonic_ns"]
    ks = []
    for r in csv.DictReader(f):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s <= t1:
            ks.append((s, e, r["Kernel_Name"].split("(")[0][:56]))
    ks.sort()
    by_next: dict[str, list] = {}
    examples = []
    end = 0
    for i in range(1, len(ks)):
        end = max(end, ks[i - 1][1])
        g = (ks[i][0] - end) / 1e3
        if g < a.min_us or "copyBuffer" not in ks[i - 1][2]:
            continue
        by_next.setdefault(ks[i][2], []).append(g)
        examples.append((g, i))
    for name, gs in sorted(by_next.items(), key=lambda kv: -sum(kv[1])):
        gs.sort()
        print(json.dumps({"after_copy": name, "count": len(gs), "total_ms": round(sum(gs) / 1e3, 2),
                          "p10_us": round(gs[len(gs) // 10], 1), "median_us": round(statistics.median(gs), 1),
                          "p90_us": round(gs[9 * len(gs) // 10], 1)}))
    examples.sort()
    mid = len(examples) // 2
    for g, i in examples[max(0, mid - a.examples // 2):mid + (a.examples + 1) // 2]:
        ref = ks[i][0]
        print(json.dumps({"gap_us": round(g, 1), "around": [
            [round((x[0] - ref) / 1e3, 1), round((x[1] - x[0]) / 1e3, 1), x[2][:40]] for x in ks[max(0, i - 5):i + 4]]}))


if __name__ == "__main__":
    main()
