"""Aggregate a rocprofv3 kernel-trace CSV by (kernel, grid, workgroup): calls, total and
median duration. Used on the GPU box to shrink a multi-hundred-MB trace to a summary
before it is copied back (``--delete`` removes the trace afterwards)."""
import argparse
import collections
import csv
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", required=True)
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--delete", action="store_true")
    a = ap.parse_args()
    d = collections.defaultdict(list)
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            key = (r["Kernel_Name"][:110], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
            d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in d.values())
    with open(a.out, "w") as o:
        o.write(f"# total kernel time {tot / 1e6:.2f} ms over {sum(len(v) for v in d.values())} dispatches\n")
        o.write("# total_ms calls median_us pct | kernel grid(x,y,z) wg\n")
        for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
            v.sort()
            o.write(f"{sum(v) / 1e6:10.2f} {len(v):7d} {v[len(v) // 2] / 1e3:9.1f} {100 * sum(v) / tot:5.1f}% | "
                    f"{k[0]} grid=({k[1]},{k[2]},{k[3]}) wg={k[4]}\n")
    if a.delete:
        os.remove(a.trace)


if __name__ == "__main__":
    main()
