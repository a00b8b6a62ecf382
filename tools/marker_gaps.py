"""roctx ranges + GPU-idle gaps of a rocprofv3 kernel/marker trace, cut to the
bench's timed window (tools/gpu/prof_markers.sh writes the inputs)."""
import argparse
import csv
import gzip
import json

ap = argparse.ArgumentParser()
ap.add_argument("--dir", default="gpurun_out/profm")
ap.add_argument("--window-json", default="gpurun_out/profm_bench.json")
ap.add_argument("--ranges", type=int, default=30)
ap.add_argument("--gap-ms", type=float, default=1.5)
a = ap.parse_args()
k = list(csv.DictReader(gzip.open(f"{a.dir}/run_kernel_trace.csv.gz", "rt")))
m = list(csv.DictReader(gzip.open(f"{a.dir}/run_marker_api_trace.csv.gz", "rt")))
t0, t1 = json.load(open(a.window_json))["detail"]["timed_monotonic_ns"]
S = lambda r: int(r["Start_Timestamp"])  # noqa: E731
E = lambda r: int(r["End_Timestamp"])  # noqa: E731
ms = sorted([r for r in m if t0 <= S(r) <= t1], key=S)
for r in ms[:a.ranges]:
    print(f"{(S(r) - t0) / 1e6:9.1f} {(E(r) - S(r)) / 1e6:8.1f} ms  {r['Function']}")
ks = sorted([r for r in k if t0 <= S(r) <= t1], key=S)
end = E(ks[0])
idle = 0
print(f"first kernel at +{(S(ks[0]) - t0) / 1e6:.1f} ms")
for r in ks[1:]:
    if S(r) - end > 0:
        idle += S(r) - end
        if S(r) - end > a.gap_ms * 1e6:
            print(f"gap {(S(r) - end) / 1e6:7.2f} ms at +{(end - t0) / 1e6:8.1f} before {r['Kernel_Name'][:50]}")
    end = max(end, E(r))
print(json.dumps({"window_ms": round((t1 - t0) / 1e6, 1), "idle_between_kernels_ms": round(idle / 1e6, 1),
                  "after_last_kernel_ms": round((t1 - end) / 1e6, 1)}))
