"""Split a rocprofv3 kernel trace of one bench step into phases (before the first
prefill kernel / prefill / decode / after the last kernel) and report the GPU-idle
time of each, from the compressed trace tools/gpu/prof_bench.sh keeps."""
import argparse
import csv
import gzip
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace", default="gpurun_out/kernel_trace.csv.gz", nargs="?")
ap.add_argument("--window-json", default="gpurun_out/prof_bench.json")
ap.add_argument("--gaps", type=float, default=2.0, help="list idle gaps longer than this (ms)")
a = ap.parse_args()
op = gzip.open if a.trace.endswith(".gz") else open
rows = list(csv.DictReader(op(a.trace, "rt")))
t0, t1 = json.load(open(a.window_json))["detail"]["timed_monotonic_ns"]
rows = [r for r in rows if int(r["Start_Timestamp"]) >= t0 and int(r["End_Timestamp"]) <= t1]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
S = lambda r: int(r["Start_Timestamp"])  # noqa: E731
E = lambda r: int(r["End_Timestamp"])  # noqa: E731
pre = [r for r in rows if "attn_prefill" in r["Kernel_Name"]]
dec = [r for r in rows if "attn_decode" in r["Kernel_Name"]]
b = {"prefill_start": S(pre[0]), "prefill_end": E(pre[-1]), "decode_start": S(dec[0]), "decode_end": E(dec[-1])}
ms = lambda ns: round(ns / 1e6, 1)  # noqa: E731
print(json.dumps({"window_ms": ms(t1 - t0), "first_kernel_ms": ms(S(rows[0]) - t0),
                  "prefill_phase_ms": ms(b["prefill_end"] - b["prefill_start"]),
                  "decode_phase_ms": ms(b["decode_end"] - b["decode_start"]),
                  "after_last_kernel_ms": ms(t1 - E(rows[-1]))}))
idle = {"start": 0, "prefill": 0, "between": 0, "decode": 0, "tail": 0}
end = E(rows[0])
for r in rows[1:]:
    s = S(r)
    if s > end:
        g = s - end
        k = ("start" if s <= b["prefill_start"] else "prefill" if s <= b["prefill_end"] else
             "between" if s <= b["decode_start"] else "decode" if s <= b["decode_end"] else "tail")
        idle[k] += g
        if g > a.gaps * 1e6:
            print(f"  idle {g / 1e6:8.2f} ms at +{(end - t0) / 1e6:8.1f} ms before {r['Kernel_Name'][:60]}")
    end = max(end, E(r))
print(json.dumps({"idle_ms": {k: ms(v) for k, v in idle.items()}}))
