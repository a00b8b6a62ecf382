"""Per-wave GPU timeline of a multi-step bench kernel trace: for each wave the
prefill span, decode span and the GPU-idle gap before its first prefill kernel
(the host pipeline turning a new wave of failures into the first prompt batch)."""
import argparse
import csv
import gzip
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--window-json", required=True)
a = ap.parse_args()
rows = list(csv.DictReader(gzip.open(a.trace, "rt") if a.trace.endswith(".gz") else open(a.trace)))
line = [x for x in open(a.window_json) if x.startswith("{") and '"metric"' in x][-1]   # bench.py's JSON line
t0, t1 = json.loads(line)["detail"]["timed_monotonic_ns"]
S = lambda r: int(r["Start_Timestamp"])  # noqa: E731
E = lambda r: int(r["End_Timestamp"])  # noqa: E731
ks = sorted([r for r in rows if t0 <= S(r) <= t1], key=S)
# a wave starts at an attn_prefill kernel that follows an attn_decode kernel (or the window start)
waves, cur, last_kind = [], None, None
for r in ks:
    n = r["Kernel_Name"]
    kind = "p" if "attn_prefill" in n else "d" if "attn_decode" in n else None
    if kind == "p" and last_kind != "p" and (last_kind is None or last_kind == "d"):
        cur = {"first_prefill": S(r), "prefill_end": E(r), "decode_start": None, "decode_end": None}
        waves.append(cur)
    if cur is not None and kind == "p":
        cur["prefill_end"] = E(r)
    if cur is not None and kind == "d":
        cur["decode_start"] = cur["decode_start"] or S(r)
        cur["decode_end"] = E(r)
    if kind:
        last_kind = kind
prev_end = t0
for i, w in enumerate(waves):
    print(json.dumps({"wave": i, "gap_before_prefill_ms": round((w["first_prefill"] - prev_end) / 1e6, 1),
                      "prefill_ms": round((w["prefill_end"] - w["first_prefill"]) / 1e6, 1),
                      "decode_ms": round(((w["decode_end"] or 0) - (w["decode_start"] or 0)) / 1e6, 1)}))
    prev_end = w["decode_end"] or prev_end
print(json.dumps({"window_ms": round((t1 - t0) / 1e6, 1), "after_last_decode_ms": round((t1 - prev_end) / 1e6, 1)}))
