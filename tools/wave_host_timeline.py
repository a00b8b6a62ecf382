"""Per-wave host timeline from a rocprofv3 --kernel-trace --marker-trace run of bench.py:
for each injected wave, ms from ``inject[w]`` to the first of each pipeline marker
(detected, collect, match.batch, scan, prompts, prefill) and to the first
attn_prefill kernel; i.e. where the detection -> first-prefill gap goes. For waves
after the first, also the previous wave's end relative to the inject (negative ms):
its last decode kernel, the engine's finish hook and the bench's hand-off mark."""
import argparse
import csv
import json
import re


def rows(path):
    with open(path) as f:
        yield from csv.DictReader(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--markers", required=True)
    ap.add_argument("--kernels", required=True)
    a = ap.parse_args()
    marks = []
    for r in rows(a.markers):
        name = r.get("Function") or r.get("Message") or r.get("Name") or r.get("Operation") or ""
        try:
            marks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
        except (KeyError, ValueError):
            continue
    marks.sort()
    prefill_k, decode_end = [], []
    for r in rows(a.kernels):
        if "attn_prefill" in r["Kernel_Name"]:
            prefill_k.append(int(r["Start_Timestamp"]))
        elif "attn_decode" in r["Kernel_Name"]:
            decode_end.append(int(r["End_Timestamp"]))
    prefill_k.sort()
    decode_end.sort()
    injects = [(s, e, n) for s, e, n in marks if re.match(r"inject\[\d+\]", n)]
    names = ("detected", "collect", "match.batch", "scan", "prompts", "prefill[")
    for i, (s0, e0, n0) in enumerate(injects):
        nxt = injects[i + 1][0] if i + 1 < len(injects) else float("inf")
        out = {"wave": n0, "inject_ms": round((e0 - s0) / 1e6, 2)}
        for nm in names:
            first = next(((s, e) for s, e, n in marks if s >= s0 and s < nxt and n.startswith(nm)), None)
            if first:
                out[nm.rstrip("[") + "_start_ms"] = round((first[0] - s0) / 1e6, 2)
                out[nm.rstrip("[") + "_end_ms"] = round((first[1] - s0) / 1e6, 2)
        # the previous wave's end: its last decode kernel -> engine finish hook ->
        # bench hand-off (every explanation counted) -> this inject (ms before inject)
        last_dec = max((t for t in decode_end if t < s0), default=None)
        if last_dec is not None and i > 0:
            out["prev_last_decode_ms"] = round((last_dec - s0) / 1e6, 2)
            fin = [(s, e) for s, e, n in marks if last_dec - 50_000_000 <= s < s0 and n.startswith("finish[")]
            if fin:
                out["prev_finish_start_ms"] = round((fin[-1][0] - s0) / 1e6, 2)
                out["prev_finish_end_ms"] = round((fin[-1][1] - s0) / 1e6, 2)
            ho = [s for s, e, n in marks if last_dec <= s <= s0 and n.startswith("handoff[")]
            if ho:
                out["prev_handoff_ms"] = round((ho[-1] - s0) / 1e6, 2)
        k = next((t for t in prefill_k if s0 <= t < nxt), None)
        if k:
            out["first_prefill_kernel_ms"] = round((k - s0) / 1e6, 2)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
