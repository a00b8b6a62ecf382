"""Where the GPU sits idle inside the flagship bench's timed window.

Reads a rocprofv3 --kernel-trace CSV of ``bench.py`` and the bench's JSON line (for
the timed window), merges the kernel intervals into busy spans and classifies every
idle gap by the wave phase around it (the waves are cut as in tools/wave_gaps.py):

  wave_boundary     previous wave's last decode kernel -> this wave's first prefill kernel
  prefill_internal  gaps inside the prefill span (batch hand-offs are the > 50 us ones)
  prefill_to_decode last prefill kernel -> first decode kernel
  decode_internal   gaps inside the decode span (window hand-offs are the > 50 us ones)
  tail              last decode kernel -> end of the timed window

Prints one JSON line per wave, one summary line (ms per wave per class) and the kernel
pairs around the largest idle gaps (which hand-off they are).
"""
import argparse
import csv
import gzip
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-json", required=True)
    ap.add_argument("--big-us", type=float, default=50.0, help="gaps above this are host hand-offs")
    ap.add_argument("--context", type=int, default=0, help="print the kernels around the N largest decode gaps")
    a = ap.parse_args()
    f = gzip.open(a.trace, "rt") if a.trace.endswith(".gz") else open(a.trace)
    line = [x for x in open(a.window_json) if x.startswith("{") and '"metric"' in x][-1]
    t0, t1 = json.loads(line)["detail"]["timed_monotonic_ns"]
    ks = []
    for r in csv.DictReader(f):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0 or s > t1:
            continue
        n = r["Kernel_Name"]
        kind = "p" if "attn_prefill" in n else "d" if "attn_decode" in n else ""
        ks.append((s, e, kind, n.split("(")[0][:60]))
    ks.sort()
    # waves: a wave starts at an attn_prefill kernel that follows an attn_decode kernel
    waves, cur, last = [], None, None
    for s, e, kind, _ in ks:
        if kind == "p" and last != "p":
            cur = {"p0": s, "p1": e, "d0": None, "d1": None}
            waves.append(cur)
        if cur is not None and kind == "p":
            cur["p1"] = e
        if cur is not None and kind == "d":
            cur["d0"] = cur["d0"] or s
            cur["d1"] = e
        if kind:
            last = kind
    # busy spans (union of kernel intervals) and the idle gaps between them
    gaps, end, prev = [], t0, "window start"
    pairs = {}   # (kernel before, kernel after) of the big gaps -> [count, ms]
    for s, e, _, name in ks:
        if s > end:
            gaps.append((end, s))
            if (s - end) / 1e3 > a.big_us:
                k = (prev, name)
                pairs.setdefault(k, [0, 0.0])
                pairs[k][0] += 1
                pairs[k][1] += (s - end) / 1e6
        if e >= end:
            prev = name
        end = max(end, e)
    if t1 > end:
        gaps.append((end, t1))

    def cls(g0, g1):
        for i, w in enumerate(waves):
            prev_end = waves[i - 1]["d1"] if i else t0
            if prev_end <= g0 and g1 <= w["p0"]:
                return i, "wave_boundary"
            if w["p0"] <= g0 and g1 <= w["p1"]:
                return i, "prefill_internal"
            if w["d0"] and w["p1"] <= g0 and g1 <= w["d0"]:
                return i, "prefill_to_decode"
            if w["d0"] and w["d0"] <= g0 and g1 <= w["d1"]:
                return i, "decode_internal"
        return len(waves) - 1, "tail"

    per = [dict(ms={}, big={}, n_big={}) for _ in waves] or [dict(ms={}, big={}, n_big={})]
    for g0, g1 in gaps:
        i, c = cls(g0, g1)
        d = (g1 - g0) / 1e6
        p = per[max(i, 0)]
        p["ms"][c] = p["ms"].get(c, 0.0) + d
        if d * 1e3 > a.big_us:
            p["big"][c] = p["big"].get(c, 0.0) + d
            p["n_big"][c] = p["n_big"].get(c, 0) + 1
    for i, (w, p) in enumerate(zip(waves, per)):
        span = ((w["d1"] or w["p1"]) - w["p0"]) / 1e6
        print(json.dumps({"wave": i, "prefill_span_ms": round((w["p1"] - w["p0"]) / 1e6, 1),
                          "decode_span_ms": round(((w["d1"] or 0) - (w["d0"] or 0)) / 1e6, 1),
                          "span_ms": round(span, 1),
                          "idle_ms": {k: round(v, 2) for k, v in sorted(p["ms"].items())},
                          "idle_big_ms": {k: round(v, 2) for k, v in sorted(p["big"].items())},
                          "n_big": p["n_big"]}))
    tot = {}
    for p in per:
        for k, v in p["ms"].items():
            tot[k] = tot.get(k, 0.0) + v
    nw = max(1, len(waves))
    print(json.dumps({"window_ms": round((t1 - t0) / 1e6, 1), "waves": len(waves),
                      "idle_ms_per_wave": {k: round(v / nw, 2) for k, v in sorted(tot.items())},
                      "idle_total_ms_per_wave": round(sum(tot.values()) / nw, 2),
                      "kernels": len(ks)}))
    if a.context:   # the kernels around the largest idle gaps inside decode spans
        big = []
        for i in range(1, len(ks)):
            g = ks[i][0] - max(x[1] for x in ks[max(0, i - 8):i])
            if g > a.big_us * 1e3 and any(w["d0"] and w["d0"] <= ks[i][0] <= w["d1"] for w in waves):
                big.append((g, i))
        for g, i in sorted(big, reverse=True)[:a.context]:
            t_ref = ks[i][0]
            print(json.dumps({"gap_us": round(g / 1e3, 1), "around": [
                [round((x[0] - t_ref) / 1e3, 1), round((x[1] - x[0]) / 1e3, 1), x[3][:48]] for x in ks[max(0, i - 4):i + 3]]}))
    top = sorted(pairs.items(), key=lambda kv: -kv[1][1])[:8]
    for (before, after), (n, ms) in top:
        print(json.dumps({"kernel_before_gap": before, "kernel_after_gap": after, "count": n, "ms": round(ms, 2)}))


if __name__ == "__main__":
    main()
