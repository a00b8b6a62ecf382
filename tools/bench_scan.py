"""BASELINE config 2: PatternLibrary scan, ~1 GB of synthetic pod logs x 1000
patterns on one MI355X (ac_scan).

Arms (one JSON line each):
  * bfs      - DFA states in breadth-first order (the compile-time numbering)
  * profiled - states renumbered by visit count over the first MiB of text
               (MatchEngine.profile_bytes, csrc/patterns/patterns.cpp reorder_dfa)
Kernel-only time is the mean of ``--iters`` back-to-back ac_scan launches over
the packed text (HIP events); ``analyze_s`` is one full MatchEngine.analyze
(pack + H2D + scan + fixup + D2H + verify + score + results) of the same docs,
best of three after a first call (reported separately: it uploads the scoring tables).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.engine.match import MatchEngine  # noqa: E402
from operator_amd.ops import kernels  # noqa: E402
from operator_amd.patterns.synth import LogFactory, synthetic_library  # noqa: E402


def kernel_ms(eng, docs, iters):
    C = kernels()
    seg = eng.last_seg
    tot_pad = sum(((len(d) + 1 + seg - 1) // seg) * seg for d in docs)
    ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
    with torch.cuda.stream(eng._stream):
        for _ in range(2):
            eng._count.zero_()
            C.ac_scan(eng._text[:tot_pad], seg, eng.cls_map, eng.table, eng.log2c, eng.hot_states, eng.out_off,
                      eng.out_ids, eng._matches, eng._count, eng._seg_nl, eng.grid_blocks, eng.hot_table, eng.chain)
        ev0.record()
        for _ in range(iters):
            eng._count.zero_()
            C.ac_scan(eng._text[:tot_pad], seg, eng.cls_map, eng.table, eng.log2c, eng.hot_states, eng.out_off,
                      eng.out_ids, eng._matches, eng._count, eng._seg_nl, eng.grid_blocks, eng.hot_table, eng.chain)
        ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters, tot_pad, int(eng._count.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=4096)
    ap.add_argument("--doc-kb", type=int, default=256)
    ap.add_argument("--patterns", type=int, default=1000)
    ap.add_argument("--seg", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--arms", default="bfs,profiled")
    ap.add_argument("--pack-sweep", action="store_true")
    ap.add_argument("--kernel-only", action="store_true", help="print the kernel timing and skip analyze()")
    ap.add_argument("--pipe-sweep", default="0,128,256,400,640",
                    help="MatchEngine.PIPE_SUB_BYTES values (MB; 0 = one batch) timed after the main arm")
    a = ap.parse_args()
    ps = synthetic_library(a.patterns)
    t0 = time.perf_counter()
    docs, _ = LogFactory(n_patterns=a.patterns, seed=1).batch(a.docs, a.doc_kb * 1024, n_failures=3)
    gen_s = time.perf_counter() - t0
    total = sum(map(len, docs))
    ref = None
    for arm in a.arms.split(","):
        eng = MatchEngine(ps, device="cuda", seg_bytes=a.seg, profile_bytes=(1 << 20) if arm == "profiled" else 0)
        raw = eng.scan_gpu(docs)
        torch.cuda.synchronize()
        ms, tot_pad, cnt = kernel_ms(eng, docs, a.iters)
        key = sorted(map(tuple, raw.tolist()))
        same = None if ref is None else (key == ref)
        ref = ref or key
        probe_stats = None
        if os.environ.get("OAMD_SCAN_PROBE") in ("4", "5", "6", "7"):
            # per-wave {cycles, slow cycles, slow entries, cold wave-steps} (csrc/kernels/scan.hip)
            cap = eng._matches.shape[0]
            w = eng._matches[cap // 2: cap // 2 + 196608].cpu().view(torch.int32).numpy().view("uint32").reshape(-1, 12)
            w = w[w[:, 0] > 0].astype("float64")
            probe_stats = {"waves": int(w.shape[0]), "cycles_mean": round(float(w[:, 0].mean())),
                           "cycles_max": round(float(w[:, 0].max())), "slow_cycles_mean": round(float(w[:, 1].mean())),
                           "slow_cycles_max": round(float(w[:, 1].max())),
                           "slow_entries_mean": round(float(w[:, 2].mean()), 2), "slow_entries_max": int(w[:, 2].max()),
                           "cold_steps_mean": round(float(w[:, 3].mean()), 1),
                           "cycles_per_slow_entry": round(float(w[:, 1].sum() / max(1.0, w[:, 2].sum()))),
                           "emit_cycles_mean": round(float(w[:, 4].mean())), "emits_mean": round(float(w[:, 5].mean()), 2),
                           "cycles_per_emit": round(float(w[:, 4].sum() / max(1.0, w[:, 5].sum()))),
                           "subchunks_mean": round(float(w[:, 6].mean()), 2),
                           "subchunk_walk_cycles_mean": round(float(w[:, 7].mean())),
                           "cold_step_cycles_mean": round(float(w[:, 8].mean()))}
        if a.kernel_only:
            print(json.dumps({"probe_stats": probe_stats,"bench": "scan_kernel", "arm": arm, "probe": os.environ.get("OAMD_SCAN_PROBE", "0"),
                              "padded_bytes": tot_pad, "kernel_ms": round(ms, 3),
                              "kernel_GBps": round(tot_pad / ms / 1e6, 1), "raw_matches": cnt,
                              "same_matches_as_first_arm": same}), flush=True)
            del eng
            continue
        t1 = time.perf_counter()
        res = eng.analyze(docs)
        t2 = time.perf_counter()
        first_s = t2 - t1
        warm = []
        for _ in range(3):   # steady state: best of three more calls (the first loads the score tables)
            del res          # the previous call's result objects are freed outside the timed call
            u1 = time.perf_counter()
            res = eng.analyze(docs)
            warm.append(time.perf_counter() - u1)
        t1, t2 = 0.0, min(warm)
        stage = {"analyze_" + k: round(v, 4) for k, v in eng.last_timing.items()}
        lz, mat = [], []
        for _ in range(3):   # lazy: events + context windows; then materialize every result object
            lres = None
            u1 = time.perf_counter()
            lres = eng.analyze(docs, lazy=True)
            u2 = time.perf_counter()
            list(lres)
            lz.append(u2 - u1)
            mat.append(time.perf_counter() - u2)
        stage["analyze_lazy_s"] = round(min(lz), 4)
        stage["lazy_materialize_all_s"] = round(min(mat), 4)
        for name, fn in (("scan_gpu", lambda: eng.scan_gpu(docs)), ("events", lambda: eng.events(docs))):
            best = 1e9
            for _ in range(3):
                u1 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - u1)
            stage[name + "_s"] = round(best, 4)
        if a.pack_sweep:   # host pack / H2D pipelining: chunk size x packing threads, best of 3
            for chunk_mb in (64, 128, 256, 4096):
                for th in (4, 8, 16):
                    eng.PACK_CHUNK, eng.pack_threads = chunk_mb << 20, th
                    best = 1e9
                    for _ in range(3):
                        u1 = time.perf_counter()
                        eng.analyze(docs)
                        best = min(best, time.perf_counter() - u1)
                    print(json.dumps({"bench": "scan_pack", "chunk_mb": chunk_mb, "threads": th,
                                      "analyze_s": round(best, 4)}), flush=True)
        pipe = {}
        sub0 = eng.PIPE_SUB_BYTES
        sweep = [int(x) for x in a.pipe_sweep.split(",") if x]
        for _ in range(5):   # round-robin over the settings: host-state drift hits every one alike
            for mb in sweep:
                eng.PIPE_SUB_BYTES = mb << 20
                r = None
                u1 = time.perf_counter()
                r = eng.analyze(docs)
                dt = time.perf_counter() - u1
                cur = pipe.setdefault(str(mb), {"analyze_s": 1e9})
                if dt < cur["analyze_s"]:
                    pipe[str(mb)] = {"analyze_s": round(dt, 4),
                                     "timing": {k: round(v, 4) for k, v in eng.last_timing.items()}}
                del r
        eng.PIPE_SUB_BYTES = sub0
        print(json.dumps({"bench": "scan", "arm": arm, "bytes": total, "padded_bytes": tot_pad,
                          "patterns": a.patterns, "states": eng.dfa_states, "hot_states": eng.hot_states,
                          "hot_coverage": eng.hot_coverage, "kernel_ms": round(ms, 3),
                          "kernel_GBps": round(tot_pad / ms / 1e6, 1), "raw_matches": cnt,
                          "same_matches_as_first_arm": same, "analyze_s": round(t2 - t1, 4),
                          "analyze_first_call_s": round(first_s, 3), "analyze_GBps": round(total / (t2 - t1) / 1e9, 1),
                          "analyses_per_s": round(len(res) / (t2 - t1), 1), "gen_s": round(gen_s, 1),
                          "stages_best_of_3": stage, "pipe_sub_mb_sweep": pipe}), flush=True)
        del eng


if __name__ == "__main__":
    main()
