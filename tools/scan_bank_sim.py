"""Host model of ac_scan's LDS bank conflicts (csrc/kernels/scan.hip, v2 fast walk).

Replays the kernel's lane -> stream mapping on the synthetic config-2 corpus: lane t of
workgroup B walks stream B*1024+t, a contiguous range of L bytes, one byte per step,
all lanes in lockstep. For each half-wave (the 32-lane group a ds_read_b32/u16 is
serviced in, MI355X_MICROARCH.md §LDS) and step, the LDS-array cycles are the largest
number of DISTINCT dwords that fall into one of the 32 banks (identical dwords
broadcast). Extra cycles = that - 1, per group; the per-instruction figure (two groups)
is what SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS measures.

Layouts compared (all hold the 256 hot states x 256 byte values, uint16 entries):
  * ``row258``   - the round-5 image: [byte][state], 258-entry rows (bank = b + s/2);
  * ``perm``     - per-byte row offsets from a profile: ``rowoff[b]`` is chosen so the
                   most frequent (byte, state) pairs land on distinct banks;
  * ``private``  - lane-private banks (the lower bound a layout can reach: 0).
Usage: python tools/scan_bank_sim.py [--groups 48] [--doc-kb 256]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.ops import patterns  # noqa: E402
from operator_amd.patterns.compiler import compile_patterns  # noqa: E402
from operator_amd.patterns.synth import LogFactory, synthetic_library  # noqa: E402


def walk(tab, cls, text, starts, L):
    """States BEFORE each step for lanes starting at `starts` (root after a 64-B look-back)."""
    n = len(starts)
    s = np.zeros(n, dtype=np.int64)
    for j in range(-64, 0):
        p = starts + j
        b = np.where(p >= 0, text[np.clip(p, 0, None)], 0)
        s = tab[s, cls[b]].astype(np.int64) & 0x7FFF
    S = np.empty((L, n), dtype=np.int32)
    B = np.empty((L, n), dtype=np.int32)
    E = np.empty((L, n), dtype=np.int32)
    for j in range(L):
        b = text[starts + j].astype(np.int64)
        S[j] = s
        B[j] = b
        e = tab[s, cls[b]].astype(np.int64)
        E[j] = e
        s = e & 0x7FFF
    return S, B, E


def cycles(dw, bank):
    """dw, bank: [steps, 32] -> per-step LDS cycles (max distinct dwords per bank)."""
    steps = dw.shape[0]
    out = np.empty(steps, dtype=np.int32)
    for j in range(steps):
        u = np.unique(dw[j])
        bk = bank(u)
        out[j] = np.bincount(bk, minlength=32).max()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=48)
    ap.add_argument("--docs", type=int, default=64)
    ap.add_argument("--doc-kb", type=int, default=256)
    ap.add_argument("--L", type=int, default=4544, help="bytes per stream (config 2: 1.19 GB / 262144)")
    ap.add_argument("--steps", type=int, default=1024)
    a = ap.parse_args()
    ps = synthetic_library(1000)
    cp = compile_patterns(ps)
    d = cp.dfa
    S, l2c = int(d["num_states"]), int(d["log2_classes"])
    docs, _ = LogFactory(n_patterns=1000, seed=1).batch(a.docs, a.doc_kb * 1024, n_failures=3)
    text = np.frombuffer(b"\0".join(docs), dtype=np.uint8)
    r = patterns().reorder_dfa(d["table"], d["out_off"], d["out_ids"], l2c, S, d["cls_map"],
                               text[: 1 << 20].tobytes(), 256)
    tab = np.frombuffer(r["table"], dtype=np.uint16).reshape(S, 1 << l2c)
    cls = np.frombuffer(d["cls_map"], dtype=np.uint8).astype(np.int64)
    rng = np.random.default_rng(0)
    lanes = []
    for _ in range(a.groups):
        g0 = int(rng.integers(64, len(text) - 33 * a.L))
        lanes.append(g0 + a.L * np.arange(32))
    starts = np.concatenate(lanes)
    St, Bt, Et = walk(tab, cls, text, starts, a.steps)
    hot = St < 256
    res = {"states": S, "classes": 1 << l2c, "hot_fraction": float(hot.mean()),
           "root_fraction": float((St == 0).mean())}
    # fast-walk re-walk triggers per 64-byte chunk: a cold state or an output entry
    ch = a.steps // 64
    cold = (~hot[: ch * 64]).reshape(ch, 64, -1).any(1)
    outs = ((Et[: ch * 64] & 0x8000) != 0).reshape(ch, 64, -1).sum(1)
    lane_flag = cold | (outs > 0)
    wave = lane_flag.reshape(ch, a.groups, 32).any(2)
    res.update({"lane_chunk_cold": float(cold.mean()), "lane_chunk_out": float((outs > 0).mean()),
                "lane_chunk_out_ge2": float((outs > 1).mean()), "lane_chunk_flag": float(lane_flag.mean()),
                "group32_chunk_flag": float(wave.mean()),
                "group32_chunk_cold": float(cold.reshape(ch, a.groups, 32).any(2).mean()),
                "outs_per_flagged_lane_chunk": float(outs.sum() / max(1, (outs > 0).sum()))})
    st = St & 0xFF

    # profile of (byte, state) pair frequencies for the perm layout
    freq = np.zeros((256, 256), dtype=np.int64)
    np.add.at(freq, (Bt.ravel(), st.ravel()), 1)

    def run(name, dword_of):
        tot = 0
        n = 0
        for g in range(a.groups):
            sl = slice(32 * g, 32 * g + 32)
            dw = dword_of(Bt[:, sl].astype(np.int64), st[:, sl].astype(np.int64), np.arange(32)[None, :])
            c = cycles(dw, lambda u: u % 32)
            tot += int((c - 1).sum())
            n += c.size
        res[name + "_extra_per_instr"] = round(2.0 * tot / n, 3)

    run("row258", lambda b, s, l: (b * 258 + s) >> 1)
    run("row256", lambda b, s, l: (b * 256 + s) >> 1)
    # XOR the state column with the byte: bank = (b*129 + ((s ^ b*k)>>1))
    run("xor_b", lambda b, s, l: (b * 258 + (s ^ (b & 0xFF))) >> 1)
    # rows for the same byte spread; column rotated by 2*b
    run("rot2b", lambda b, s, l: (b * 258 + ((s + 2 * b * 17) & 0xFF)) >> 1)
    # greedy per-byte row bank: order bytes by frequency, give each the bank offset that
    # minimises the collision mass with the bytes placed before it
    pb = freq.sum(1)
    order = np.argsort(-pb)
    load = np.zeros(32)
    rowbank = np.zeros(256, dtype=np.int64)
    for b in order:
        # mass of this byte's row per bank for each candidate offset o
        colmass = np.zeros(32)
        np.add.at(colmass, (np.arange(256) >> 1) % 32, freq[b])
        best, bo = None, 0
        for o in range(32):
            m = np.roll(colmass, o)
            cost = float((m * load).sum())
            if best is None or cost < best:
                best, bo = cost, o
        rowbank[b] = bo
        load += np.roll(colmass, bo)
    rb = rowbank
    run("perm", lambda b, s, l: b * 256 + ((rb[b] + (s >> 1)) % 32) + 32 * ((s >> 1) // 32))
    cl = cls
    fold = np.arange(256); fold[65:91] += 32
    run("row_fold", lambda b, s, l: (fold[b] * 258 + s) >> 1)
    run("row_class", lambda b, s, l: (cl[b] * 258 + s) >> 1)
    res["private"] = 0.0
    print(json.dumps(res))


if __name__ == "__main__":
    main()
