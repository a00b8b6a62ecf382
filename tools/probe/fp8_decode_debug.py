"""Localise fp8-KV decode attention errors: fp8 kernel vs the bf16 kernel over the
dequantised cache (identical math up to fp32 summation order)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from operator_amd import ops  # noqa: E402
from operator_amd.ops import reference as ref  # noqa: E402

dev = "cuda"
torch.manual_seed(14)
for (Hq, Hkv, lens, ks, vs) in [(8, 8, [16], 1.0, 1.0), (8, 8, [64], 1.0, 1.0), (32, 8, [70, 300], 1.0, 1.0),
                               (32, 8, [70, 300], 0.5, 2.0)]:
    P, D = 64, 128
    B = len(lens)
    maxp = (max(lens) + P - 1) // P + 1
    pages = B * maxp + 2
    kf, vf = torch.randn(pages, Hkv, P, D, device=dev), torch.randn(pages, Hkv, P, D, device=dev)
    kc, vc = ref.kv_store(kf, torch.float8_e4m3fn, ks), ref.kv_store(vf, torch.float8_e4m3fn, vs)
    kb, vb = (kc.float() * ks).to(torch.bfloat16), (vc.float() * vs).to(torch.bfloat16)
    bt = torch.arange(B * maxp, device=dev).reshape(B, maxp).int()
    sl = torch.tensor(lens, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq, D, device=dev).to(torch.bfloat16)
    sc = 1 / math.sqrt(D)
    o8 = ops.attn_decode(q, kc, vc, bt, sl, sc, 1, k_scale=ks, v_scale=vs).float()
    ob = ops.attn_decode(q, kb, vb, bt, sl, sc, 1).float()
    err = (o8 - ob).abs()
    print(f"Hq={Hq} Hkv={Hkv} lens={lens} ks={ks} vs={vs}: max err {err.max():.4f}; per row "
          f"{[round(float(e), 4) for e in err.amax((1, 2))]}; per head(row0) "
          f"{[round(float(e), 3) for e in err[0].amax(1)][:8]}; dims with err>0.05 (row0 head0): "
          f"{(err[0, 0] > 0.05).nonzero().flatten().tolist()[:24]}", flush=True)
    # V only: make K all zero -> uniform attention -> output = mean of V rows
    kz = torch.zeros_like(kc)
    o8v = ops.attn_decode(q, kz, vc, bt, sl, sc, 1, k_scale=ks, v_scale=vs).float()
    obv = ops.attn_decode(q, torch.zeros_like(kb), vb, bt, sl, sc, 1).float()
    print(f"   V-only max err {(o8v - obv).abs().max():.4f}", flush=True)
