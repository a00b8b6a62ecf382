"""Numerics of every gfx950 HIP kernel against the plain-PyTorch fp32 reference."""
import math

import pytest
import torch

from operator_amd import ops
from operator_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(*shape, dtype=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


def test_native_module_is_loaded():
    C = ops.kernels()
    assert C.ARCH == "gfx950"
    maps = open("/proc/self/maps").read()
    assert "_C.cpython" in maps
    hip_libs = {l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}
    assert len(hip_libs) == 1, f"two HIP runtimes mapped: {hip_libs}"


@pytest.mark.parametrize("rows,hidden", [(1, 4096), (7, 4096), (64, 8192), (3, 128)])
@pytest.mark.parametrize("fused", [False, True])
def test_rmsnorm(rows, hidden, fused):
    torch.manual_seed(0)
    x = _rand(rows, hidden)
    w = _rand(hidden) * 0.5 + 1
    r = _rand(rows, hidden) if fused else None
    r_ref = r.clone() if fused else None
    y = ops.rmsnorm(x, w, 1e-5, residual=r)
    y_ref, nr = ref.rmsnorm(x.cpu(), w.cpu(), 1e-5, r_ref.cpu() if fused else None)
    torch.testing.assert_close(y.cpu().float(), y_ref.float(), atol=2e-2, rtol=2e-2)
    if fused:
        torch.testing.assert_close(r.cpu().float(), nr.float(), atol=0, rtol=0)


def test_silu_mul():
    gu = _rand(37, 2 * 1408)
    out = ops.silu_mul(gu)
    torch.testing.assert_close(out.cpu().float(), ref.silu_mul(gu.cpu()).float(), atol=2e-2, rtol=2e-2)


def test_embedding():
    table = _rand(1000, 512)
    ids = torch.randint(0, 1000, (33,), device=DEV)
    torch.testing.assert_close(ops.embedding(ids, table).cpu(), table.cpu()[ids.cpu()])


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (16, 16)])
def test_rope_kv_and_cache(Hq, Hkv):
    torch.manual_seed(1)
    T, D, P, pages = 19, 128, 16, 8
    cos, sin = ref.rope_tables(4096, D, 500000.0, device=DEV)
    qkv = _rand(T, (Hq + 2 * Hkv) * D)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    kc = torch.zeros(pages, Hkv, P, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    slots = torch.randperm(pages * P, device=DEV)[:T]
    slots[3] = -1
    q, k, v = ops.rope_kv(qkv, pos, cos, sin, Hq, Hkv, kc, vc, slots)
    kc_r, vc_r = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q_r, k_r, v_r = ref.rope_kv(qkv.cpu(), pos.cpu(), cos.cpu(), sin.cpu(), Hq, Hkv, kc_r, vc_r, slots.cpu())
    torch.testing.assert_close(q.cpu().float(), q_r.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(k.cpu().float(), k_r.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(v.cpu(), v_r)
    torch.testing.assert_close(kc.cpu().float(), kc_r.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(vc.cpu(), vc_r)


@pytest.mark.parametrize("lens", [[1], [17, 64, 130], [300, 5, 64]])
@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 8), (16, 2), (8, 4), (64, 8), (24, 8), (28, 4), (10, 2), (12, 2)])
@pytest.mark.parametrize("variant", [3, 2, 1, 4])
def test_attn_prefill(lens, Hq, Hkv, variant):
    if variant == 2 and Hq // Hkv not in (1, 2, 4, 8):
        pytest.skip("v2 takes GQA groups 1, 2, 4, 8 only")
    if variant == 4 and Hq // Hkv > 4:
        pytest.skip("v4 (4-wave workgroups) takes GQA groups <= 4")
    torch.manual_seed(2)
    T, D = sum(lens), 128
    q, k, v = _rand(T, Hq, D), _rand(T, Hkv, D), _rand(T, Hkv, D)
    scale = 1 / math.sqrt(D)
    cu = [0]
    for L in lens:
        cu.append(cu[-1] + L)
    ws, wq = ops.prefill_work_list(lens, ops.prefill_block_q(Hq, Hkv, variant))
    it = lambda x: torch.tensor(x, dtype=torch.int32, device=DEV)  # noqa: E731
    o = ops.attn_prefill(q, k, v, lens, scale, work=(it(cu), it(ws), it(wq), variant))
    o_r = ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), cu, scale)
    torch.testing.assert_close(o.cpu().float(), o_r.float(), atol=2e-2, rtol=3e-2)


@pytest.mark.parametrize("variant", [None, 3, 4])
def test_attn_prefill_large_scores(variant):
    """Spike one key so the running max jumps mid-sequence (forces the rescale path; v3
    defers a rescale until the max rises by more than 2^8)."""
    torch.manual_seed(3)
    lens, Hq, Hkv, D = [256], 8, 8, 128
    q, k, v = _rand(256, Hq, D), _rand(256, Hkv, D), _rand(256, Hkv, D)
    k[200] = (q[220].float() * 6).to(torch.bfloat16)[: Hkv]
    work = None
    if variant is not None:
        ws, wq = ops.prefill_work_list(lens, ops.prefill_block_q(Hq, Hkv, variant))
        it = lambda x: torch.tensor(x, dtype=torch.int32, device=DEV)  # noqa: E731
        work = (it([0, 256]), it(ws), it(wq), variant)
    o = ops.attn_prefill(q, k, v, lens, 1 / math.sqrt(D), work=work)
    o_r = ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), [0, 256], 1 / math.sqrt(D))
    torch.testing.assert_close(o.cpu().float(), o_r.float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("lens", [[1, 5, 300], [1000, 0, 2049], [4096]])
@pytest.mark.parametrize("Hq,Hkv,P", [(32, 8, 64), (8, 1, 16), (16, 16, 32), (24, 8, 64), (28, 4, 64), (5, 1, 16),
                                      (12, 2, 32)])
def test_attn_decode(lens, Hq, Hkv, P):
    torch.manual_seed(4)
    B, D = len(lens), 128
    maxp = (max(lens) + P - 1) // P + 1
    pages = B * maxp + 3
    kc, vc = _rand(pages, Hkv, P, D), _rand(pages, Hkv, P, D)
    bt = torch.randperm(pages, device=DEV)[: B * maxp].reshape(B, maxp).int()
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = _rand(B, Hq, D)
    scale = 1 / math.sqrt(D)
    o_r = ref.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), sl.cpu(), scale)
    # every split count is a valid schedule (1 = one workgroup walks the whole
    # context; more splits than chunks leaves empty workgroups), both variants
    for ns in sorted({1, 3, ops.decode_splits(max(lens), B, Hkv), 64}):
        for variant in (0, 2):
            o = ops.attn_decode(q, kc, vc, bt, sl, scale, ns, variant=variant)
            torch.testing.assert_close(o.cpu().float(), o_r.float(), atol=2e-2, rtol=3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sample(dtype):
    torch.manual_seed(5)
    B, V = 6, 5000
    logits = (torch.randn(B, V, device=DEV) * 3).to(dtype)
    temp = torch.tensor([0.0, 0.3, 1.0, 0.0, 0.7, 2.0], device=DEV)
    seeds = torch.arange(B, device=DEV) * 7 + 1
    pos = torch.arange(B, device=DEV) + 100
    tok = ops.sample(logits, temp, seeds, pos).cpu()
    tok_r = ref.sample(logits.cpu().float(), temp.cpu(), seeds.cpu(), pos.cpu())
    for r in range(B):
        if tok[r] != tok_r[r]:
            # accept fp32-vs-fp64 near-ties only
            x = logits[r].double().cpu()
            t = float(temp[r])
            if t > 0:
                x = x / t + ref.gumbel_noise_ref(int(seeds[r]), int(pos[r]), V)
            assert abs(float(x[tok[r]] - x[tok_r[r]])) < 1e-3
    assert tok[0] == int(torch.argmax(logits[0].float()))
    # deterministic replay
    assert torch.equal(ops.sample(logits, temp, seeds, pos).cpu(), tok)


def test_sample_distribution():
    """Token frequencies over many seeds match softmax(x / T) (the Gumbel-max identity),
    and a vocab-sized row never yields a token whose noise overflowed (u rounding to 1)."""
    torch.manual_seed(6)
    V, R, T = 32, 32768, 0.7
    row = torch.randn(V) * 1.5
    logits = row.expand(R, V).contiguous().to(DEV)
    temp = torch.full((R,), T, device=DEV)
    seeds = torch.arange(R, device=DEV) * 2654435761 % (1 << 40)
    pos = torch.full((R,), 17, device=DEV, dtype=torch.long)
    tok = ops.sample(logits, temp, seeds, pos).cpu()
    freq = torch.bincount(tok, minlength=V).double() / R
    p = torch.softmax(row.double() / T, 0)
    assert (freq - p).abs().max().item() < 4 * (p * (1 - p) / R).sqrt().max().item() + 1e-3
    # 128k-vocab rows with one dominant logit: the noise is bounded (max ~17 nats), so a
    # 40-nat lead always wins; an infinite noise value would hand the row to another column
    big = torch.zeros(64, 128256, device=DEV, dtype=torch.bfloat16)
    big[:, 1234] = 40.0
    out = ops.sample(big, torch.ones(64, device=DEV), torch.arange(64, device=DEV) + 99,
                     torch.arange(64, device=DEV)).cpu()
    assert (out == 1234).all()


@pytest.mark.parametrize("M", [64, 128, 192, 256])
@pytest.mark.parametrize("N,K", [(256, 512), (640, 2048), (128, 4096)])
def test_gemm_decode(M, N, K):
    torch.manual_seed(7)
    x = _rand(M, K)
    w = _rand(N, K) * 0.05
    ref_ = (x.float() @ w.float().t())
    for bm in (64, 128, 256):
        for bn in (64, 128):
            for S in (1, 2, 4, 5, 8):   # S = 5: uneven K slices (K / 64 steps not divisible)
                if M % bm or K // 64 < S or N % bn:
                    continue
                for ns in ((2, 3, 4) if bm <= 128 else (3, 4) if bm + bn <= 320 else (3,)):
                    y = ops.linear(x, w, splits=S, bn=bn, bm=bm, stages=ns)
                    torch.testing.assert_close(y.float(), ref_, atol=2e-2, rtol=2e-2)
    # default split choice and the hipBLASLt fallback shape agree too
    torch.testing.assert_close(ops.linear(x, w).float(), ref_, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(ops.linear(x[:M - 3].contiguous(), w).float(), ref_[:M - 3], atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 2, 5, 16, 17, 32])
@pytest.mark.parametrize("N,K", [(256, 512), (640, 2048), (128, 4096), (1024, 14336)])
def test_gemm_skinny(M, N, K):
    """Weight-streaming MFMA GEMM for M <= 32 decode buckets, every split count,
    plain / deferred (slabs) / reduced outputs, against an fp32 reference."""
    from operator_amd.ops import kernels

    torch.manual_seed(12)
    x = _rand(M, K)
    w = _rand(N, K) * 0.05
    ref_ = x.float() @ w.float().t()
    for S in (1, 2, 4, 8):
        if K % (128 * S):
            continue
        y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        p = torch.empty(S * M * N, dtype=torch.float32, device=DEV) if S > 1 else None
        kernels().gemm_skinny(x, w, y, p, S, False)
        torch.testing.assert_close(y.float(), ref_, atol=2e-2, rtol=2e-2)
        if S > 1:
            torch.testing.assert_close(p.view(S, M, N).sum(0), ref_, atol=1e-3, rtol=1e-3)
            d = ops.linear(x, w, splits=S, defer_reduce=True)
            torch.testing.assert_close(d.materialize().float(), ref_, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(ops.linear(x, w).float(), ref_, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [64, 128, 192, 256, 40, 1, 7, 16, 32])
def test_gate_up_silu_fused(M):
    torch.manual_seed(8)
    K, inter = 1024, 640
    x = _rand(M, K)
    g, u = _rand(inter, K) * 0.05, _rand(inter, K) * 0.05
    wgu = ops.interleave_gate_up(g, u)
    gf = (x.float() @ g.float().t()).to(torch.bfloat16)
    uf = (x.float() @ u.float().t()).to(torch.bfloat16)
    ref_ = ref.silu_mul(torch.cat([gf, uf], 1))
    got = ops.gate_up_silu(x, wgu, ops.GU_BLOCK)
    torch.testing.assert_close(got.float(), ref_.float(), atol=2e-2, rtol=2e-2)
    # the unfused path over the same interleaved layout agrees
    un = ops.silu_mul(torch.nn.functional.linear(x, wgu), block=ops.GU_BLOCK)
    torch.testing.assert_close(un.float(), ref_.float(), atol=2e-2, rtol=2e-2)
    if M in (64, 128, 256):   # every LDS ring depth of the fused kernel
        for bm in (64, 128, 256):
            for ns in (2, 3, 4):
                if bm > M or M % bm or (ns == 2 and bm != 64) or (ns == 4 and bm == 256):
                    continue
                y = torch.empty(M, inter, dtype=x.dtype, device=x.device)
                ops.kernels().gemm_decode(x, wgu, y, None, 1, 128, bm, True, False, ns)
                torch.testing.assert_close(y.float(), ref_.float(), atol=2e-2, rtol=2e-2, msg=f"bm={bm} ns={ns}")


@pytest.mark.parametrize("M,inter,K", [(256, 14336, 4096), (200, 14336, 4096), (256, 15360, 512)])
def test_gate_up_silu_stream_k(M, inter, K):
    """Stream-K gemm_pp (one block per CU over the flattened (tile, K-step) stream, cut tiles
    finished through an fp32 partial + flag) against the fp32 formula, three calls in a row
    (the flags must come back zero), plus the per-tile launch of the same kernel."""
    from operator_amd.ops import kernels

    N = 2 * inter
    assert kernels().gemm_pp_sk_grid(N // 128, K // 64) > N // 128   # the stream-K form runs
    torch.manual_seed(21)
    x = _rand(M, K)
    g, u = _rand(inter, K) * 0.05, _rand(inter, K) * 0.05
    wgu = ops.interleave_gate_up(g, u)
    gf = (x.float() @ g.float().t()).to(torch.bfloat16)
    uf = (x.float() @ u.float().t()).to(torch.bfloat16)
    ref_ = ref.silu_mul(torch.cat([gf, uf], 1)).float()
    ws = torch.full((N // 128 * 32768,), float("nan"), dtype=torch.float32, device=DEV)
    fl = torch.zeros(N // 128, dtype=torch.int32, device=DEV)
    for _ in range(3):
        y = torch.full((M, inter), float("nan"), dtype=torch.bfloat16, device=DEV)
        kernels().gemm_pp(x, wgu, y, None, 1, 256, True, True, False, ws, fl)
        torch.cuda.synchronize()
        torch.testing.assert_close(y.float(), ref_, atol=2e-2, rtol=2e-2)
        assert int(fl.abs().sum()) == 0
    y0 = torch.empty(M, inter, dtype=torch.bfloat16, device=DEV)
    kernels().gemm_pp(x, wgu, y0, None, 1, 256, True, True)
    torch.testing.assert_close(y0.float(), ref_, atol=2e-2, rtol=2e-2)
    # the sums differ only in fp32 association (the cut tile's partial is added last): the bf16
    # outputs agree bit for bit almost everywhere
    assert (y == y0).float().mean().item() > 0.95


@pytest.mark.parametrize("K", [1024, 3584, 8192, 14336, 20480])  # reg paths 2/4/8 vectors + streaming
def test_quantize_fp8_matches_torch(K):
    torch.manual_seed(9)
    x = _rand(37, K) * 3
    x[5] = 0  # all-zero row: scale 1, zeros
    q, sx = ops.quantize_fp8(x)
    amax = x.float().abs().amax(1)
    want_s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    torch.testing.assert_close(sx, want_s)
    want_q = (x.float() / want_s[:, None]).to(torch.float8_e4m3fn).float()
    got = q.float()
    # round-to-nearest-even both ways; allow one e4m3 ulp where 1/s products differ in the last bit
    ulp = torch.clamp(want_q.abs(), min=2 ** -6) * 2 ** -3
    assert ((got - want_q).abs() <= ulp + 1e-12).all()
    assert (q[5].float() == 0).all()


@pytest.mark.parametrize("inter", [1024, 3584, 14336])
def test_silu_quantize_fp8_matches_unfused(inter):
    """Fused SwiGLU + per-row quantization == quantize_fp8(silu_mul(gu)) (64-interleaved)."""
    torch.manual_seed(10)
    gu = _rand(19, 2 * inter) * 2
    q, sx = ops.silu_quantize_fp8(gu, block=64)
    m = ops.silu_mul(gu, block=64)
    q0, s0 = ops.quantize_fp8(m)
    torch.testing.assert_close(sx, s0, rtol=1e-6, atol=0)
    got, want = q.float(), q0.float()
    ulp = torch.clamp(want.abs(), min=2 ** -6) * 2 ** -3
    assert ((got - want).abs() <= ulp + 1e-12).all()
    assert (got == want).float().mean() > 0.99


@pytest.mark.parametrize("S", [2, 3, 4, 8])
def test_silu_quantize_fp8_from_splitk_slabs(S):
    """SplitK gate|up slabs -> summed + bf16-rounded in-kernel == reduce then fused kernel
    (S = 2, 4, 8: compile-time slab counts, every load issued first; 3: the runtime loop)."""
    torch.manual_seed(11)
    M, inter = 23, 3584
    P = torch.randn(S, M, 2 * inter, device="cuda") / 2
    a = P[0].clone()
    for k in range(1, S):
        a += P[k]
    q0, s0 = ops.silu_quantize_fp8(a.to(torch.bfloat16), block=64)
    q, sx = ops.silu_quantize_fp8(ops.SplitK(P.reshape(-1), S, M, 2 * inter), block=64)
    assert torch.equal(sx, s0)
    assert torch.equal(q.view(torch.uint8), q0.view(torch.uint8))


def test_linear_fp8_deferred_slabs_match_reduced():
    torch.manual_seed(12)
    M, N, K = 64, 1280, 8192
    x = _rand(M, K)
    w8, sw = ops.quantize_fp8(_rand(N, K) * 0.05)
    plan = (64, 64, 8)
    y = ops.linear_fp8(x, w8, sw, plan=plan)
    sk = ops.linear_fp8(x, w8, sw, plan=plan, defer_reduce=True)
    assert isinstance(sk, ops.SplitK) and sk.S == 8
    assert torch.equal(sk.materialize(), y) or torch.allclose(sk.materialize().float(), y.float(), atol=1e-2)


@pytest.mark.parametrize("M", [1, 37, 64, 200, 256])
@pytest.mark.parametrize("N,K", [(256, 512), (640, 2048), (128, 4096)])
def test_gemm_fp8(M, N, K):
    torch.manual_seed(10)
    x = _rand(M, K)
    w = _rand(N, K) * 0.05
    w8, sw = ops.quantize_fp8(w)
    q, sx = ops.quantize_fp8(x)
    ref_ = (q.float() * sx[:, None]) @ (w8.float() * sw[:, None]).t()
    for bm in (64, 128, 256):
        for bn in (64, 128):
            for S in (1, 2, 3, 4, 8, 12):   # 3 / 12: uneven K slices
                if K // 128 < S or N % bn:
                    continue
                y = ops.linear_fp8(x, w8, sw, plan=(bm, bn, S))
                torch.testing.assert_close(y.float(), ref_, atol=2e-2, rtol=2e-2)
    # and W8A8 stays close to the bf16 product (e4m3: ~3 mantissa bits per operand)
    exact = x.float() @ w.float().t()
    rel = (ops.linear_fp8(x, w8, sw).float() - exact).norm() / exact.norm()
    assert rel < 0.06, float(rel)


@pytest.mark.parametrize("S", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("N", [1024, 3072, 4096])   # 3072 / 4096: the 512-thread slab-sum path
def test_rmsnorm_sums_splitk_slabs(S, N):
    torch.manual_seed(11)
    M = 128
    P = torch.randn(S * M * N, device=DEV, dtype=torch.float32)
    w = _rand(N)
    r1 = _rand(M, N)
    r2 = r1.clone()
    y1 = ops.rmsnorm(ops.SplitK(P, S, M, N), w, 1e-5, residual=r1)
    y2 = ops.rmsnorm(ops.SplitK(P, S, M, N).materialize(), w, 1e-5, residual=r2)
    torch.testing.assert_close(r1.float(), r2.float(), atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(y1.float(), y2.float(), atol=2e-2, rtol=2e-2)


def test_deferred_splitk_decode_matches_plain():
    """Decode-bucket projections with the split-K reduction folded into rmsnorm give
    the same logits as the plain path."""
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import ForwardBatch, LlamaModel

    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device=DEV).init_random(seed=3)
    kv = PagedKVCache(cfg.layers, 256, cfg.kv_heads, 128, 16, device=DEV)
    B = 64
    lens = torch.randint(1, 200, (B,), device=DEV, dtype=torch.int32)
    bt = torch.arange(B * 13, device=DEV, dtype=torch.int32).reshape(B, 13) % 256
    fb = ForwardBatch(torch.randint(0, cfg.vocab_size, (B,), device=DEV), (lens - 1).long(),
                      torch.full((B,), -1, dtype=torch.long, device=DEV), False, None, block_tables=bt,
                      context_lens=lens, num_splits=1)
    assert ops.gemm_plan(B, cfg.hidden, cfg.heads * cfg.head_dim)[2] > 1  # the o-proj really splits
    a = m.forward(fb, kv)
    orig = m.tp.world
    lin = m._lin
    m._lin = lambda x, w, sc, defer=False: lin(x, w, sc, False)
    b = m.forward(fb, kv)
    m._lin = lin
    torch.testing.assert_close(a.float(), b.float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("S", [4, 5, 3])   # 4 / 5: compiled slab counts (5 = the 8B qkv plan), 3: runtime S
def test_rope_kv_from_splitk_slabs(S):
    torch.manual_seed(12)
    T, Hq, Hkv, D = 64, 8, 2, 128
    W = (Hq + 2 * Hkv) * D
    P = torch.randn(S * T * W, device=DEV, dtype=torch.float32)
    sk = ops.SplitK(P, S, T, W)
    cos, sin = ref.rope_tables(4096, D, 500000.0)
    cos, sin = cos.to(DEV), sin.to(DEV)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    kc1 = torch.zeros(8, Hkv, 16, D, device=DEV, dtype=torch.bfloat16)
    vc1, kc2, vc2 = kc1.clone(), kc1.clone(), kc1.clone()
    slots = torch.randperm(128, device=DEV)[:T]
    q1, k1, v1 = ops.rope_kv(sk, pos, cos, sin, Hq, Hkv, kc1, vc1, slots)
    q2, k2, v2 = ops.rope_kv(sk.materialize(), pos, cos, sin, Hq, Hkv, kc2, vc2, slots)
    for a, b in ((q1, q2), (k1, k2), (v1, v2), (kc1, kc2), (vc1, vc2)):
        torch.testing.assert_close(a.float(), b.float(), atol=3e-2, rtol=2e-2)


def test_rope_kv_bias_slabs_and_rows():
    """Qwen2 q/k/v bias: added in fp32 to the split-K slab sum before the one bf16
    rounding, and to a bf16 qkv row otherwise; equal to bias-then-rope in fp32."""
    torch.manual_seed(13)
    T, Hq, Hkv, D, S = 64, 7, 1, 128, 2
    W = (Hq + 2 * Hkv) * D
    P = torch.randn(S * T * W, device=DEV, dtype=torch.float32)
    sk = ops.SplitK(P, S, T, W)
    bias = (torch.randn(W, device=DEV) * 2).to(torch.bfloat16)
    cos, sin = ref.rope_tables(4096, D, 1e6)
    cos, sin = cos.to(DEV), sin.to(DEV)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    slots = torch.randperm(128, device=DEV)[:T]
    exact = (P.view(S, T, W).sum(0) + bias.float()).to(torch.bfloat16)
    kc_r, vc_r = torch.zeros(8, Hkv, 16, D, dtype=torch.bfloat16), torch.zeros(8, Hkv, 16, D, dtype=torch.bfloat16)
    q_r, k_r, v_r = ref.rope_kv(exact.cpu(), pos.cpu(), cos.cpu(), sin.cpu(), Hq, Hkv, kc_r, vc_r, slots.cpu())
    for src in (sk, sk.materialize()):
        kc = torch.zeros(8, Hkv, 16, D, device=DEV, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        q, k, v = ops.rope_kv(src, pos, cos, sin, Hq, Hkv, kc, vc, slots, bias=bias)
        for a, b in ((q, q_r), (k, k_r), (v, v_r), (kc, kc_r), (vc, vc_r)):
            torch.testing.assert_close(a.cpu().float(), b.float(), atol=6e-2, rtol=2e-2)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (28, 4), (16, 2)])
@pytest.mark.parametrize("variant", [0, 2])
def test_attn_decode_fp8_cache(Hq, Hkv, variant):
    """e4m3fn KV cache (stored x / scale): the kernel equals the fp32 reference over
    the dequantised cache (the fp8 -> bf16 widening is exact), for both tilings and
    split schedules."""
    torch.manual_seed(14)
    lens, P, D = [1, 70, 300, 1029], 64, 128
    B = len(lens)
    maxp = (max(lens) + P - 1) // P + 1
    pages = B * maxp + 2
    k_scale, v_scale = 0.5, 2.0
    kf, vf = torch.randn(pages, Hkv, P, D, device=DEV) * 3, torch.randn(pages, Hkv, P, D, device=DEV) * 3
    kc = ref.kv_store(kf, torch.float8_e4m3fn, k_scale)
    vc = ref.kv_store(vf, torch.float8_e4m3fn, v_scale)
    bt = torch.randperm(pages, device=DEV)[: B * maxp].reshape(B, maxp).int()
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = _rand(B, Hq, D)
    scale = 1 / math.sqrt(D)
    o_r = ref.attn_decode(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), sl.cpu(), scale, k_scale, v_scale)
    for ns in (1, 4):
        o = ops.attn_decode(q, kc, vc, bt, sl, scale, ns, variant=variant, k_scale=k_scale, v_scale=v_scale)
        torch.testing.assert_close(o.cpu().float(), o_r.float(), atol=3e-2, rtol=3e-2)


def test_rope_kv_writes_fp8_cache():
    """rope_kv into an e4m3fn cache stores e4m3(bf16(rotated k) / k_scale), v / v_scale."""
    torch.manual_seed(15)
    T, Hq, Hkv, D, P, pages = 40, 8, 2, 128, 16, 8
    k_scale, v_scale = 0.25, 4.0
    cos, sin = ref.rope_tables(4096, D, 500000.0, device=DEV)
    qkv = _rand(T, (Hq + 2 * Hkv) * D)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    slots = torch.randperm(pages * P, device=DEV)[:T]
    kc = torch.zeros(pages, Hkv, P, D, dtype=torch.float8_e4m3fn, device=DEV)
    vc = torch.zeros_like(kc)
    ops.rope_kv(qkv, pos, cos, sin, Hq, Hkv, kc, vc, slots, k_scale=k_scale, v_scale=v_scale)
    kb = torch.zeros(pages, Hkv, P, D, dtype=torch.bfloat16, device=DEV)
    vb = torch.zeros_like(kb)
    ops.rope_kv(qkv, pos, cos, sin, Hq, Hkv, kb, vb, slots)
    # same rotated values as the bf16 cache, quantised: at most one e4m3 step apart
    kd, vd = ref.kv_load(kc.cpu(), k_scale), ref.kv_load(vc.cpu(), v_scale)
    torch.testing.assert_close(kd, kb.cpu().float(), atol=0.07 * k_scale, rtol=0.07)
    torch.testing.assert_close(vd, vb.cpu().float(), atol=0.07 * v_scale, rtol=0.07)
    exact = ref.kv_store(vb.cpu().float(), torch.float8_e4m3fn, v_scale)
    assert torch.equal(vc.cpu().view(torch.uint8), exact.view(torch.uint8))


@pytest.mark.parametrize("Hq,Hkv,splits,variant", [(8, 1, 8, 0), (8, 1, 1, 0), (32, 8, 4, 0), (64, 8, 2, 2),
                                                   (64, 8, 64, 0), (40, 8, 64, 0)])
def test_attn_decode_fused_quant_matches_quantized_output(Hq, Hkv, splits, variant):
    """quant=True: the split-combine kernel's e4m3fn rows == quantize_fp8 of the bf16 output.
    Hq x splits > 2048 (70B / Qwen2.5-32B heads at 64 splits) overflows the fused kernel's LDS
    statistics and takes the combine-then-quantize path."""
    torch.manual_seed(21)
    B, D, page = 6, 128, 16
    lens = torch.tensor([1, 17, 300, 64, 129, 511], dtype=torch.int32)
    pages = (int(lens.max()) + page - 1) // page
    kc = _rand(B * pages, Hkv, page, D)
    vc = _rand(B * pages, Hkv, page, D)
    bt = torch.arange(B * pages, dtype=torch.int32).view(B, pages)
    q = _rand(B, Hq, D)
    dev = "cuda"
    args = (q.to(dev), kc.to(dev), vc.to(dev), bt.to(dev), lens.to(dev), D ** -0.5, splits)
    o = ops.attn_decode(*args, variant=variant)
    q8, sx = ops.attn_decode(*args, variant=variant, quant=True)
    q0, s0 = ops.quantize_fp8(o.view(B, Hq * D))
    torch.testing.assert_close(sx, s0, rtol=0, atol=0)
    assert torch.equal(q8.view(torch.uint8), q0.view(torch.uint8))


def test_decode_step_bookkeeping_kernels_match_torch():
    """decode_slots / decode_advance (one thread per row) == the torch formulation of a
    decode step's slot computation and state advance, padding rows (ctx 0) included."""
    torch.manual_seed(31)
    B, MP, P, ms = 200, 24, 64, 8
    bt = torch.randint(0, 5000, (B, MP), dtype=torch.int32, device=DEV)
    ctx = torch.randint(1, MP * P, (B,), dtype=torch.int32, device=DEV)
    ctx[::7] = 0
    pos = (ctx.long() - 1).clamp_min(0)
    act = ctx > 0
    pg = torch.gather(bt, 1, torch.clamp(pos // P, max=MP - 1).unsqueeze(1)).squeeze(1)
    want_slots = torch.where(act, pg.long() * P + pos % P, torch.full_like(pos, -1))
    slots, spos = torch.empty_like(pos), torch.empty_like(pos)
    ops.kernels().decode_slots(bt, pos, ctx, slots, spos, P)
    assert torch.equal(slots, want_slots) and torch.equal(spos, pos + 1)
    tok = torch.randint(0, 128000, (B,), device=DEV)
    for step0 in (0, 5, 7, 13):
        ids, hist = torch.zeros(B, dtype=torch.long, device=DEV), torch.zeros(B, ms, dtype=torch.long, device=DEV)
        p2, c2, st = pos.clone(), ctx.clone(), torch.tensor([step0], device=DEV)
        ops.kernels().decode_advance(tok, ids, hist, p2, c2, st)
        want_hist = torch.zeros_like(hist)
        want_hist[:, step0 % ms] = tok
        assert torch.equal(ids, tok) and torch.equal(hist, want_hist)
        assert torch.equal(p2, pos + act.long()) and torch.equal(c2, ctx + act.int()) and st.item() == step0 + 1


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (28, 4)])
@pytest.mark.parametrize("splits_qkv", [1, 2, 4, 8])
@pytest.mark.parametrize("fp8", [False, True])
def test_attn_decode_rope_equals_rope_kv_then_attn(Hq, Hkv, splits_qkv, fp8):
    """The decode RoPE + KV write folded into decode attention (ops.attn_decode_rope) is
    bit-identical to rope_kv then attn_decode: the same cache bytes for the new token and
    the same output rows (and e4m3fn rows with quant), for every split schedule. The new
    token's slot holds NaN before the call, so a workgroup reading it before its own write
    (the chunk requested in the prologue, or a clamped copy of the token) poisons the row.
    Contexts 1 / 17 / 64 / 65 / 130 / 700 cover the one- and two-chunk reload paths; qkv
    as bf16 rows (1), runtime (2) and compiled (4, 8) slab counts; a Qwen2-style bias."""
    torch.manual_seed(21)
    lens, P, D = [1, 17, 64, 65, 130, 700, 0], 16, 128
    B = len(lens)
    maxp = (max(lens) + P - 1) // P + 1
    pages = B * maxp + 3
    ncol = (Hq + 2 * Hkv) * D
    k_scale, v_scale = (0.5, 2.0) if fp8 else (1.0, 1.0)
    kf, vf = torch.randn(pages, Hkv, P, D, device=DEV), torch.randn(pages, Hkv, P, D, device=DEV)
    if fp8:
        kc0, vc0 = ref.kv_store(kf, torch.float8_e4m3fn, k_scale), ref.kv_store(vf, torch.float8_e4m3fn, v_scale)
    else:
        kc0, vc0 = kf.to(torch.bfloat16), vf.to(torch.bfloat16)
    bt = torch.randperm(pages, device=DEV)[: B * maxp].reshape(B, maxp).int()
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    pos = torch.tensor([max(n - 1, 0) for n in lens], dtype=torch.long, device=DEV)
    slots = torch.tensor([int(bt[b, (n - 1) // P]) * P + (n - 1) % P if n > 0 else -1 for b, n in enumerate(lens)],
                         dtype=torch.long, device=DEV)
    # the new tokens' slots start as NaN (whatever a freed page held)
    for b, n in enumerate(lens):
        if n > 0:
            pg, off = int(bt[b, (n - 1) // P]), (n - 1) % P
            kc0.view(torch.uint8)[pg, :, off] = 0x7F if fp8 else 0
            vc0.view(torch.uint8)[pg, :, off] = 0x7F if fp8 else 0
            if not fp8:
                kc0[pg, :, off] = float("nan")
                vc0[pg, :, off] = float("nan")
    theta = 500000.0
    inv = 1.0 / theta ** (torch.arange(0, D, 2, device=DEV).float() / D)
    ang = torch.arange(4096, device=DEV).float()[:, None] * inv[None]
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    bias = (torch.randn(ncol, device=DEV) * 0.1).to(torch.bfloat16) if Hq == 28 else None
    if splits_qkv == 1:
        qkv = (torch.randn(B, ncol, device=DEV)).to(torch.bfloat16)
    else:
        qkv = ops.SplitK(torch.randn(splits_qkv * B * ncol, device=DEV) * 0.5, splits_qkv, B, ncol)
    scale = 1 / math.sqrt(D)
    for ns in (1, 2, 4):
        for quant in ((False, True) if Hq * D <= 8192 else (False,)):
            kc_a, vc_a, kc_b, vc_b = kc0.clone(), vc0.clone(), kc0.clone(), vc0.clone()
            q, _, _ = ops.rope_kv(qkv, pos, cos, sin, Hq, Hkv, kc_a, vc_a, slots, want_kv=False, bias=bias,
                                  k_scale=k_scale, v_scale=v_scale)
            want = ops.attn_decode(q, kc_a, vc_a, bt, sl, scale, ns, k_scale=k_scale, v_scale=v_scale, quant=quant)
            got = ops.attn_decode_rope(qkv, pos, cos, sin, Hq, kc_b, vc_b, slots, bt, sl, scale, ns, bias=bias,
                                       k_scale=k_scale, v_scale=v_scale, quant=quant)
            torch.cuda.synchronize()
            assert torch.equal(kc_a.view(torch.uint8), kc_b.view(torch.uint8))
            assert torch.equal(vc_a.view(torch.uint8), vc_b.view(torch.uint8))
            if quant:
                assert torch.equal(got[0].view(torch.uint8), want[0].view(torch.uint8))
                assert torch.equal(got[1], want[1])
            else:
                live = sl.cpu() > 0
                assert torch.isfinite(got.float()[live.to(DEV)]).all()
                assert torch.equal(got.view(torch.int16)[live.to(DEV)], want.view(torch.int16)[live.to(DEV)])
