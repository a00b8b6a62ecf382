"""gfx950 256x256-tile GEMM (csrc/kernels/gemm_tile.hip: prefill projections and the
lm_head) against the plain-PyTorch fp32 reference: M / N tails, every epilogue
(store, bias, fused SwiGLU over the 64-row interleaved gate|up weight), strided
outputs, and an asymmetric-operand layout check (cdna_hip_programming.md §3)."""
import pytest
import torch

from operator_amd import ops
from operator_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
VARIANTS = (0, 1, 2, 3, 4, 5)   # gemm_tile schedules: auto, 4-wave two-buffer four-phase (h4), 8-wave 2-segment, 8-wave 4-segment,
# 4-wave with W-fragment MFMA groups, persistent one-workgroup-per-CU p5 (variant 5 needs K >= 128)


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def _close(y, r, tol=2e-2):
    torch.testing.assert_close(y.float(), r.float(), atol=tol, rtol=tol)


@pytest.mark.parametrize("M", [1, 77, 256, 300, 1024])
@pytest.mark.parametrize("N,K", [(16, 64), (272, 192), (512, 1024), (6144, 4096), (4096, 14336)])
def test_gemm_tile_store_and_bias(M, N, K):
    if M * N * K > 1024 * 6144 * 4096:
        pytest.skip("covered by the smaller shapes")
    torch.manual_seed(M * 7 + N + K)
    x = _rand(M, K)
    w = _rand(N, K, scale=0.05)
    r = x.float() @ w.float().t()
    b = _rand(N, scale=0.5)
    for v in VARIANTS:
        y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_tile(x, w, y, None, False, v)
        _close(y, r)
        yb = torch.empty_like(y)
        ops.kernels().gemm_tile(x, w, yb, b, False, v)
        _close(yb, r + b.float())


def test_gemm_tile_layout_exact():
    """Small-integer operands (exact in bf16 and fp32): every output element must be
    bit-exact, which catches a transposed or shifted fragment / store map."""
    M, N, K = 300, 528, 256
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randint(-3, 4, (M, K), generator=g).to(DEV, torch.bfloat16)
    w = torch.randint(-3, 4, (N, K), generator=g).to(DEV, torch.bfloat16)
    w[5, :] = 0
    w[5, 17] = 1   # column 5 of y = x[:, 17]
    r = x.float() @ w.float().t()     # exact in fp32; y is that rounded once to bf16
    for v in VARIANTS:
        y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_tile(x, w, y, None, False, v)
        assert torch.equal(y, r.to(torch.bfloat16))
        assert torch.equal(y[:, 5].float(), x[:, 17].float())


@pytest.mark.parametrize("M", [5, 256, 513])
@pytest.mark.parametrize("inter,K", [(64, 128), (192, 256), (1536, 1024)])
def test_gemm_tile_silu(M, inter, K):
    torch.manual_seed(inter + M)
    x = _rand(M, K)
    g = _rand(inter, K, scale=0.05)
    u = _rand(inter, K, scale=0.05)
    wgu = ops.interleave_gate_up(g, u)
    gg = (x.float() @ g.float().t()).to(torch.bfloat16)
    uu = (x.float() @ u.float().t()).to(torch.bfloat16)
    r = ref.silu_mul(torch.cat([gg, uu], 1), None)
    for v in VARIANTS:
        y = torch.empty(M, inter, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_tile(x, wgu, y, None, True, v)
        _close(y, r, 3e-2)


@pytest.mark.parametrize("S", [2, 4])
def test_gemm_tile_split_k(S):
    """Split-K: fp32 slabs [S][M][N] (consumer-summed), the reduced bf16 output and the
    fused-SwiGLU reduce of interleaved gate|up slabs, against fp32 references."""
    M, N, K = 300, 512, 1024
    torch.manual_seed(S)
    x, w = _rand(M, K), _rand(N, K, scale=0.05)
    r = x.float() @ w.float().t()
    P = torch.empty(S * M * N, dtype=torch.float32, device=DEV)
    ops.kernels().gemm_tile(x, w, None, None, False, 0, S, P)
    torch.cuda.synchronize()
    _close(P.view(S, M, N).sum(0), r, 1e-3)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.kernels().gemm_tile(x, w, y, None, False, 0, S, P)
    _close(y, r)
    g, u = _rand(256, K, scale=0.05), _rand(256, K, scale=0.05)
    wgu = ops.interleave_gate_up(g, u)
    gg = (x.float() @ g.float().t()).to(torch.bfloat16)
    uu = (x.float() @ u.float().t()).to(torch.bfloat16)
    ys = torch.empty(M, 256, dtype=torch.bfloat16, device=DEV)
    ops.kernels().gemm_tile(x, wgu, ys, None, True, 0, S, P)
    _close(ys, ref.silu_mul(torch.cat([gg, uu], 1), None), 3e-2)


@pytest.mark.parametrize("M,N,K", [(8192 + 77, 2304, 192), (4096, 4096 + 16, 128), (2048, 16384, 320), (300, 1024, 4096)])
@pytest.mark.parametrize("epi", ["store", "bias", "silu"])
def test_gemm_tile_persistent_rounds(M, N, K, epi):
    """Persistent p5 (variant 5): blocks walk several tiles (tiles > CUs), odd K-step
    counts (the LDS buffer parity carries across tiles), M / N tails, grids below the CU
    count -- every epilogue against the fp32 reference."""
    torch.manual_seed(M + N + K)
    x = _rand(M, K)
    if epi == "silu":
        if N % 128:
            pytest.skip("the interleaved gate|up weight needs N % 128 == 0")
        g, u = _rand(N // 2, K, scale=0.05), _rand(N // 2, K, scale=0.05)
        w = ops.interleave_gate_up(g, u)
        gg = (x.float() @ g.float().t()).to(torch.bfloat16)
        uu = (x.float() @ u.float().t()).to(torch.bfloat16)
        r = ref.silu_mul(torch.cat([gg, uu], 1), None)
        y = torch.empty(M, N // 2, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_tile(x, w, y, None, True, 5)
        _close(y, r, 3e-2)
        return
    w = _rand(N, K, scale=0.05)
    b = _rand(N, scale=0.5) if epi == "bias" else None
    r = x.float() @ w.float().t() + (b.float() if b is not None else 0.0)
    for v in ((5, 6, 7, 8, 9, 10, 11, 12, 13, 14) if b is None else (5,)):   # 6-14: p5 schedule arms (store epilogue)
        y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_tile(x, w, y, b, False, v)
        _close(y, r)


def test_gemm_tile_strided_output():
    """Writing into a column slice of a wider buffer (ldy > N) leaves the rest alone."""
    M, N, K = 130, 256, 128
    x, w = _rand(M, K), _rand(N, K, scale=0.1)
    buf = torch.full((M, N + 64), 7.0, dtype=torch.bfloat16, device=DEV)
    ops.kernels().gemm_tile(x, w, buf[:, 32:32 + N])
    _close(buf[:, 32:32 + N], x.float() @ w.float().t())
    assert (buf[:, :32] == 7).all() and (buf[:, 32 + N:] == 7).all()


def test_gemm_tile_rejects_bad_shapes():
    x, w = _rand(8, 100), _rand(32, 100)
    with pytest.raises(RuntimeError):
        ops.kernels().gemm_tile(x, w, torch.empty(8, 32, dtype=torch.bfloat16, device=DEV))


@pytest.mark.parametrize("M", [1, 64, 130, 256])
@pytest.mark.parametrize("N,K", [(128, 64), (384, 192), (1024, 1024), (4096, 4096)])
def test_gemm_pp_decode(M, N, K):
    """Ping-pong decode GEMM (gemm_pp.hip): both row tiles, every split count, nt and
    default weight policy, reduced and deferred (slab) outputs."""
    torch.manual_seed(M + N + K)
    x = _rand(M, K)
    w = _rand(N, K, scale=0.05)
    r = x.float() @ w.float().t()
    P = torch.empty(8 * M * N, dtype=torch.float32, device=DEV)
    for bm in (128, 256):
        for S in (1, 2, 4, 8):
            if K % (64 * S):
                continue
            for nt in (True, False):
                y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
                ops.kernels().gemm_pp(x, w, y, P if S > 1 else None, S, bm, False, nt)
                _close(y, r)
            if S > 1:
                ops.kernels().gemm_pp(x, w, None, P, S, bm, False, True)
                torch.cuda.synchronize()
                _close(P[:S * M * N].view(S, M, N).sum(0), r)
            if bm == 256:   # one barrier segment per K-tile
                y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
                ops.kernels().gemm_pp(x, w, y, P if S > 1 else None, S, bm, False, True, True)
                _close(y, r)


@pytest.mark.parametrize("M", [3, 128, 256])
def test_gemm_pp_silu(M):
    inter, K = 1024, 2048
    torch.manual_seed(M)
    x = _rand(M, K)
    g = _rand(inter, K, scale=0.05)
    u = _rand(inter, K, scale=0.05)
    wgu = ops.interleave_gate_up(g, u)
    gg = (x.float() @ g.float().t()).to(torch.bfloat16)
    uu = (x.float() @ u.float().t()).to(torch.bfloat16)
    r = ref.silu_mul(torch.cat([gg, uu], 1), None)
    for bm, one in ((128, False), (256, False), (256, True)):
        y = torch.empty(M, inter, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_pp(x, wgu, y, None, 1, bm, True, True, one)
        _close(y, r, 3e-2)
