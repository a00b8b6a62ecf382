"""gfx950 gemm_xr (csrc/kernels/gemm_xr.hip): the 256-row decode GEMM whose activations stream
through a register ring in the fragment-major tiled layout. Against the plain-PyTorch fp32
reference: every epilogue (fp32 split-K slabs, bf16 rows, fused SwiGLU row-major and tiled),
every split count the decode plans use, the tiled layout written by tile_rows and by rmsnorm
(tiled_out), and step counts that exercise the prologue / steady / tail paths of the loop."""
import pytest
import torch

from operator_amd import ops
from operator_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


def untile(xt: torch.Tensor, M: int, K: int) -> torch.Tensor:
    """The tiled layout [K/64][M/16][2 k-half][4 (k%32)/8][16 row%16][8] -> row-major [M, K]."""
    return xt.reshape(K // 64, M // 16, 2, 4, 16, 8).permute(1, 4, 0, 2, 3, 5).reshape(M, K)


def test_tile_rows_roundtrip():
    x = _rand(256, 1024)
    xt = torch.empty_like(x)
    ops.kernels().tile_rows(x, xt)
    torch.cuda.synchronize()
    assert torch.equal(untile(xt, 256, 1024), x)
    assert not torch.equal(xt, x)


@pytest.mark.parametrize("N,K,S", [(128, 64, 1), (256, 512, 1), (384, 1024, 2), (1024, 4096, 4), (6144, 4096, 4),
                                   (4096, 14336, 8), (512, 2048, 8), (256, 3072, 3)])
def test_gemm_xr_slabs_and_store(N, K, S):
    """T = K / (64 S) from 1 (prologue only) through 8 / 16 / 28 (steady loop + tail)."""
    torch.manual_seed(N + K + S)
    x, w = _rand(256, K), _rand(N, K, scale=0.05)
    r = x.float() @ w.float().t()
    xt = torch.empty_like(x)
    ops.kernels().tile_rows(x, xt)
    P = torch.empty(S * 256 * N, dtype=torch.float32, device=DEV)
    ops.kernels().gemm_xr(xt, w, None, P, S, 0)
    torch.cuda.synchronize()
    torch.testing.assert_close(P.view(S, 256, N).sum(0), r, atol=2e-3, rtol=2e-3)
    if S == 1:
        y = torch.empty(256, N, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_xr(xt, w, y, None, 1, 1)
        torch.testing.assert_close(y.float(), r, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("inter,K", [(64, 128), (1024, 2048), (14336, 4096)])
def test_gemm_xr_swiglu_rows_and_tiled(inter, K):
    torch.manual_seed(inter)
    x = _rand(256, K)
    g, u = _rand(inter, K, scale=0.05), _rand(inter, K, scale=0.05)
    wgu = ops.interleave_gate_up(g, u)
    gg = (x.float() @ g.float().t()).to(torch.bfloat16)
    uu = (x.float() @ u.float().t()).to(torch.bfloat16)
    r = ref.silu_mul(torch.cat([gg, uu], 1), None)
    xt = torch.empty_like(x)
    ops.kernels().tile_rows(x, xt)
    y = torch.empty(256, inter, dtype=torch.bfloat16, device=DEV)
    ops.kernels().gemm_xr(xt, wgu, y, None, 1, 2)
    torch.testing.assert_close(y.float(), r.float(), atol=3e-2, rtol=3e-2)
    if inter % 64 == 0:
        yt = torch.empty(256, inter, dtype=torch.bfloat16, device=DEV)
        ops.kernels().gemm_xr(xt, wgu, yt, None, 1, 3)
        torch.cuda.synchronize()
        assert torch.equal(untile(yt, 256, inter), y)   # same values, tiled for the next gemm_xr


def test_rmsnorm_tiled_output_feeds_gemm_xr():
    """rmsnorm(tiled_out=True) writes exactly the tiled image of its row-major output
    (with and without summing split-K slabs), and gemm_xr on it matches the fp32 reference."""
    torch.manual_seed(7)
    M, H = 256, 4096
    h = _rand(M, H)
    nw = _rand(H, scale=0.5)
    res1, res2 = _rand(M, H), None
    res2 = res1.clone()
    y = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    yt = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    ops.kernels().rmsnorm(h, res1, nw, y, 1e-5)
    ops.kernels().rmsnorm(h, res2, nw, yt, 1e-5, None, 1, True)
    torch.cuda.synchronize()
    assert torch.equal(res1, res2) and torch.equal(untile(yt, M, H), y)
    S = 4
    P = (torch.randn(S * M * H, device=DEV) * 0.1).float()
    ys = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    yst = torch.empty(M, H, dtype=torch.bfloat16, device=DEV)
    r3, r4 = res1.clone(), res1.clone()
    ops.kernels().rmsnorm(ys, r3, nw, ys, 1e-5, P, S)
    ops.kernels().rmsnorm(yst, r4, nw, yst, 1e-5, P, S, True)
    torch.cuda.synchronize()
    assert torch.equal(r3, r4) and torch.equal(untile(yst, M, H), ys)
    w = _rand(1024, H, scale=0.05)
    P2 = torch.empty(4 * M * 1024, dtype=torch.float32, device=DEV)
    ops.kernels().gemm_xr(yst, w, None, P2, 4, 0)
    torch.cuda.synchronize()
    torch.testing.assert_close(P2.view(4, M, 1024).sum(0), ys.float() @ w.float().t(), atol=2e-3, rtol=2e-3)


def test_gemm_xr_rejects_bad_shapes():
    x, w = _rand(128, 256), _rand(128, 256)
    with pytest.raises(RuntimeError):
        ops.kernels().gemm_xr(x, w, torch.empty(128, 128, dtype=torch.bfloat16, device=DEV), None, 1, 1)
    x = _rand(256, 256)
    with pytest.raises(RuntimeError):
        ops.kernels().gemm_xr(x, _rand(100, 256), torch.empty(256, 100, dtype=torch.bfloat16, device=DEV), None, 1, 1)
