"""One-shot IPC all-reduce (csrc/kernels/allreduce.hip) with 2 ranks.

The gpurun box has one MI355X, so both ranks are processes on the SAME device:
the kernel's peer path (hipIpc export/open, pushes into the peer's
fine-grained buffer, system-scope flags) is exercised exactly as across xGMI,
just over local HBM. The handle exchange runs over a gloo group (RCCL refuses
two ranks on one device). Reference: fp32 sum of both ranks' inputs, rounded
once — the kernel accumulates in fp32 in rank order, so results must be exact. The
fused residual + RMSNorm epilogue is checked against the plain fp32 torch formula
(HF Llama rounding points), not against another HIP kernel.
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(rank: int, n: int, dtype, call: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 * rank + 17 * call + n)
    return torch.randn(n, generator=g, dtype=torch.float32).to(dtype)


def _rmsnorm_fp32(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor):
    """HF Llama numerics in plain torch: h = bf16(x + residual); y = bf16(bf16(h * rsqrt(
    mean(h^2) + eps)) * w), everything computed in fp32. Returns (y, h)."""
    h = (x.float() + residual.float()).to(torch.bfloat16)
    hf = h.float()
    y = (hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + eps)).to(torch.bfloat16)
    return (y.float() * w.float()).to(torch.bfloat16), h


def _worker(rank: int, world: int, port: int, q, protocol: str = "auto") -> None:
    try:
        os.environ["OAMD_CAR_PROTOCOL"] = protocol
        import torch.distributed as dist

        from operator_amd.parallel.comm import Group

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        grp = Group()
        assert grp.enable_oneshot(dev, max_bytes=4 << 20)
        car = grp.oneshot
        checked = 0
        call = 0
        for dtype in (torch.bfloat16, torch.float32):
            for n in (8, 4096, 8192 * 3, 1 << 20 if dtype == torch.float32 else 2 << 20):
                for _ in range(3):  # both parities of the receive buffer, repeated
                    xs = [_inputs(r, n, dtype, call) for r in range(world)]
                    want = sum(x.float() for x in xs).to(dtype)
                    t = xs[rank].to(dev)
                    grp.all_reduce_(t)
                    torch.cuda.synchronize()
                    assert torch.equal(t.cpu(), want), (dtype, n, (t.cpu().float() - want.float()).abs().max())
                    call += 1
                    checked += 1
        # fused all-reduce + residual + RMSNorm (the TP block epilogue), interleaved with
        # plain calls on the same per-block round counters
        from operator_amd import ops

        for rows, hidden in ((1, 4096), (7, 8192), (64, 8192), (256, 8192), (100, 16384)):
            xs = [_inputs(r, rows * hidden, torch.bfloat16, call).view(rows, hidden) for r in range(world)]
            h0 = _inputs(99, rows * hidden, torch.bfloat16, call).view(rows, hidden).to(dev)
            wv = (1 + 0.1 * _inputs(98, hidden, torch.float32, call)).to(torch.bfloat16).to(dev)
            ssum = sum(x.float() for x in xs).to(torch.bfloat16).to(dev)
            y_ref, h_ref = _rmsnorm_fp32(ssum, wv, 1e-5, h0)
            h = h0.clone()
            y = grp.all_reduce_rmsnorm(xs[rank].to(dev), wv, 1e-5, residual=h)
            torch.cuda.synchronize()
            assert torch.equal(h, h_ref), (rows, hidden, (h.float() - h_ref.float()).abs().max())
            torch.testing.assert_close(y.float(), y_ref.float(), atol=1e-2, rtol=1e-2)
            # split-K slabs in (summed in slab order, bf16-rounded) and e4m3fn rows out
            for S in (2, 3, 4):   # two- and four-slab paths load every slab together; 3: the loop
                ps = [(_inputs(50 + r, S * rows * hidden, torch.float32, call) / S).view(S, rows, hidden)
                      for r in range(world)]
                ts = []
                for pr in ps:
                    a = pr[0].clone()
                    for k in range(1, S):
                        a += pr[k]
                    ts.append(a.to(torch.bfloat16))
                ssum = sum(x.float() for x in ts).to(torch.bfloat16).to(dev)
                y_ref, h_ref = _rmsnorm_fp32(ssum, wv, 1e-5, h0)
                h = h0.clone()
                slabs = ops.SplitK(ps[rank].reshape(-1).to(dev), S, rows, hidden)
                q8, sx = grp.all_reduce_rmsnorm(slabs, wv, 1e-5, residual=h, quant=True)
                torch.cuda.synchronize()
                assert torch.equal(h, h_ref), ("slabs", rows, hidden, (h.float() - h_ref.float()).abs().max())
                # the e4m3fn rows: per-row scale max|y| / 448 of the fp32-formula y, then round
                amax = y_ref.float().abs().amax(-1)
                s_ref = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
                q_ref = (y_ref.float() / s_ref[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
                torch.testing.assert_close(sx, s_ref, rtol=2e-2, atol=0)
                deq, deq_ref = q8.float() * sx[:, None], q_ref.float() * s_ref[:, None]
                torch.testing.assert_close(deq, deq_ref, atol=3e-2 * float(deq_ref.abs().max()), rtol=0.07)
            t = xs[rank].reshape(-1).to(dev)
            grp.all_reduce_(t)                      # a plain call in between
            torch.cuda.synchronize()
            assert torch.equal(t.cpu(), sum(x.float() for x in xs).to(torch.bfloat16).reshape(-1))
            call += 1
            checked += 1
        # hipGraph capture: the round counter lives on the device, so replays stay in step
        n = 16384
        buf = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        out = torch.zeros_like(buf)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            out.copy_(car.all_reduce(buf))
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out.copy_(car.all_reduce(buf))
        for rep in range(5):
            xs = [_inputs(r, n, torch.bfloat16, 500 + rep) for r in range(world)]
            buf.copy_(xs[rank].to(dev))
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out.cpu(), sum(x.float() for x in xs).to(torch.bfloat16)), rep
            checked += 1
        car.check()
        dist.barrier()
        car.close()
        dist.destroy_process_group()
        q.put((rank, "ok", checked))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("protocol", ["auto", "oneshot", "twoshot", "fence", "ll"])
def test_oneshot_allreduce_two_ranks_one_gpu(protocol):
    """Every protocol (auto: one-shot up to 512 KB, two-shot above; each forced; the
    original system-fence one-shot; LL flag-in-data packets, one-shot past their half-
    capacity limit) gives the exact fp32-in-rank-order sums, fused epilogues included,
    interleaved on the same per-block round counters."""
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from operator_amd.ops import kernels

    assert hasattr(kernels(), "CustomAllReduce")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, protocol)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in procs:
            res.append(q.get(timeout=100))
    finally:
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    errs = [r for r in res if r[1] != "ok"]
    assert not errs, errs[0][2]
    assert all(r[2] >= 30 for r in res), res


def _missing_peer_worker(rank: int, world: int, port: int, q, protocol: str = "oneshot") -> None:
    """Rank 1 skips one all-reduce: rank 0 must time out with an error and NaN output,
    never return its own partial sum; after that the error is sticky on both ranks."""
    try:
        os.environ["OAMD_CAR_PROTOCOL"] = protocol
        import time

        import torch.distributed as dist

        from operator_amd.parallel.comm import Group
        from operator_amd.parallel.custom_ar import CollectiveTimeout, OneShotAllReduce

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        car = OneShotAllReduce(Group(), dev, max_bytes=1 << 20, timeout_s=0.2)
        n = 8192
        # one good call first: the protocol works with both ranks present
        x = torch.full((n,), float(rank + 1), dtype=torch.bfloat16, device=dev)
        y = car.all_reduce(x)
        torch.cuda.synchronize()
        assert torch.equal(y.cpu(), torch.full((n,), 3.0, dtype=torch.bfloat16)) and not car.failed
        dist.barrier()
        out = {}
        if rank == 0:
            t0 = time.perf_counter()
            y = car.all_reduce(x)           # rank 1 never arrives
            torch.cuda.synchronize()
            out["wait_s"] = time.perf_counter() - t0
            out["all_nan"] = bool(torch.isnan(y.float()).all())
            out["failed"] = car.failed
            try:
                car.check()
                out["raised"] = False
            except CollectiveTimeout:
                out["raised"] = True
            t0 = time.perf_counter()
            y = car.all_reduce(x)           # sticky: NaN at once, no wait, no peer touched
            torch.cuda.synchronize()
            out["sticky_nan"] = bool(torch.isnan(y.float()).all())
            out["sticky_s"] = time.perf_counter() - t0
        dist.barrier()
        if rank == 1:
            # one-shot: rank 0 pushed its slice before it timed out, so rank 1's call of that
            # round still completes with the true sum ...
            y = car.all_reduce(x)
            torch.cuda.synchronize()
            out["late_ok"] = torch.equal(y.cpu(), torch.full((n,), 3.0, dtype=torch.bfloat16)) and not car.failed
            out["late_nan"] = bool(torch.isnan(y.float()).all())
            y = car.all_reduce(x)           # ... but rank 0 now pushes nothing: timeout, NaN
            torch.cuda.synchronize()
            out["all_nan"] = bool(torch.isnan(y.float()).all())
            out["failed"] = car.failed
        dist.barrier()
        car.close()
        dist.destroy_process_group()
        q.put((rank, "ok", out))
    except BaseException:  # noqa: BLE001
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("protocol", ["oneshot", "twoshot", "ll"])
def test_oneshot_allreduce_missing_peer_fails_loudly(protocol):
    """One-shot and LL: rank 1's late call still completes (rank 0 pushed before timing out),
    its next one times out. Two-shot: rank 0 never reaches the all-gather phase, so rank
    1's late call already times out. Either way: NaN, never a partial sum, and sticky."""
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_missing_peer_worker, args=(r, 2, port, q, protocol)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            r = q.get(timeout=100)
            res[r[0]] = r
    finally:
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    errs = [r for r in res.values() if r[1] != "ok"]
    assert not errs, errs[0][2]
    r0, r1 = res[0][2], res[1][2]
    assert r0["failed"] and r0["raised"] and r0["all_nan"], r0
    assert 0.15 < r0["wait_s"] < 5.0, r0
    assert r0["sticky_nan"] and r0["sticky_s"] < 0.1, r0
    if protocol in ("oneshot", "ll"):
        assert r1["late_ok"] and r1["failed"] and r1["all_nan"], r1
    else:   # rank 0 never published its gather piece: the late call already fails
        assert not r1["late_ok"] and r1["late_nan"] and r1["failed"] and r1["all_nan"], r1


def _calibrate_worker(rank: int, world: int, port: int, q) -> None:
    try:
        import torch.distributed as dist

        from operator_amd.engine.factory import calibrate_allreduce
        from operator_amd.parallel.comm import Group
        from operator_amd.parallel.custom_ar import PROTO_BACKEND

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        grp = Group()
        assert grp.enable_oneshot(dev, max_bytes=4 << 20)
        rep = calibrate_allreduce(grp, hidden=1024, max_batch=256, iters=5)
        car = grp.oneshot
        assert car.table and rep["table"], rep
        # after calibration every size still sums exactly (whichever protocol it routes to)
        ok = 0
        for rows in (1, 16, 256):
            x = [_inputs(r, rows * 1024, torch.bfloat16, 900 + rows) for r in range(world)]
            ref = (x[0].float() + x[1].float()).to(torch.bfloat16)
            t = x[rank].to(dev)
            grp.all_reduce_(t)
            torch.cuda.synchronize()
            assert torch.equal(t.cpu(), ref), rows
            ok += 1
        q.put((rank, "ok", rep, [(b, p) for b, p in car.table], car.route(2048) != PROTO_BACKEND or True, ok))
        dist.barrier()
        car.close()
        dist.destroy_process_group()
    except Exception:
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_allreduce_calibration_two_ranks_one_gpu():
    """calibrate() at engine start (engine.oneshot_max_kb = 0): both ranks time one-shot,
    two-shot and the group backend on the decode message sizes, take the max over ranks
    and install the SAME dispatch table; all-reduces routed by it stay exact."""
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_calibrate_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in procs:
            res.append(q.get(timeout=100))
    finally:
        for p in procs:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
    errs = [r for r in res if r[1] != "ok"]
    assert not errs, errs[0][2]
    (_, _, rep0, t0, _, ok0), (_, _, rep1, t1, _, ok1) = res
    assert t0 == t1 and rep0["table"] == rep1["table"]   # one table for the whole group
    assert rep0["sizes"] == [rows * 1024 * 2 for rows in (1, 2, 4, 8, 16, 32, 64, 128, 256)]
    assert set(rep0["us"]) == {"ll", "oneshot", "twoshot", "backend"} and ok0 == ok1 == 3
    assert rep0["table"][-1][0] == rep0["sizes"][-1]
