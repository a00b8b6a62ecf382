"""LLM generation engine: continuous batching over a paged KV cache with
hipGraph-captured decode steps.

* Admission reserves the pages a request can ever need (prompt + max_tokens),
  so a running request is never preempted; with 288 GB of HBM per GPU the
  reservation costs nothing in practice (Llama-3-8B: ~1.5M tokens of KV).
* Prefill runs over a packed multi-sequence batch, replayed from a captured graph of
  the smallest token bucket that holds it (``_PrefillGraph``; eager on the CPU).
* Decode steps for a batch padded to a bucket size (1, 2, 4, ... max_batch)
  are captured once per bucket as a hipGraph (torch.cuda.CUDAGraph) and
  replayed: embedding -> 32 x (norm, QKV GEMM, rope+KV write, paged attention,
  O GEMM, norm, gate|up GEMM, silu*mul, down GEMM) -> norm -> lm_head ->
  sampler, with every input at a fixed device address. Padded rows have
  context length 0 and slot -1 (no cache write, zero attention).
* Under tensor parallelism every rank of the TP group must receive the same
  requests in the same order; scheduling is deterministic, so ranks stay in
  lockstep without broadcasting decisions.
* Shared prompt prefixes: requests whose first whole KV pages hold the same tokens
  (every explanation prompt starts with the same instructions) map ONE set of pages,
  computed once, at the head of their block tables; their prefill computes only their
  own tokens, attending to the cached prefix K/V (``_SharedPrefix``).
"""
from __future__ import annotations

import contextlib
import gc
import itertools
import threading
import time
from collections import deque
from dataclasses import dataclass, field

import numpy as np
import torch

from operator_amd import ops
from operator_amd.models.kv_cache import PagedKVCache
from operator_amd.models.llama import ForwardBatch, LlamaModel
from operator_amd.utils.tracing import trace_range


def _launch_graph(graph: "torch.cuda.CUDAGraph", count: int, device) -> None:
    """Launch a captured graph ``count`` times on the current stream without holding
    the GIL (operator_amd._C.graph_launch; torch's replay() is the same hipGraphLaunch
    plus RNG bookkeeping that these graphs do not use)."""
    ops.kernels().graph_launch(graph.raw_cuda_graph_exec(), count, torch.cuda.current_stream(device).cuda_stream)


@dataclass(eq=False)  # identity semantics: two requests are never "equal"
class GenRequest:
    prompt: list[int]
    max_tokens: int = 500
    temperature: float = 0.3
    seed: int = 0
    ignore_eos: bool = False
    rid: int = -1
    # runtime state
    pages: list[int] = field(default_factory=list)
    prefix: "_SharedPrefix | None" = None   # shared prompt-prefix pages at the head of ``pages``
    output: list[int] = field(default_factory=list)
    done: bool = False
    cancelled: bool = False
    done_pending: bool = False     # EOS seen inside a multi-step window
    error: str | None = None
    t_submit: float = 0.0
    t_first: float = 0.0
    t_done: float = 0.0
    event: threading.Event = field(default_factory=threading.Event, repr=False)
    text: str | None = None        # detokenized output, filled by LLMEngine.finish_hook when set
    detok: bytearray | None = None  # streaming detokenization (LLMEngine.token_hook): bytes so far
    detok_pos: int = 0              # ... of output[:detok_pos]

    @property
    def length(self) -> int:
        return len(self.prompt) + len(self.output)


@dataclass
class EngineStats:
    prefill_tokens: int = 0
    decode_tokens: int = 0
    prefill_s: float = 0.0
    decode_s: float = 0.0
    steps: int = 0
    graph_replays: int = 0
    prefill_graph_replays: int = 0
    prefill_padded_tokens: int = 0   # bucket padding computed by prefill-graph replays
    prefill_eager: int = 0           # prefill batches run eagerly (no graphs, or above every bucket)
    prefix_hits: int = 0             # requests whose prompt started with the shared prefix
    prefix_tokens: int = 0           # ... prompt tokens they did not prefill
    prefix_builds: int = 0           # shared prefixes computed
    decode_launch_s: float = 0.0     # host time inside decode-window graph launches (a launch that
    decode_wait_s: float = 0.0       # ... blocks means the GPU queue is full) / waiting for windows
    decode_windows: int = 0          # decode windows launched
    decode_windows_ahead: int = 0    # ... of them queued behind the previous one (pipelined)
    no_pipeline: dict = field(default_factory=dict)   # why a window was not queued ahead


# Decode-window waits spin (the default event). Parking the engine thread in the driver
# (hipEventBlockingSync) measured slower on one MI355X box, 5-step flagship: blocking
# 29.37 / 29.25 vs spinning 29.43 / 29.44 analyses/s (profiles/blocking_wait_ab.txt), so
# the blocking variant was removed.


@dataclass
class _Window:
    """A launched multi-step decode window whose tokens are still on the device."""
    st: "_BucketState"
    reqs: list[GenRequest]
    B: int
    k: int
    host: torch.Tensor
    event: object
    s0: int = 0           # hist column of the window's first step (columns wrap mod multi_step)


def _prefill_bucket_sizes(max_tokens: int) -> list[int]:
    """Prefill graph buckets: every 512 tokens up to 4096, then steps of 1/4 of the
    power of two below (5k, 6k, 7k, 8k, 10k, ...), capped at ``max_tokens`` (always a
    bucket). A batch cut at bucket T (LLMEngine._prefill_cap) holds more than T minus
    one request, so it replays a graph padded by at most ~20 %; with power-of-two
    buckets and a 15 % padding rule, the batches cut at 2-4k tokens missed their bucket
    and ran eagerly (57 of 231 batches in the round-4 20-wave driver-shaped run, each
    ~400 launches under the operator threads' GIL contention)."""
    out, t = set(), 512
    while t < max_tokens:
        out.add(t)
        t += 512 if t < 4096 else (1 << (t.bit_length() - 1)) // 4
    out.add(max_tokens)
    return sorted(out)


# decode batch sizes with no bucket of their own: 9-64 rows run in the 64-row bucket. At 16 /
# 32 rows the bf16 decode GEMMs run on gemm_skinny (made for a few rows: it streams the
# weights once per 16-row tile): 5.2 / 6.8 ms per 8B token step against 4.9 ms for 64 rows
# on the gemm_decode / gemm_pp plans (profiles/decode_bucket32_r5.jsonl; open-loop p50 at
# 8 failures/s 3.89 -> 2.83 s). Padding rows cost nothing in attention (context 0) and
# little in the weight-streaming GEMMs. An engine whose max_batch is one of them keeps it.
SKIP_BUCKETS = (16, 32)


def _buckets(max_batch: int) -> list[int]:
    b, out = 1, []
    while b < max_batch:
        if not (b in SKIP_BUCKETS and max_batch > b):
            out.append(b)
        b *= 2
    out.append(max_batch)
    return out


class _BucketState:
    """Device-resident decode state of one batch bucket (shared by its graphs).

    One step = forward + sample + state advance (ids <- sampled token,
    pos/ctx += 1 on active rows, token appended to ``hist[:, step]``), so the
    host can replay several steps back-to-back and read ``hist`` once.
    Rows with ctx == 0 are padding: slot -1 (no KV write), zero attention.
    """

    def __init__(self, eng: "LLMEngine", bp: int):
        dev = eng.device
        self.bp = bp
        # the per-row state ``load`` rewrites lives in one byte buffer (one H2D copy per
        # batch-composition change instead of six)
        mp = eng.max_pages
        self._spec = (("step", (1,), torch.long), ("ids", (bp,), torch.long), ("pos", (bp,), torch.long),
                      ("seeds", (bp,), torch.long), ("ctx", (bp,), torch.int32), ("temp", (bp,), torch.float32),
                      ("bt", (bp, mp), torch.int32))
        self._nbytes = sum(int(np.prod(s)) * torch.empty((), dtype=dt).element_size() for _, s, dt in self._spec)
        self._buf = torch.zeros(self._nbytes, dtype=torch.uint8, device=dev)
        for n, t in self._views(self._buf).items():
            setattr(self, n, t)
        self.hist = torch.zeros(bp, eng.multi_step, dtype=torch.long, device=dev)
        # steps replayed since the last load: the device counter (``step``, bumped by every
        # replay; hist column = step % multi_step) mirrored on the host, so a window needs
        # no kernel to reset it (the one-element fill it replaced sat ~1 ms behind the previous
        # window's token copy on the GPU at every window boundary, round-4 flagship trace)
        self.step_host = 0
        self.slots = torch.zeros(bp, dtype=torch.long, device=dev)   # per step: cache slot of each row's token
        self.spos = torch.zeros(bp, dtype=torch.long, device=dev)    # per step: sampler stream position

    def _views(self, buf: torch.Tensor) -> dict:
        out, off = {}, 0
        for n, shape, dt in self._spec:   # 8-byte fields first, then 4-byte: every view aligned
            nb = int(np.prod(shape)) * torch.empty((), dtype=dt).element_size()
            out[n] = buf[off:off + nb].view(dt).view(shape)
            off += nb
        return out

    def load(self, reqs: list[GenRequest], max_pages: int) -> None:
        """Write the per-row state of ``reqs`` (rows beyond are padding). Built in numpy
        (one pass over the rows, no per-element tensor indexing: ~0.3 ms instead of
        ~10 ms for 256 rows at every batch-composition change) and copied in once."""
        n = len(reqs)
        host = torch.zeros(self._nbytes, dtype=torch.uint8)
        v = {k: t.numpy() for k, t in self._views(host).items()}
        ids, pos, ctx, bt, temp, seeds = v["ids"], v["pos"], v["ctx"], v["bt"], v["temp"], v["seeds"]
        assert bt.shape[1] == max_pages
        if n:
            lens = np.fromiter((r.length for r in reqs), dtype=np.int64, count=n)
            ids[:n] = np.fromiter((r.output[-1] for r in reqs), dtype=np.int64, count=n)
            pos[:n] = lens - 1
            ctx[:n] = lens
            temp[:n] = np.fromiter((r.temperature for r in reqs), dtype=np.float32, count=n)
            seeds[:n] = np.fromiter((r.seed for r in reqs), dtype=np.int64, count=n)
            for i, r in enumerate(reqs):
                bt[i, :len(r.pages)] = r.pages
        nb = self._buf.is_cuda
        self._buf.copy_(host.pin_memory() if nb else host, non_blocking=nb)   # step = 0
        self.step_host = 0


@contextlib.contextmanager
def _no_gc():
    """No Python garbage collection while a hipGraph is being captured. Recent PyTorch
    no longer collects on entering ``torch.cuda.graph``, so a collection triggered by
    an allocation inside the capture could free a dead cycle's GPU tensors there; a
    tensor used on another stream (the scan stream) then
    records an event on that stream mid-capture, which aborts the process. Dead
    cycles are collected first, then collection waits until the capture ends."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


class _DecodeGraph:
    """One decode step over a bucket's state, with ``splits`` decode-attention
    workgroups per (sequence, kv-head) (``ops.decode_splits``)."""

    def __init__(self, eng: "LLMEngine", st: _BucketState, splits: int):
        self.eng, self.st, self.splits = eng, st, splits
        self.graph: torch.cuda.CUDAGraph | None = None

    def _run(self) -> None:
        e, st = self.eng, self.st
        P = e.kv.page_size
        gpu = st.ids.is_cuda
        if gpu:   # one bookkeeping kernel before and one after the forward (norm_act.hip)
            ops.kernels().decode_slots(st.bt, st.pos, st.ctx, st.slots, st.spos, P)
            slots, spos = st.slots, st.spos
        else:
            act = st.ctx > 0
            pg = torch.gather(st.bt, 1, torch.clamp(st.pos // P, max=e.max_pages - 1).unsqueeze(1)).squeeze(1)
            slots = torch.where(act, pg.to(torch.long) * P + st.pos % P, torch.full_like(st.pos, -1))
            spos = st.pos + 1
        fb = ForwardBatch(st.ids, st.pos, slots, False, None, block_tables=st.bt, context_lens=st.ctx,
                          num_splits=self.splits)
        logits = e.model.forward(fb, e.kv)
        tok = e.model.sample(logits, st.temp, st.seeds, spos)
        if gpu:
            ops.kernels().decode_advance(tok, st.ids, st.hist, st.pos, st.ctx, st.step)
        else:
            st.ids.copy_(tok)
            st.hist.index_copy_(1, st.step % e.multi_step, tok.unsqueeze(1))   # wrap: a stray replay can never index past hist
            st.pos.add_(act.to(torch.long))
            st.ctx.add_(act.to(torch.int32))
            st.step.add_(1)

    def capture(self, pool) -> None:
        # warm up on a side stream (allocator + hipBLASLt heuristics), then capture; the
        # state is snapshotted and restored so capture never perturbs live rows
        st = self.st
        snap = [t.clone() for t in (st.ids, st.pos, st.ctx, st.step)]
        s = torch.cuda.Stream(device=self.eng.device)
        s.wait_stream(torch.cuda.current_stream())
        saved_ctx = st.ctx.clone()
        st.ctx.zero_()  # all rows padding while warming up: no KV writes
        with torch.cuda.stream(s):
            for _ in range(2):
                st.step.zero_()
                self._run()
        torch.cuda.current_stream().wait_stream(s)
        st.ctx.copy_(torch.zeros_like(saved_ctx))
        g = torch.cuda.CUDAGraph()
        with _no_gc(), torch.cuda.graph(g, pool=pool):
            self._run()
        self.graph = g
        for t, v in zip((st.ids, st.pos, st.ctx, st.step), snap):
            t.copy_(v)

    def run(self, use_graph: bool) -> None:
        if use_graph and self.graph is not None:
            self.graph.replay()
        else:
            self._run()


class _PrefillGraph:
    """A prefill of up to ``T`` packed tokens / ``S`` sequences captured as one
    hipGraph: embedding -> 32 layers (gemm_tile GEMMs with fused SwiGLU, norms,
    RoPE + KV write, flash prefill attention) -> last-token lm_head -> sampler.

    Why: an eager prefill is ~400 launches from the engine thread, each needing
    the GIL. At the start of a wave the operator's pipeline threads hold it for
    most of ~0.4 s (watch events, log collection, scan post-processing, prompt
    rendering) and the first prefill measured 1.9x its GPU time. Inputs live at
    fixed addresses: the real tokens are copied in, the tail is padding (id 0,
    slot -1: no KV write, no attention work item, logits discarded), unused
    attention work items are -1 (the kernel returns at once)."""

    def __init__(self, eng: "LLMEngine", T: int, S: int, variant: int, block_q: int):
        dev = eng.device
        self.eng, self.T, self.S, self.variant = eng, T, S, variant
        self.W = T // block_q + S               # work items: sum ceil(len / bq) <= T / bq + S
        i64, i32 = torch.long, torch.int32
        # every input is a view into ONE byte buffer, so a launch is one H2D copy (the
        # eleven separate copies it replaced each needed the GIL between them: with the
        # operator's threads holding it at a wave start, up to ~1.7 ms of GPU idle each,
        # profiles/bench_r4_flagship_idle.jsonl "copyBuffer -> copyBuffer")
        spec = (("ids", T, i64), ("pos", T, i64), ("slots", T, i64), ("last", S, i64), ("seeds", S, i64),
                ("spos", S, i64), ("cu", S + 1, i32), ("ws", self.W, i32), ("wq", self.W, i32),
                ("temp", S, torch.float32), ("pfx", S, i32))
        self._layout, off = [], 0
        for n, k, dt in spec:
            isz = torch.empty((), dtype=dt).element_size()
            self._layout.append((n, off, k, dt))
            off += (k * isz + 15) // 16 * 16
        self._nbytes = off
        self._dbuf = torch.zeros(off, dtype=torch.uint8, device=dev)
        self.dev = self._views(self._dbuf)
        # two pinned input sets + sampled-token buffers, used alternately: a launch
        # returns without waiting for the GPU, so the engine can queue the next
        # prefill batch before reading this one's tokens (LLMEngine._prefill); a set is
        # rewritten only after the event of its previous launch (two launches ago)
        self._hbufs = [torch.zeros(off, dtype=torch.uint8).pin_memory() for _ in range(2)]
        self.hosts = [self._views(b) for b in self._hbufs]
        self.outs = [torch.zeros(S, dtype=i64).pin_memory() for _ in range(2)]
        self.events: list = [None, None]
        self._i = 0
        self.graph: torch.cuda.CUDAGraph | None = None
        self.tok: torch.Tensor | None = None

    def _views(self, buf: torch.Tensor) -> dict:
        out = {}
        for n, off, k, dt in self._layout:
            isz = torch.empty((), dtype=dt).element_size()
            out[n] = buf[off:off + k * isz].view(dt)
        return out

    def _run(self) -> None:
        e, d = self.eng, self.dev
        pre = (e._pk, e._pv, d["pfx"], None) if e.prefix_sharing else None
        fb = ForwardBatch(d["ids"], d["pos"], d["slots"], True, d["last"], seq_lens=[],
                          prefill_work=(d["cu"], d["ws"], d["wq"], self.variant), prefix=pre)
        logits = e.model.forward(fb, e.kv)
        self.tok = e.model.sample(logits, d["temp"], d["seeds"], d["spos"])

    def capture(self, pool) -> None:
        # every work item padding and every slot -1 while warming up: no KV writes
        self.dev["slots"].fill_(-1)
        self.dev["ws"].fill_(-1)
        s = torch.cuda.Stream(device=self.eng.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._run()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with _no_gc(), torch.cuda.graph(g, pool=pool):
            self._run()
        self.graph = g

    def launch(self, ids, pos, slots, cu, ws, wq, last, temp, seeds, spos, pfx=None):
        """Queue one replay for the real batch (numpy inputs, <= T tokens, <= S
        sequences); returns (pinned token buffer, event): ``event`` completes when the
        batch's sampled first tokens are in the buffer."""
        i = self._i
        self._i ^= 1
        if self.events[i] is not None:
            self.events[i].synchronize()   # this set's copies (two launches ago) are done
        h = self.hosts[i]
        b = len(last)
        for name, arr, fill in (("ids", ids, 0), ("pos", pos, 0), ("slots", slots, -1), ("last", last, 0),
                                ("seeds", seeds, 0), ("spos", spos, 0), ("temp", temp, 0.0), ("ws", ws, -1),
                                ("wq", wq, 0), ("cu", cu, int(cu[-1])), ("pfx", pfx if pfx is not None else [], 0)):
            v = h[name].numpy()
            v[:len(arr)] = arr
            v[len(arr):] = fill
        self._dbuf.copy_(self._hbufs[i], non_blocking=True)
        _launch_graph(self.graph, 1, self.eng.device)
        out = self.outs[i]
        out[:b].copy_(self.tok[:b], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[i] = ev
        return out[:b], ev

    def run(self, *args) -> list[int]:
        """``launch`` and wait for the sampled tokens."""
        out, ev = self.launch(*args)
        ev.synchronize()
        return out.tolist()


class _SharedPrefix:
    """The first ``n`` prompt tokens (whole KV pages) many requests share: their KV pages,
    written once by a prefill of just these tokens and mapped at the head of every such
    request's block table (read-only: a request's own tokens start on its own pages), and
    their post-RoPE K/V per layer in ``LLMEngine._pk`` / ``_pv`` for the prefill attention
    of the requests' own tokens. Freed when replaced and no request holds it."""

    def __init__(self, tokens: tuple, pages: list[int]):
        self.tokens, self.pages, self.n = tokens, pages, len(tokens)
        self.users = 0
        self.retired = False


@dataclass
class _PendingPrefill:
    """A launched prefill batch whose first tokens are still on the device."""
    batch: list[GenRequest]
    toks: object          # list[int] (known) or a pinned tensor filled when ``event`` completes
    event: object
    t0: float
    tokens: int


class LLMEngine:
    # shared prompt prefixes: whole pages, at most PREFIX_MAX_TOKENS tokens, built once a
    # page-aligned prefix has been seen at the head of PREFIX_MIN_SEEN of the last
    # PREFIX_WINDOW prompts
    PREFIX_MAX_TOKENS = 256
    PREFIX_MIN_SEEN = 2
    PREFIX_WINDOW = 64

    def __init__(self, model: LlamaModel, kv: PagedKVCache, max_batch: int = 256, max_prefill_tokens: int = 16384,
                 max_context: int | None = None, use_graphs: bool = True, multi_step: int = 8,
                 admit_wait_s: float = 0.0, prefill_graphs: bool = True, prefix_sharing: bool = True):
        self.model, self.kv = model, kv
        # arrival batching window used by the loop that drives step() (EngineLoop):
        # an idle engine given less than a full prefill batch waits this long for more
        # requests. Not part of step() itself, which stays deterministic for TP.
        self.admit_wait_s = admit_wait_s
        # graph-captured prefill buckets (tokens): the largest is max_prefill_tokens; a
        # batch runs in the smallest bucket >= its tokens (_prefill_bucket_sizes: spaced
        # so the padding stays below one typical request / 20 %)
        self.prefill_graphs = use_graphs and model.device.type == "cuda" and prefill_graphs
        self.prefill_buckets = _prefill_bucket_sizes(max_prefill_tokens)
        self._prefill_g: dict[int, _PrefillGraph] = {}
        self._prefill_pool = None
        self.device = model.device
        self.max_batch = max_batch
        self.max_prefill_tokens = max_prefill_tokens
        self.max_context = min(max_context or model.cfg.max_position, model.cfg.max_position)
        self.max_pages = kv.pages_needed(self.max_context)
        if model.device.type == "cuda" and self.max_pages > 1024:   # attn_decode.hip kMaxPagesLds
            raise ValueError(f"max_context {self.max_context} needs {self.max_pages} KV pages of "
                             f"{kv.page_size} tokens per sequence (at most 1024): raise engine.page_size")
        self.hkv = model.hkv
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self.multi_step = max(1, multi_step)
        self._active: _BucketState | None = None   # bucket whose device state matches self.running
        self.waiting: deque[GenRequest] = deque()
        self.running: list[GenRequest] = []
        # the batch between _admit (pages allocated, off `waiting`) and its append to
        # `running`: abort_all must release it too if the prefill raises
        self._prefilling: list[GenRequest] = []
        # the last launched prefill batch, finished (first tokens read, rows joined to
        # `running`) only after the next batch is queued behind it or when no batch follows
        self._pf: _PendingPrefill | None = None
        self.stats = EngineStats()
        self._rid = itertools.count()
        self._graphs: dict[tuple[int, int], _DecodeGraph] = {}
        self._states: dict[int, _BucketState] = {}
        self._pool = None
        self.buckets = _buckets(max_batch)
        self.eos = set(model.cfg.eos_ids)
        # called with the requests a step finished, before their waiters wake (ExplainEngine
        # detokenizes a whole finished batch in one GIL-free call there)
        self.finish_hook = None
        # called with a decode window's requests once its tokens are appended, while the next
        # window runs on the GPU (ExplainEngine streams their bytes, so a finished wave's text
        # is ready without a detokenization pass on the critical path)
        self.token_hook = None
        self._lock = threading.Lock()
        # Decode windows are pipelined on the GPU: window w+1 is launched before the
        # host reads window w's tokens, so the device never idles on the host's
        # per-window bookkeeping (EOS rows of window w+1 are discarded).
        self.pipeline = self.use_graphs
        self._inflight: _Window | None = None
        self._hb = 0
        # called after every engine step; raise to fail the engine (e.g. a TP collective
        # that timed out: TPLLMEngine registers the one-shot all-reduce's check)
        self.health_checks: list = []
        self._host_bufs = None
        if self.device.type == "cuda":
            self._host_bufs = [torch.empty(max_batch, self.multi_step, dtype=torch.long, pin_memory=True)
                               for _ in range(2)]
        # shared prompt prefix: the GPU path needs the v3 / v4 prefill attention kernel; TP
        # followers replay the leader's admissions, so every rank builds the same prefix at
        # the same step (tests/test_tp_scale.py::test_tp_prefix_sharing_matches_tp1)
        self.prefix_sharing = prefix_sharing and (
            self.device.type != "cuda" or ops.prefill_variant(model.hq, model.hkv) in (3, 4))
        self._pfx: _SharedPrefix | None = None
        self._pfx_seen: deque = deque()
        self._pfx_count: dict = {}
        self._pfx_last: list = []   # the page-aligned prefixes of the last admitted prompt
        self._pk = self._pv = None
        if self.prefix_sharing:
            n = max(kv.page_size, self.PREFIX_MAX_TOKENS // kv.page_size * kv.page_size)
            shape = (model.cfg.layers, n, model.hkv, model.cfg.head_dim)
            self._pk = torch.zeros(shape, dtype=torch.bfloat16, device=self.device)
            self._pv = torch.zeros(shape, dtype=torch.bfloat16, device=self.device)

    # ------------------------------------------------------------------ API
    def submit(self, req: GenRequest) -> GenRequest:
        if not req.prompt:
            raise ValueError("empty prompt")
        if len(req.prompt) + req.max_tokens > self.max_context:
            req.max_tokens = max(1, self.max_context - len(req.prompt))
            if len(req.prompt) >= self.max_context:
                raise ValueError(f"prompt of {len(req.prompt)} tokens exceeds max_context {self.max_context}")
        with self._lock:
            req.rid = next(self._rid)
            req.t_submit = time.perf_counter()
            self.waiting.append(req)
        return req

    def cancel(self, req: GenRequest) -> None:
        """Cancel from any thread; the engine loop frees the pages at its next reap."""
        req.cancelled = True
        with self._lock:
            if req in self.waiting:
                self.waiting.remove(req)
                req.done = True
                req.error = "cancelled"
                req.event.set()

    def abort_all(self, reason: str) -> None:
        """Fail every queued and running request after a step raised (e.g. out of
        memory): their waiters are released with ``reason``, their KV pages go back to
        the allocator and the next step starts from a clean batch. Work the failed step
        left queued on the device is drained first, so no late kernel writes into pages
        that are handed out again (if the device itself is broken, that sync raises and
        the caller treats the engine as lost)."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        with self._lock:
            reqs = list({id(r): r for r in (*self.running, *self._prefilling, *self.waiting)}.values())
            self.running, self.waiting, self._prefilling = [], deque(), []
            self._pf = None
        for r in reqs:
            self._release(r)
            r.error = reason
            r.done = True
            r.event.set()
        self._inflight = None
        self._active = None

    @property
    def prefix_pages(self) -> int:
        """KV pages the current shared prompt prefix holds (outside any request)."""
        return len(self._pfx.pages) if self._pfx is not None else 0

    def _release(self, r: GenRequest) -> None:
        """Return a request's own KV pages; shared prefix pages stay with the prefix."""
        pf = r.prefix
        own = r.pages[len(pf.pages):] if pf is not None else r.pages
        if own:
            self.kv.allocator.release(own)
        r.pages = []
        if pf is not None:
            r.prefix = None
            pf.users -= 1
            if pf.retired and pf.users == 0:
                self.kv.allocator.release(pf.pages)

    # ------------------------------------------------------------------ shared prompt prefixes
    def _prefix_keys(self, prompt: list[int]) -> list[tuple]:
        """Page-aligned prompt prefixes a request could share (longest last), each leaving
        at least one token of its own to prefill (its logits sample the first output)."""
        P = self.kv.page_size
        k = min(self._pk.shape[1] // P, (len(prompt) - 1) // P)
        return [tuple(prompt[:j * P]) for j in range(1, k + 1)]

    def _note_prefix(self, prompt: list[int]) -> None:
        self._pfx_last = self._prefix_keys(prompt)
        for key in self._pfx_last:
            self._pfx_seen.append(key)
            self._pfx_count[key] = self._pfx_count.get(key, 0) + 1
        while len(self._pfx_seen) > self.PREFIX_WINDOW * (self._pk.shape[1] // self.kv.page_size):
            old = self._pfx_seen.popleft()
            c = self._pfx_count[old] - 1
            if c:
                self._pfx_count[old] = c
            else:
                del self._pfx_count[old]

    def _maybe_build_prefix(self) -> None:
        """Compute a shared prefix when the latest admitted prompt starts with a page-aligned
        prefix seen at the head of PREFIX_MIN_SEEN recent prompts (the longest such) that
        is not the one in place, and no request holds the current one. One eager prefill of
        just the prefix tokens writes its KV pages and hands each layer's K/V to
        ``_pk`` / ``_pv``."""
        best = None
        for key in self._pfx_last:
            if self._pfx_count.get(key, 0) >= self.PREFIX_MIN_SEEN:
                best = key   # keys are shortest first
        cur = self._pfx
        if best is None or (cur is not None and (cur.tokens == best or cur.users > 0)):
            return
        npages = len(best) // self.kv.page_size
        if npages + 1 > self.kv.allocator.free:
            return
        pages = self.kv.allocator.alloc(npages)
        n = len(best)
        dev = self.device
        P = self.kv.page_size
        slots = torch.tensor([pages[j // P] * P + j % P for j in range(n)], dtype=torch.long, device=dev)

        def sink(i, k, v):
            self._pk[i, :n].copy_(k.reshape(n, *self._pk.shape[2:]))
            self._pv[i, :n].copy_(v.reshape(n, *self._pv.shape[2:]))

        work = None
        if dev.type == "cuda":
            var = ops.prefill_variant(self.model.hq, self.model.hkv)
            ws, wq = ops.prefill_work_list([n], ops.prefill_block_q(self.model.hq, self.model.hkv, var))
            work = (torch.tensor([0, n], dtype=torch.int32, device=dev), torch.tensor(ws, dtype=torch.int32, device=dev),
                    torch.tensor(wq, dtype=torch.int32, device=dev), var)
        fb = ForwardBatch(torch.tensor(best, dtype=torch.long, device=dev), torch.arange(n, device=dev), slots, True,
                          torch.tensor([n - 1], dtype=torch.long, device=dev), seq_lens=[n], prefill_work=work,
                          kv_sink=sink)
        try:
            with trace_range(f"prefix[{n}]"):
                self.model.forward(fb, self.kv)
        except BaseException:
            # the pages belong to no request yet: _fail_all would never see them
            self.kv.allocator.release(pages)
            raise
        if cur is not None:
            cur.retired = True
            if cur.users == 0:
                self.kv.allocator.release(cur.pages)
        self._pfx = _SharedPrefix(best, pages)
        self.stats.prefix_builds += 1

    def _drop_idle_prefix(self) -> bool:
        """Release the shared prefix's pages when no request holds them (admission would
        otherwise turn a request away, or stall, for pages only the idle prefix occupies).
        It is rebuilt once its prompts come back."""
        cur = self._pfx
        if cur is None or cur.users > 0:
            return False
        cur.retired = True
        self.kv.allocator.release(cur.pages)
        self._pfx = None
        return True

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self._pf is not None)

    def idle(self) -> bool:
        """Nothing running or in flight on the device (the next step would be a prefill)."""
        return not self.running and self._inflight is None and self._pf is None

    def queued_prompt_tokens(self) -> int:
        """Prompt tokens waiting for admission that a prefill would compute (a prompt that
        starts with the shared prefix counts its own tokens only; stops counting at one
        full prefill batch)."""
        n = 0
        pf = self._pfx
        with self._lock:
            for r in self.waiting:
                n += len(r.prompt)
                if pf is not None and len(r.prompt) > pf.n and r.prompt[0] == pf.tokens[0] \
                        and tuple(r.prompt[:pf.n]) == pf.tokens:
                    n -= pf.n
                if n >= self.max_prefill_tokens:
                    break
        return n

    def generate(self, reqs: list[GenRequest]) -> list[GenRequest]:
        for r in reqs:
            self.submit(r)
        while any(not r.done for r in reqs):
            self.step()
        return reqs

    def warmup(self, buckets: list[int] | None = None, splits: list[int] | None = None) -> None:
        """Capture decode graphs ahead of time (largest first so they share one pool).
        ``splits`` defaults to every split count a bucket can use up to max_context."""
        if not self.use_graphs:
            return
        bs = sorted(buckets or self.buckets, reverse=True)
        for bp in bs:
            for ns in (splits or self.split_options(bp)):
                self._graph(bp, ns)
        if self.prefill_graphs:
            for T in sorted(self.prefill_buckets, reverse=True):
                self._prefill_graph(T)
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ scheduling
    def step(self) -> list[GenRequest]:
        self.stats.steps += 1
        if self._inflight is not None and (self._admittable() or not self.running):
            self._consume(self._inflight)   # composition is about to change: drain first
            self._inflight = None
            return self._reap()
        batch = self._admit() if self._inflight is None else []
        if batch:
            # launch this batch, then finish the previous one: its first tokens are read
            # while this batch is already queued on the GPU behind it (no host gap
            # between prefill batches)
            prev = self._pf
            self._pf = self._prefill(batch)
            if prev is not None:
                self._finish_prefill(prev)
        elif self._pf is not None:
            prev, self._pf = self._pf, None
            self._finish_prefill(prev)
        elif self.running:
            self._decode()
        for chk in self.health_checks:
            chk()
        return self._reap()

    def _rows(self) -> int:
        """Rows holding a decode slot: running + the launched, unfinished prefill batch."""
        return len(self.running) + (len(self._pf.batch) if self._pf is not None else 0)

    def _admittable(self) -> bool:
        return bool(self.waiting) and self._rows() < self.max_batch

    # a queue that pads its graph bucket by at most this many tokens is prefilled whole;
    # a larger pad (only above 4k tokens, where buckets are 1/4 octave apart) is cut at
    # the bucket below and the rest follows in the next batch
    PREFILL_MAX_PAD = 1024

    def _prefill_cap(self) -> int:
        """Token budget of the next prefill batch: a full batch (max_prefill_tokens)
        when that many prompt tokens wait; else everything queued when its graph bucket
        pads it by <= PREFILL_MAX_PAD tokens, else the largest bucket the queue fills (a
        batch padded by less than one request; the rest is queued behind it)."""
        # the admitted queue only (never a TP leader's not-yet-broadcast submissions):
        # every rank must cut the same batch
        q = LLMEngine.queued_prompt_tokens(self)
        if q >= self.max_prefill_tokens or not self.prefill_graphs:
            return self.max_prefill_tokens
        up = next(b for b in self.prefill_buckets if b >= q)
        if up - q <= self.PREFILL_MAX_PAD:
            return self.max_prefill_tokens
        fit = [b for b in self.prefill_buckets if b <= q]
        return fit[-1] if fit else self.max_prefill_tokens

    def _admit(self) -> list[GenRequest]:
        out, toks = [], 0
        rows = self._rows()
        cap = self._prefill_cap()
        if self.prefix_sharing and self._pfx_count:
            self._maybe_build_prefix()
        pf = self._pfx
        with self._lock:
            while self.waiting and rows + len(out) < self.max_batch:
                r = self.waiting[0]
                if r.cancelled:
                    self.waiting.popleft()
                    continue
                shared = (pf is not None and len(r.prompt) > pf.n and r.prompt[0] == pf.tokens[0]
                          and tuple(r.prompt[:pf.n]) == pf.tokens)
                own = len(r.prompt) - (pf.n if shared else 0)   # tokens this batch prefills for r
                if out and toks + own > cap:
                    break
                need = self.kv.pages_needed(len(r.prompt) + r.max_tokens) - (len(pf.pages) if shared else 0)
                if need > self.kv.allocator.free and not shared and self._drop_idle_prefix():
                    pf = None   # its pages were what stood in the way
                if need > self.kv.allocator.free:
                    if not rows and not out:
                        r.error = "KV cache too small for request"
                        r.done = True
                        self.waiting.popleft()
                        r.event.set()
                        continue
                    break
                r.pages = self.kv.allocator.alloc(need)
                if shared:
                    r.pages = pf.pages + r.pages
                    r.prefix = pf
                    pf.users += 1
                    self.stats.prefix_hits += 1
                    self.stats.prefix_tokens += pf.n
                if self.prefix_sharing:
                    self._note_prefix(r.prompt)
                self.waiting.popleft()
                out.append(r)
                self._prefilling = (self._pf.batch if self._pf is not None else []) + out
                toks += own
        return out

    def _prefill(self, batch: list[GenRequest]) -> _PendingPrefill:
        """Launch the prefill of ``batch``; ``_finish_prefill`` joins its rows."""
        pend = self._pf.batch if self._pf is not None else []
        self._prefilling = pend + batch
        with trace_range(f"prefill[{len(batch)}]"):
            return self._prefill_impl(batch)

    def _finish_prefill(self, pf: _PendingPrefill) -> None:
        """Read a launched batch's first tokens and join its rows to ``running``."""
        if pf.event is not None:
            pf.event.synchronize()
        toks = pf.toks.tolist() if isinstance(pf.toks, torch.Tensor) else pf.toks
        now = time.perf_counter()
        for r, tk in zip(pf.batch, toks):
            r.output.append(int(tk))
            r.t_first = now
            self.running.append(r)
        self._active = None  # new rows joined
        self._prefilling = self._pf.batch if self._pf is not None else []
        self.stats.prefill_tokens += pf.tokens
        self.stats.prefill_s += now - pf.t0

    def _prefill_impl(self, batch: list[GenRequest]) -> _PendingPrefill:
        t0 = time.perf_counter()
        dev = self.device
        # packed token ids / positions / cache slots built with numpy: this runs on the
        # engine thread between prefill batches, while the GPU waits for it
        P = self.kv.page_size
        # a request holding the shared prefix prefills only its own tokens (positions n..)
        skip = [r.prefix.n if r.prefix is not None else 0 for r in batch]
        full = [len(r.prompt) for r in batch]
        lens = [f - n for f, n in zip(full, skip)]
        ar = [np.arange(n, f, dtype=np.int64) for n, f in zip(skip, full)]
        ids = np.concatenate([np.asarray(r.prompt[n:], dtype=np.int64) for r, n in zip(batch, skip)])
        pos = np.concatenate(ar)
        slots = np.concatenate([np.asarray(r.pages, dtype=np.int64)[a // P] * P + a % P for r, a in zip(batch, ar)])
        cu = np.zeros(len(lens) + 1, dtype=np.int64)
        cu[1:] = np.cumsum(lens)
        pfx = skip if any(skip) else None
        last = cu[1:] - 1
        var = ops.prefill_variant(self.model.hq, self.model.hkv)
        ws, wq = ops.prefill_work_list(lens, ops.prefill_block_q(self.model.hq, self.model.hkv, var))
        temps = [r.temperature for r in batch]
        seeds = [r.seed for r in batch]
        g = self._prefill_graph_for(len(ids), len(batch))
        if g is not None:
            toks, ev = g.launch(ids, pos, slots, cu, ws, wq, last, temps, seeds, full, skip)
            self.stats.prefill_graph_replays += 1
            self.stats.prefill_padded_tokens += g.T - len(ids)
        else:
            self.stats.prefill_eager += 1
            t = lambda x, dt=torch.long: torch.as_tensor(np.asarray(x)).to(dtype=dt).to(dev, non_blocking=True)  # noqa: E731
            work = (t(cu, torch.int32), t(ws, torch.int32), t(wq, torch.int32), var) if dev.type == "cuda" else None
            pre = None if pfx is None else (self._pk, self._pv, t(pfx, torch.int32), pfx)
            fb = ForwardBatch(t(ids), t(pos), t(slots), True, t(last), seq_lens=lens, prefill_work=work, prefix=pre)
            logits = self.model.forward(fb, self.kv)
            tk = self.model.sample(logits, t(temps, torch.float32), t(seeds), t(full))
            if dev.type == "cuda":
                toks = torch.empty(len(batch), dtype=torch.long, pin_memory=True)
                toks.copy_(tk, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            else:
                toks, ev = tk.tolist(), None
        return _PendingPrefill(batch, toks, ev, t0, len(ids))

    def _prefill_graph(self, T: int) -> _PrefillGraph:
        g = self._prefill_g.get(T)
        if g is None:
            var = ops.prefill_variant(self.model.hq, self.model.hkv)
            g = _PrefillGraph(self, T, self.max_batch, var, ops.prefill_block_q(self.model.hq, self.model.hkv, var))
            if self._prefill_pool is None:   # its own pool: prefill and decode graphs never share memory
                self._prefill_pool = torch.cuda.graph_pool_handle()
            g.capture(self._prefill_pool)
            self._prefill_g[T] = g
        return g

    def _prefill_graph_for(self, tokens: int, seqs: int) -> _PrefillGraph | None:
        """Graph bucket for a prefill of ``tokens`` tokens: the smallest bucket that
        holds it (None: run eagerly)."""
        if not self.prefill_graphs or seqs > self.max_batch:
            return None
        for T in self.prefill_buckets:
            if T >= tokens:
                return self._prefill_graph(T)
        return None

    def _state(self, bp: int) -> _BucketState:
        st = self._states.get(bp)
        if st is None:
            st = self._states[bp] = _BucketState(self, bp)
        return st

    def split_options(self, bp: int) -> list[int]:
        top = ops.decode_splits(self.max_context, bp, self.hkv)
        return [1 << i for i in range(top.bit_length())]

    def _graph(self, bp: int, splits: int) -> _DecodeGraph:
        g = self._graphs.get((bp, splits))
        if g is None:
            g = _DecodeGraph(self, self._state(bp), splits)
            if self.use_graphs:
                if self._pool is None:
                    self._pool = torch.cuda.graph_pool_handle()
                g.capture(self._pool)
            self._graphs[(bp, splits)] = g
        return g

    def _launch(self, ahead: int = 0) -> _Window:
        """Launch one window of up to ``multi_step`` decode steps for ``self.running``;
        ``ahead`` tokens per request are already in flight in an earlier window."""
        reqs = list(self.running)
        B = len(reqs)
        bp = next(b for b in self.buckets if b >= B)
        k = max(1, min(self.multi_step, min(r.max_tokens - len(r.output) - ahead for r in reqs)))
        # decode-attention split count for the longest context reached in this window
        splits = ops.decode_splits(max(r.length for r in reqs) + ahead + k - 1, bp, self.hkv)
        g = self._graph(bp, splits)
        st = g.st
        if self._active is not st:
            assert ahead == 0, "device state must be current before it is reloaded"
            # rows longest context first: decode attention dispatches its workgroups in
            # row order, so the long rows start first and short ones fill the tail
            # (-3 % attention time at +-45 % context spread, tools/bench_attn.py --sort desc).
            # Deterministic (rid tie-break), so TP followers build the same order.
            self.running.sort(key=lambda r: (-r.length, r.rid))
            reqs = list(self.running)
            st.load(reqs, self.max_pages)
            self._active = st
        s0 = st.step_host % self.multi_step
        st.step_host += k
        with trace_range(f"decode[{bp}x{k}]"):
            if self.use_graphs and g.graph is not None:
                # the whole window from C++ with the GIL released: ROCm feeds a graph's
                # kernels from the launching thread, and Python-level replays beside
                # GIL-holding operator threads measured 2.2x slower per step
                # (tools/bench_graph_contention.py)
                t_l = time.perf_counter()
                _launch_graph(g.graph, k, self.device)
                self.stats.decode_launch_s += time.perf_counter() - t_l
            else:
                for _ in range(k):
                    g.run(False)
        if self._host_bufs is not None:
            self._hb ^= 1
            host = self._host_bufs[self._hb]
            host[:B].copy_(st.hist[:B], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = st.hist, None
        self.stats.graph_replays += k if self.use_graphs else 0
        self.stats.decode_windows += 1
        return _Window(st, reqs, B, k, host, ev, s0)

    def _consume(self, win: _Window) -> None:
        if win.event is not None:
            t_w = time.perf_counter()
            win.event.synchronize()
            self.stats.decode_wait_s += time.perf_counter() - t_w
        ms = self.multi_step
        if win.s0 + win.k <= ms:
            toks = win.host[:win.B, win.s0:win.s0 + win.k].tolist()
        else:   # the window's columns wrap
            toks = win.host[:win.B].numpy()[:, [(win.s0 + i) % ms for i in range(win.k)]].tolist()
        for r, row in zip(win.reqs, toks):
            if r.done:   # finished (EOS / cancel) in an earlier window: discard
                continue
            for tk in row:
                if r.done_pending:
                    break
                r.output.append(int(tk))
                if (not r.ignore_eos) and int(tk) in self.eos:
                    r.done_pending = True
        self.stats.decode_tokens += win.B * win.k
        if self.token_hook is not None:
            try:
                self.token_hook(win.reqs)
            except Exception:  # noqa: BLE001 - the finish hook / waiters decode from scratch
                self.token_hook = None

    def _decode(self) -> None:
        """Up to ``multi_step`` decode steps per window with no host round trip in
        between; the next window is queued behind the current one when the batch
        composition cannot change at the boundary."""
        t0 = time.perf_counter()
        prev = self._inflight or self._launch()
        self._inflight = None
        nxt = None
        same = len(prev.reqs) == len(self.running) and all(a is b for a, b in zip(prev.reqs, self.running))
        why = ("off" if not self.pipeline else "composition" if not same else "state" if self._active is not prev.st
               else "admit" if self._admittable()
               else "tail" if not all(r.max_tokens - len(r.output) - prev.k >= 1 for r in prev.reqs) else None)
        if why is None:
            nxt = self._launch(ahead=prev.k)
            self.stats.decode_windows_ahead += 1
        else:
            self.stats.no_pipeline[why] = self.stats.no_pipeline.get(why, 0) + 1
        self._consume(prev)
        self._inflight = nxt
        self.stats.decode_s += time.perf_counter() - t0

    def _reap(self) -> list[GenRequest]:
        fin, keep = [], []
        now = time.perf_counter()
        for r in self.running:
            hit_eos = r.done_pending or ((not r.ignore_eos) and r.output and r.output[-1] in self.eos)
            if r.cancelled:
                r.error = r.error or "cancelled"
            if len(r.output) >= r.max_tokens or hit_eos or r.cancelled:
                r.done = True
                r.t_done = now
                self._release(r)
                fin.append(r)
            else:
                keep.append(r)
        if fin:
            self._active = None  # batch composition changed: reload device state next step
            with trace_range(f"finish[{len(fin)}]"):
                if self.finish_hook is not None:
                    try:
                        self.finish_hook([r for r in fin if not r.cancelled])
                    except Exception:  # noqa: BLE001 - waiters fall back to their own detokenization
                        pass
                for r in fin:
                    r.event.set()
        self.running = keep
        return fin
