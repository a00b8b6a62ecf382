"""Explanation service: AnalysisResult + AIProviderConfig -> AIResponse.

On-node replacement for the reference's ai-interface hop
(POST /api/v1/analysis/analyze, J/service/AIInterfaceRestClient.java:37-39;
request built in J/service/AIInterfaceClient.java:45-59). Semantics kept from
the AIProvider contract (aiprovider-crd.yaml; defaults 30 s / 3 retries /
caching on / 500 tokens / T=0.3 per AIInterfaceClient.java:78-84):

* ``maxTokens``      -> generation length cap
* ``temperature``    -> sampler temperature (0 = greedy)
* ``timeoutSeconds`` -> per-attempt deadline; the request is cancelled (its KV
                        pages freed) and retried up to ``maxRetries`` times
* ``cachingEnabled`` -> LRU of responses keyed by (model, prompt, T, maxTokens)
* ``promptTemplate`` -> operator_amd.engine.prompt.render

Requests from any number of threads are batched continuously by one engine
loop thread that owns the GPU (LLMEngine.step).
"""
from __future__ import annotations

import hashlib
import sys
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass

import torch

from operator_amd.api.models import AIProviderConfig, AIResponse, AnalysisResult

from operator_amd.parallel.custom_ar import CollectiveTimeout

from . import prompt as prompt_mod
from .llm import GenRequest, LLMEngine


class ExplainError(RuntimeError):
    pass


class EngineLoop(threading.Thread):
    """Owns the LLMEngine; steps it whenever requests are pending."""

    def __init__(self, llm: LLMEngine):
        super().__init__(name="llm-engine-loop", daemon=True)
        self.llm = llm
        self._cv = threading.Condition()
        self._stopping = False
        self.error: BaseException | None = None
        self.fatal: BaseException | None = None

    def notify(self) -> None:
        with self._cv:
            self._cv.notify()

    def stop(self) -> None:
        with self._cv:
            self._stopping = True
            self._cv.notify()

    # GIL hand-off interval while this thread feeds the GPU: at CPython's default
    # (5 ms) every kernel-launch burst of a prefill step can wait that long behind the
    # operator's worker threads, leaving the GPU idle (measured: ~0.3-0.5 s of idle
    # per 256-failure wave). 0.5 ms bounds that wait at a small context-switch cost.
    GIL_SWITCH_S = 0.0005

    def _gather_arrivals(self) -> None:
        """Failures arrive in bursts that the pipeline feeds to the engine over tens of
        ms (scan batches, prompt batches). An idle engine that admitted the first
        arrival alone would run a 1-request prefill and queue everything behind it
        (measured at the start of a 256-failure wave: a 1-request prefill stretched to
        174 ms by the launch-side GIL contention of the burst, ahead of the first full
        batch). So when idle, wait up to ``admit_wait_s`` for half a prefill batch; while
        a prefill batch runs, queue the next one once a full batch waits or the running
        one is done (prefill batches are pipelined: LLMEngine.step)."""
        llm = self.llm
        wait = getattr(llm, "admit_wait_s", 0.0)
        if wait <= 0:
            return
        full = llm.max_prefill_tokens
        if llm.idle():
            # half a batch starts the first prefill (LLMEngine._prefill_cap cuts it at a
            # full graph bucket); the rest of the burst queues behind it
            deadline = time.perf_counter() + wait
            while (not self._stopping and time.perf_counter() < deadline
                   and llm.queued_prompt_tokens() < full // 2):
                time.sleep(0.001)
            return
        pf = getattr(llm, "_pf", None)
        ev = getattr(pf, "event", None)
        if ev is None or not llm.waiting:
            return
        # a prefill batch is still running on the GPU: queue the next one behind it only
        # once a full batch waits, or when the GPU is about to need it (the running batch
        # is done), instead of cutting the arrivals into small, padded batches
        deadline = time.perf_counter() + 1.0
        while (not self._stopping and time.perf_counter() < deadline and not ev.query()
               and llm.queued_prompt_tokens() < full):
            time.sleep(0.0002)

    def run(self) -> None:
        if self.llm.device.type == "cuda":
            if self.llm.device.index is not None:   # "cuda" alone: the thread's default device
                torch.cuda.set_device(self.llm.device)
            if sys.getswitchinterval() > self.GIL_SWITCH_S:
                sys.setswitchinterval(self.GIL_SWITCH_S)
        while True:
            with self._cv:
                while not self._stopping and not self.llm.has_work():
                    self._cv.wait(timeout=0.5)
                if self._stopping:
                    close = getattr(self.llm, "close", None)
                    if close is not None:   # TP leader: release the followers
                        close()
                    return
            self._gather_arrivals()
            try:
                self.llm.step()
            except BaseException as e:  # surface to every waiter
                self.error = e
                fatal = getattr(e, "fatal", False) or isinstance(e, CollectiveTimeout)
                if not fatal:
                    try:   # release the failed batch's KV pages so the engine keeps serving
                        self.llm.abort_all(f"engine failure: {e}")
                        continue
                    except BaseException as e2:  # noqa: BLE001 - the device is gone: stop serving
                        fatal, e = True, e2
                # the replica's device state is inconsistent (e.g. a TP peer never arrived:
                # no device sync, it could wait forever): fail every waiter and stop
                # serving; the pool worker exits and is respawned
                for r in (list(self.llm.running) + list(getattr(self.llm, "_prefilling", []))
                          + list(self.llm.waiting)):
                    r.error = f"engine failure: {e}"
                    r.done = True
                    r.event.set()
                self.llm.running.clear()
                self.llm.waiting.clear()
                if hasattr(self.llm, "_prefilling"):
                    self.llm._prefilling = []
                if hasattr(self.llm, "_pf"):
                    self.llm._pf = None
                self.fatal = e
                return


@dataclass
class _Pending:
    req: GenRequest
    key: str | None
    cfg: AIProviderConfig
    t0: float
    attempt: int = 0


class PromptBatcher(threading.Thread):
    """Coalesces prompt building of concurrent ``explain()`` callers.

    The pipeline calls ``explain`` from one worker thread per failure; building
    each prompt there (render + shrink-ladder tokenization, ~2-4 ms of
    GIL-holding ``encode`` per prompt at 1k tokens) starved the engine-loop
    thread that launches the GPU work. Callers instead enqueue and wait; this
    thread takes everything queued (after ``wait_s`` for stragglers) and
    tokenizes it with ``render_bounded_batch`` (Rust ``encode_batch``, GIL
    released, parallel). ``build_many`` returns each caller's result, or an exception
    for that caller alone; ExplainEngine's also submits the batch's requests to the
    engine here, so a burst reaches the engine in whole batches instead of one
    request per waiter thread as each wakes (~20 ms of a wave's start under the GIL)."""

    def __init__(self, build_many, wait_s: float = 0.002, max_batch: int = 32):
        super().__init__(name="prompt-batcher", daemon=True)
        import queue as _queue

        self.build_many, self.wait_s, self.max_batch = build_many, wait_s, max_batch
        self.q: _queue.Queue = _queue.Queue()
        self._empty = _queue.Empty

    def build(self, result: AnalysisResult, cfg: AIProviderConfig):
        from concurrent.futures import Future

        f: Future = Future()
        self.q.put((result, cfg, f))
        r = f.result()
        if isinstance(r, BaseException):
            raise r
        return r

    def stop(self) -> None:
        self.q.put(None)

    def run(self) -> None:
        while True:
            item = self.q.get()
            if item is None:
                return
            batch = [item]
            deadline = time.perf_counter() + self.wait_s
            while len(batch) < self.max_batch:
                try:
                    nxt = self.q.get(timeout=max(0.0, deadline - time.perf_counter()))
                except self._empty:
                    break
                if nxt is None:
                    self.q.put(None)
                    break
                batch.append(nxt)
            try:
                ids = self.build_many([(r, c) for r, c, _ in batch])
                for (_, _, f), x in zip(batch, ids):
                    f.set_result(x)
            except BaseException as e:  # noqa: BLE001 - delivered to every caller
                for _, _, f in batch:
                    if not f.done():
                        f.set_exception(e)


class ExplainEngine:
    def __init__(self, llm: LLMEngine, tokenizer, model_id: str = "local", max_prompt_tokens: int = 1024,
                 cache_size: int = 4096, ignore_eos: bool = False, start_loop: bool = True):
        self.llm, self.tok = llm, tokenizer
        self.model_id = model_id
        self.max_prompt_tokens = max_prompt_tokens
        self.ignore_eos = ignore_eos
        self._cache: OrderedDict[str, AIResponse] = OrderedDict()
        self._cache_size = cache_size
        self._lock = threading.Lock()
        self.loop = EngineLoop(llm)
        if hasattr(tokenizer, "decode_batch"):
            llm.finish_hook = self._detokenize
        # byte-level BPE: stream each request's bytes per decode window (exact: checked by
        # Tokenizer.byte_table), so finishing a wave only UTF-8-decodes 256 buffers
        self._stream = hasattr(tokenizer, "byte_table") and tokenizer.byte_table() is not None
        if self._stream:
            llm.token_hook = self._feed
        self.prompts = PromptBatcher(self._batch_build)
        self.prompts.start()
        if start_loop:
            self.loop.start()

    def close(self, join_s: float = 0.0) -> None:
        self.prompts.stop()
        self.loop.stop()
        if join_s and self.loop.is_alive():
            self.loop.join(join_s)

    # ------------------------------------------------------------------ helpers
    def build_prompt(self, result: AnalysisResult, cfg: AIProviderConfig) -> list[int]:
        return prompt_mod.render_bounded(result, self.tok, self.max_prompt_tokens, cfg.prompt_template)

    def build_prompts(self, items: list[tuple[AnalysisResult, AIProviderConfig]]) -> list[list[int]]:
        from operator_amd.utils.tracing import trace_range

        with trace_range(f"prompts[{len(items)}]"):
            return prompt_mod.render_bounded_batch([(r, c.prompt_template) for r, c in items], self.tok,
                                                   self.max_prompt_tokens)

    def _key(self, ids: list[int], cfg: AIProviderConfig) -> str:
        h = hashlib.sha256()
        h.update(f"{cfg.model_id}|{cfg.temperature}|{cfg.max_tokens}|".encode())
        h.update(bytes(str(ids), "ascii"))
        return h.hexdigest()

    def _feed(self, reqs: list[GenRequest]) -> None:
        """Engine-loop hook after each decode window: append the window's token bytes."""
        feed = self.tok.feed
        for r in reqs:
            if r.detok is None:
                r.detok = bytearray()
            if r.detok_pos < len(r.output):
                feed(r.detok, r.output[r.detok_pos:])
                r.detok_pos = len(r.output)

    def _detokenize(self, reqs: list[GenRequest]) -> None:
        """Engine-loop hook: the text of every request a step finished, before their
        waiters wake (256 waiters each detokenizing 500 tokens under the GIL held up the
        hand-off of a finished wave): the streamed bytes' UTF-8 text (byte-level BPE) or
        one decode_batch call."""
        if not reqs:
            return
        if self._stream:
            self._feed(reqs)
            for r in reqs:
                r.text = self.tok.text_of(r.detok)
            return
        for r, t in zip(reqs, self.tok.decode_batch([r.output for r in reqs])):
            r.text = t

    def _seed(self, ids: list[int]) -> int:
        return int(hashlib.sha1(bytes(str(ids), "ascii")).hexdigest()[:8], 16)

    def _start(self, p: _Pending, ids: list[int], notify: bool = True) -> None:
        cfg = p.cfg
        p.req = GenRequest(ids, max_tokens=max(1, int(cfg.max_tokens)), temperature=float(cfg.temperature),
                           seed=self._seed(ids) + p.attempt, ignore_eos=self.ignore_eos)
        self.llm.submit(p.req)
        if notify:
            self.loop.notify()

    def _batch_build(self, items: list[tuple[AnalysisResult, AIProviderConfig]]) -> list:
        ids = self.build_prompts(items)
        return self._admit_many(items, ids)

    def _admit_many(self, items: list[tuple[AnalysisResult, AIProviderConfig]],
                    prompts: list[list[int]]) -> list[_Pending | AIResponse | BaseException]:
        """Cache lookups and engine submission for a batch of built prompts, one engine
        wake-up for the batch; an item's own failure (e.g. a prompt the engine cannot
        hold) is returned in its slot."""
        out: list[_Pending | AIResponse | BaseException] = []
        for (res, cfg), ids in zip(items, prompts):
            try:
                key = self._key(ids, cfg) if cfg.caching_enabled else None
                if key is not None:
                    with self._lock:
                        hit = self._cache.get(key)
                        if hit is not None:
                            self._cache.move_to_end(key)
                            out.append(hit.model_copy(update={"cached": True}))
                            continue
                p = _Pending(None, key, cfg, time.perf_counter())  # type: ignore[arg-type]
                p.ids = ids  # type: ignore[attr-defined]
                self._start(p, ids, notify=False)
                out.append(p)
            except Exception as e:  # noqa: BLE001 - delivered to this item's caller
                out.append(e)
        self.loop.notify()
        return out

    # ------------------------------------------------------------------ API
    def explain_many(self, items: list[tuple[AnalysisResult, AIProviderConfig]]) -> list[AIResponse | ExplainError]:
        """Explain a batch concurrently (continuous batching); per-item errors are returned, not raised
        (except a failure to admit a single coalesced item, raised as before)."""
        if len(items) == 1 and self.prompts.is_alive():   # one caller of many: coalesced with the others
            pend = [self.prompts.build(*items[0])]
        else:
            pend = self._admit_many(items, self.build_prompts(items))
        if len(pend) == 1 and isinstance(pend[0], BaseException):
            raise pend[0]
        # several items: the ones admitted are already generating, so a failed admission is
        # that item's ExplainError and every other item is still waited for (raising here
        # would leave their requests decoding to max_tokens with no waiter)
        out: list[AIResponse | ExplainError] = []
        for p in pend:
            if isinstance(p, BaseException):
                out.append(p if isinstance(p, ExplainError) else ExplainError(str(p) or type(p).__name__))
                continue
            if not isinstance(p, _Pending):
                out.append(p)
                continue
            out.append(self._wait(p))
        return out

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        r = self.explain_many([(result, cfg)])[0]
        if isinstance(r, ExplainError):
            raise r
        return r

    def _wait(self, p: _Pending) -> AIResponse | ExplainError:
        cfg = p.cfg
        while True:
            deadline = max(0.001, float(cfg.timeout_seconds or 30))
            ok = p.req.event.wait(timeout=deadline)
            err = None
            if not ok:
                self.llm.cancel(p.req)
                err = f"explanation timed out after {cfg.timeout_seconds}s"
            elif p.req.error:
                err = p.req.error
            if err is None:
                break
            if p.attempt >= int(cfg.max_retries or 0):
                return ExplainError(f"{err} (after {p.attempt + 1} attempt(s))")
            p.attempt += 1
            self._start(p, p.ids)  # type: ignore[attr-defined]
        r = p.req
        text = r.text if r.text is not None else self.tok.decode(r.output)
        resp = AIResponse(explanation=text, provider_id=cfg.provider_id or "local", model_id=cfg.model_id or self.model_id,
                          tokens_generated=len(r.output), latency_ms=round((r.t_done - p.t0) * 1e3, 3), cached=False,
                          prompt_tokens=len(r.prompt), queue_ms=round((r.t_first - p.t0) * 1e3, 3),
                          decode_ms=round((r.t_done - r.t_first) * 1e3, 3))
        if p.key is not None:
            with self._lock:
                self._cache[p.key] = resp
                while len(self._cache) > self._cache_size:
                    self._cache.popitem(last=False)
        return resp

    # ------------------------------------------------------------------ raw completions
    def complete(self, ids: list[int], max_tokens: int = 500, temperature: float = 0.3, seed: int | None = None,
                 timeout_s: float | None = None) -> dict:
        """Generate from raw prompt token ids on the same continuous batch as the
        explanations (the OpenAI / Ollama endpoints of engine/server.py). Raises
        ExplainError on a timeout, an engine error or a prompt the engine cannot hold."""
        req = GenRequest(list(ids), max_tokens=max(1, int(max_tokens)), temperature=max(0.0, float(temperature)),
                         seed=self._seed(ids) if seed is None else int(seed), ignore_eos=self.ignore_eos)
        want = req.max_tokens
        t0 = time.perf_counter()
        try:
            self.llm.submit(req)
        except ValueError as e:
            raise ExplainError(str(e)) from None
        self.loop.notify()
        if not req.event.wait(timeout=timeout_s if timeout_s else None):
            self.llm.cancel(req)
            raise ExplainError(f"completion timed out after {timeout_s}s")
        if req.error:
            raise ExplainError(req.error)
        return {"text": req.text if req.text is not None else self.tok.decode(req.output),
                "prompt_tokens": len(req.prompt),
                "completion_tokens": len(req.output),
                "finish_reason": "length" if len(req.output) >= min(want, req.max_tokens) else "stop",
                "latency_ms": round((req.t_done - t0) * 1e3, 3)}
