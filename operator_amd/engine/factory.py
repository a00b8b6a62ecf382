"""Construct the on-node engines from Settings (one process per GPU)."""
from __future__ import annotations

import logging
import os

import torch

from operator_amd.config import Settings
from operator_amd.patterns.schema import PatternSet

log = logging.getLogger(__name__)


def parse_model_spec(spec: str) -> tuple[str, str | None]:
    """``engine.extra_models`` entry -> (name, HF checkpoint dir or None)."""
    name, _, path = spec.partition("=")
    return name.strip(), (path.strip() or None)


def decode_message_sizes(hidden: int, max_batch: int) -> list[int]:
    """Bytes of the TP decode all-reduces: bf16 [rows, hidden] for every decode bucket
    row count (powers of two up to ``max_batch``)."""
    rows, out = 1, []
    while rows <= max(1, max_batch):
        out.append(rows * hidden * 2)
        rows *= 2
    return out


def calibrate_allreduce(tp, hidden: int, max_batch: int, iters: int = 20) -> dict:
    """Measure the IPC all-reduce protocols against RCCL on this node's TP group (collective;
    before any graph capture) and install the dispatch table; the report is kept on the group
    (``tp.oneshot.calibration``) for the bench JSON lines."""
    car = getattr(tp, "oneshot", None)
    if car is None or car.forced is not None:
        return {}
    rep = car.calibrate(decode_message_sizes(hidden, max_batch), iters=iters)
    log.info("TP all-reduce dispatch (world %d): %s", tp.world, rep.get("table"))
    return rep


def build_llm(s: Settings, device: str | torch.device | None = None, tp=None):
    """(model, kv, LLMEngine, Tokenizer) for the configured explanation model."""
    from operator_amd.engine.llm import LLMEngine
    from operator_amd.engine.tokenizer import Tokenizer, load_chat_template
    from operator_amd.models.config import config_from_hf, get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models import weight_cache
    from operator_amd.models.llama import LlamaModel

    e = s.engine
    dev = torch.device(device or e.device)
    # a checkpoint's own config.json defines the architecture (llama / mistral / qwen2)
    if e.model_path and os.path.exists(os.path.join(e.model_path, "config.json")):
        cfg = config_from_hf(e.model_path, name=e.model)
    else:
        cfg = get_config(e.model)
    dtype = getattr(torch, e.dtype)
    if tp is not None and tp.world > 1 and dev.type == "cuda" and e.oneshot_allreduce_mb > 0 \
            and getattr(tp, "oneshot", None) is None:
        if tp.enable_oneshot(dev, int(e.oneshot_allreduce_mb * (1 << 20)), int(max(e.oneshot_max_kb, 0) * 1024) or None) \
                and e.oneshot_max_kb <= 0:
            calibrate_allreduce(tp, cfg.hidden, e.max_batch, e.allreduce_calibrate_iters)
    model = LlamaModel(cfg, device=dev, tp=tp, dtype=dtype, weight_dtype=e.weight_dtype)
    weight_cache.load_or_build(model, e.weight_cache_dir, e.model_path, e.seed)
    # KV cache: the compute dtype, or OCP fp8 (e4m3fn, per-tensor scales) with engine.kv_dtype=fp8
    if e.kv_dtype not in ("auto", "fp8"):
        raise ValueError(f"engine.kv_dtype must be auto or fp8, not {e.kv_dtype!r}")
    kv_dtype = torch.float8_e4m3fn if e.kv_dtype == "fp8" else dtype
    pages = PagedKVCache.pages_for_budget(int(e.kv_cache_gb * 1e9), cfg.layers, model.hkv, cfg.head_dim,
                                          e.page_size, torch.finfo(kv_dtype).bits // 8)
    kv = PagedKVCache(cfg.layers, pages, model.hkv, cfg.head_dim, e.page_size, device=dev, dtype=kv_dtype,
                      k_scale=e.kv_scale, v_scale=e.kv_scale)
    kw = dict(max_batch=e.max_batch, max_prefill_tokens=e.max_prefill_tokens, max_context=e.max_context,
              use_graphs=e.use_graphs, multi_step=e.multi_step, admit_wait_s=e.admit_wait_ms / 1e3,
              prefill_graphs=e.prefill_graphs, prefix_sharing=e.prefix_sharing)
    if tp is not None and tp.world > 1:   # one replica over the TP group: lock-stepped engines
        from operator_amd.engine.tp import TPLLMEngine, control_group

        llm = TPLLMEngine(model, kv, tp_group=tp, ctrl_group=control_group(tp), **kw)
    else:
        llm = LLMEngine(model, kv, **kw)
    tok = Tokenizer(cfg.vocab_size, cfg.bos_id, cfg.eos_ids[0],
                    path=(f"{e.model_path}/tokenizer.json" if e.model_path else None), add_bos=cfg.add_bos,
                    chat_template=load_chat_template(e.chat_template, e.model_path))
    log.info("explanation model %s: %.1f GB weights, %d KV pages (%d tokens)", cfg.name,
             model.weight_bytes() / 1e9, pages, pages * e.page_size)
    return model, kv, llm, tok


def build_explain_service(s: Settings, metrics=None, tp=None):
    from operator_amd.engine import service

    kind = s.services.explain
    if kind == "none":
        return None
    if kind == "echo":
        return service.EchoExplainService()
    if kind == "remote":
        return service.RemoteAIInterface(s.services.ai_interface_url, s.services.ai_interface_read_timeout_s,
                                         s.services.ai_interface_connect_timeout_s)
    from operator_amd.engine.explain import ExplainEngine

    extra = [parse_model_spec(x) for x in s.engine.extra_models] if (tp is None or tp.world == 1) else []

    def warm(llm):
        # capture the decode / prefill graphs now, before the controller starts watching:
        # a lazy capture mid-wave stalls the engine loop and runs under the global capture
        # mode while the scan thread issues GPU work (as the pool worker does, pool.py)
        if s.engine.warmup_graphs and (tp is None or tp.world == 1):
            llm.warmup()

    if not extra:
        _, _, llm, tok = build_llm(s, tp=tp)
        warm(llm)
        ee = ExplainEngine(llm, tok, model_id=s.engine.model, max_prompt_tokens=s.engine.max_prompt_tokens,
                           ignore_eos=s.engine.ignore_eos)
        return service.LocalExplainService(ee, metrics)
    # several local models: each its own engine (weights, paged KV cache, graphs, loop
    # thread) with an equal share of the KV budget; AIProviders pick one by modelId
    services = {}
    for name, path in [(s.engine.model, s.engine.model_path)] + extra:
        sm = s.model_copy(deep=True)
        sm.engine.model, sm.engine.model_path = name, path
        sm.engine.kv_cache_gb = s.engine.kv_cache_gb / (1 + len(extra))
        _, _, llm, tok = build_llm(sm, tp=tp)
        warm(llm)
        ee = ExplainEngine(llm, tok, model_id=name, max_prompt_tokens=s.engine.max_prompt_tokens,
                           ignore_eos=s.engine.ignore_eos)
        services[name] = service.LocalExplainService(ee, metrics)
    return service.MultiModelExplainService(services, default=s.engine.model)


def build_match_engine(s: Settings, patterns: PatternSet, device: str | None = None):
    from operator_amd.engine.match import MatchEngine

    dev = device or (s.engine.device if s.services.match == "local" else "cpu")
    if dev.startswith("cuda") and not torch.cuda.is_available():
        raise RuntimeError("services.match=local needs a GPU; use services.match=cpu without one")
    return MatchEngine(patterns, device=dev, seg_bytes=s.patterns.seg_bytes, max_events=s.patterns.max_events,
                       significance=s.patterns.significance_threshold)


def build_match_service(s: Settings, patterns: PatternSet, metrics=None):
    from operator_amd.engine import service

    if s.services.match == "remote":
        return service.RemoteLogParser(s.services.log_parser_url, s.services.log_parser_read_timeout_s,
                                       s.services.log_parser_connect_timeout_s)
    if s.services.match == "stub":
        return service.StubMatchService()
    return service.LocalMatchService(build_match_engine(s, patterns), s.services.match_max_batch,
                                     s.services.match_batch_wait_ms, metrics)
