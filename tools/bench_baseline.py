"""Reference-shaped "before" measurement (BASELINE.md "What we will measure instead").

The reference publishes no numbers; its compute lives in two external REST
services (a CPU regex log-parser and an LLM behind ai-interface). This tool
measures that shape on the same MI355X with the same synthetic workload as
``bench.py``:

* pattern analysis: pure-Python ``re`` per pattern over the log lines
  (``operator_amd.patterns.oracle`` — the semantics our GPU scan is tested
  against), one failure at a time, as a CPU log-parser would;
* explanation: HuggingFace ``transformers`` ``LlamaForCausalLM`` (eager
  PyTorch, SDPA attention, dynamic KV cache, ``generate``) with random-init
  Llama-3-8B weights in bf16, static batches of ``--hf-batch`` prompts,
  ``max_tokens`` new tokens at temperature 0.3 (EOS ignored, as in bench.py).

Prints one JSON line: analyses/s and p50 latency for that path.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--failures", type=int, default=64)
    ap.add_argument("--hf-batch", type=int, default=64)
    ap.add_argument("--max-tokens", type=int, default=500)
    ap.add_argument("--prompt-tokens", type=int, default=1024)
    ap.add_argument("--log-kb", type=int, default=64)
    ap.add_argument("--patterns", type=int, default=1000)
    ap.add_argument("--model", default="llama3-8b")
    a = ap.parse_args()

    import torch
    from transformers import LlamaConfig as HFConfig
    from transformers import LlamaForCausalLM

    from operator_amd.engine.match import MatchEngine
    from operator_amd.engine.prompt import render_bounded
    from operator_amd.engine.tokenizer import Tokenizer
    from operator_amd.models.config import get_config
    from operator_amd.patterns import oracle
    from operator_amd.patterns.compiler import compile_patterns
    from operator_amd.patterns.synth import LogFactory, synthetic_library

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    ps = synthetic_library(a.patterns, seed=0)
    fac = LogFactory(n_patterns=a.patterns, seed=0)
    docs, _ = fac.batch(a.failures, a.log_kb * 1024, n_failures=3, seed=1000)
    cp = compile_patterns(ps, build_dfa=False)
    cfg = get_config(a.model)
    tok = Tokenizer(cfg.vocab_size, cfg.bos_id, cfg.eos_ids[0])
    meng = MatchEngine(ps, device="cpu")
    results = meng.analyze(docs, [(f"app-{i}", "default") for i in range(len(docs))])
    prompts = [render_bounded(r, tok, a.prompt_tokens) for r in results]

    hfc = HFConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden, intermediate_size=cfg.intermediate,
                   num_hidden_layers=cfg.layers, num_attention_heads=cfg.heads, num_key_value_heads=cfg.kv_heads,
                   max_position_embeddings=8192, rope_theta=cfg.rope_theta, rms_norm_eps=cfg.rms_eps,
                   tie_word_embeddings=False, attn_implementation="sdpa", pad_token_id=0)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        model = LlamaForCausalLM(hfc)
    model.eval()

    # ---- timed: per-failure regex analysis + batched HF generate ----
    lat = []
    t0 = time.perf_counter()
    for d in docs:
        oracle.analyze_docs(cp, [d])
    t_match = time.perf_counter() - t0
    for i in range(0, len(prompts), a.hf_batch):
        chunk = prompts[i:i + a.hf_batch]
        L = max(map(len, chunk))
        ids = torch.zeros(len(chunk), L, dtype=torch.long)
        mask = torch.zeros(len(chunk), L, dtype=torch.long)
        for j, p in enumerate(chunk):
            ids[j, L - len(p):] = torch.tensor(p)
            mask[j, L - len(p):] = 1
        with torch.no_grad():
            model.generate(ids.to(dev), attention_mask=mask.to(dev), max_new_tokens=a.max_tokens,
                           min_new_tokens=a.max_tokens, do_sample=True, temperature=0.3, top_k=0, top_p=1.0)
        if dev == "cuda":
            torch.cuda.synchronize()
        now = time.perf_counter() - t0
        lat += [now] * len(chunk)
    el = time.perf_counter() - t0
    print(json.dumps({"bench": "reference-shaped baseline", "model": a.model, "failures": a.failures,
                      "hf_batch": a.hf_batch, "max_tokens": a.max_tokens,
                      "prompt_tokens_mean": round(sum(map(len, prompts)) / len(prompts), 1),
                      "match_s": round(t_match, 2), "total_s": round(el, 2),
                      "analyses_per_s": round(a.failures / el, 3),
                      "p50_latency_ms": round(statistics.median(lat) * 1e3, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
