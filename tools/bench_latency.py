"""Open-loop latency benchmark (BASELINE configs 3/4: p50/p99 explanation latency).

bench.py measures throughput with waves of simultaneous failures; a real cluster
sees failures arrive one by one. Here failed pods arrive as a Poisson process at
each ``--rates`` value (per second) for ``--seconds`` (after ``--warmup-s`` of the
same load), each through the full operator path (FakeKube watch -> collect -> GPU
scan -> prompt -> Llama explanation on the continuous-batching engine ->
annotations, status ring, Events). Reported per rate: achieved analyses/s and the
p50 / p90 / p99 latency from the failed pod being written to the API server to its
analysis being stored. Synthetic logs, random-init weights, generation runs to
``--max-tokens`` (AIProvider default 500). One JSON line per rate.
"""
import argparse
import json
import os
import random
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, max(0, int(round(p / 100.0 * (len(xs) - 1)))))] if xs else float("nan")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="2,8,16")
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--warmup-s", type=float, default=5.0)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--max-tokens", type=int, default=500)
    ap.add_argument("--prompt-tokens", type=int, default=1024)
    ap.add_argument("--log-kb", type=int, default=64)
    ap.add_argument("--patterns", type=int, default=1000)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--kv-gb", type=float, default=96.0)
    ap.add_argument("--seed", type=int, default=5, help="arrival process seed (one per shard)")
    ap.add_argument("--dump-lat", default=None, help="write each rate's raw latencies (s) to this JSON file")
    ap.add_argument("--start-at", type=float, default=0.0,
                    help="time.time() to start the first rate at (aligns shard processes)")
    a = ap.parse_args()

    import torch

    from operator_amd.config import load_settings
    from operator_amd.controller.operator import Operator
    from operator_amd.engine.explain import ExplainEngine
    from operator_amd.engine.factory import build_llm
    from operator_amd.engine.match import MatchEngine
    from operator_amd.engine.service import LocalExplainService, LocalMatchService
    from operator_amd.kube.fake import FakeKube, failed_pod, running_pod
    from operator_amd.kube.resources import AIPROVIDERS, PODMORTEMS, PODS
    from operator_amd.patterns.synth import LogFactory, synthetic_library

    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    s = load_settings(env={}, overrides={
        "engine.model": a.model, "engine.device": dev, "engine.max_batch": a.max_batch,
        "engine.max_context": a.prompt_tokens + a.max_tokens + 64, "engine.max_prompt_tokens": a.prompt_tokens,
        "engine.kv_cache_gb": a.kv_gb if dev != "cpu" else 1.0, "engine.ignore_eos": True, "health.enabled": False,
        "operator.workers": 512, "operator.io_workers": 16, "patterns.cache_dir": f"/tmp/oamd-lat-{os.getpid()}"})
    meng = MatchEngine(synthetic_library(a.patterns, seed=0), device=dev, seg_bytes=s.patterns.seg_bytes)
    model, kv, llm, tok = build_llm(s, device=dev)
    llm.warmup([b for b in llm.buckets if b <= a.max_batch])
    ee = ExplainEngine(llm, tok, model_id=a.model, max_prompt_tokens=a.prompt_tokens, ignore_eos=True)
    fk = FakeKube()
    op = Operator(fk, s, match_service=LocalMatchService(meng, max_batch=64, max_wait_ms=2.0),
                  explain_service=LocalExplainService(ee))
    fk.create(AIPROVIDERS, {"metadata": {"name": "local-llm", "namespace": "default"},
                            "spec": {"providerId": "local", "modelId": a.model, "maxTokens": a.max_tokens,
                                     "temperature": 0.3, "cachingEnabled": False, "timeoutSeconds": 3600}})
    fk.create(PODMORTEMS, {"metadata": {"name": "lat-monitor", "namespace": "default"},
                           "spec": {"podSelector": {"matchLabels": {"app": "lat"}}, "aiAnalysisEnabled": True,
                                    "aiProviderRef": {"name": "local-llm"}}})
    t_inject: dict[str, float] = {}
    done: dict[str, float] = {}
    lock = threading.Lock()

    def on_done(monitor, pod, outcome):
        with lock:
            done[pod["metadata"]["name"]] = time.perf_counter()

    op.pipeline.listeners.append(on_done)
    op.start(http=False)
    while not op.monitors.list():
        time.sleep(0.01)
    pool = LogFactory(n_patterns=a.patterns, seed=7).batch(256, a.log_kb * 1024, n_failures=3, seed=11)[0]
    rng = random.Random(a.seed)
    seq = [0]
    dump = {}
    if a.start_at:
        time.sleep(max(0.0, a.start_at - time.time()))

    def inject(prefix: str) -> str:
        i = seq[0]
        seq[0] += 1
        name = f"{prefix}-{i}"
        fk.create(PODS, running_pod(name, labels={"app": "lat"}))
        fk.set_log("default", name, pool[i % len(pool)])
        cur = fk.get(PODS, name, "default")
        cur["status"] = failed_pod(name, finished_at="2025-08-29T10:00:00Z")["status"]
        with lock:
            t_inject[name] = time.perf_counter()
        fk.replace(PODS, cur)
        return name

    for rate in [float(x) for x in a.rates.split(",")]:
        names = []
        t_warm = time.perf_counter() + a.warmup_s
        t_end = t_warm + a.seconds
        nxt = time.perf_counter()
        while True:
            now = time.perf_counter()
            if now >= t_end:
                break
            if now < nxt:
                time.sleep(min(0.01, nxt - now))
                continue
            n = inject(f"r{rate:g}")
            if now >= t_warm:
                names.append(n)
            nxt += rng.expovariate(rate)
        deadline = time.perf_counter() + 600
        while time.perf_counter() < deadline:
            with lock:
                if all(n in done for n in names):
                    break
            time.sleep(0.05)
        with lock:
            lat = [done[n] - t_inject[n] for n in names if n in done]
            span = (max(done[n] for n in names if n in done) - min(t_inject[n] for n in names)) if lat else 0
        dump[f"{rate:g}"] = {"lat": lat, "span": span}
        print(json.dumps({"bench": "open-loop latency", "model": a.model, "offered_rate": rate,
                          "failures": len(names), "completed": len(lat),
                          "analyses_per_s": round(len(lat) / span, 2) if span > 0 else None,
                          "p50_ms": round(statistics.median(lat) * 1e3, 1) if lat else None,
                          "p90_ms": round(pct(lat, 90) * 1e3, 1), "p99_ms": round(pct(lat, 99) * 1e3, 1),
                          "max_tokens": a.max_tokens, "prompt_tokens_cap": a.prompt_tokens,
                          "data": "synthetic logs, random-init weights"}), flush=True)
        op.drain(120)
    op.stop()
    ee.close()
    if a.dump_lat:
        with open(a.dump_lat, "w") as f:
            json.dump(dump, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
