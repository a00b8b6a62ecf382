"""OpenAI- and Ollama-compatible endpoints of the compat server (engine/server.py),
served by the on-node engine (a tiny model on the CPU here): response shapes,
sampling parameters, streaming as one chunk, errors, model routing, and the
round trip through this framework's own external-provider client."""
import json

import httpx
import pytest

from operator_amd.config import load_settings
from operator_amd.engine.factory import build_explain_service
from operator_amd.engine.server import CompatServer


@pytest.fixture(scope="module")
def server():
    s = load_settings(env={}, overrides={"engine.model": "tiny", "engine.extra_models": ["tiny-gqa4"],
                                         "engine.device": "cpu", "engine.dtype": "float32",
                                         "engine.kv_cache_gb": 0.04, "engine.use_graphs": False,
                                         "engine.max_batch": 4, "engine.max_context": 512,
                                         "engine.max_prompt_tokens": 256})
    svc = build_explain_service(s)
    srv = CompatServer(None, svc, "127.0.0.1", 0).start()
    yield srv, svc
    srv.stop()
    svc.close()


def _post(srv, path, body, **kw):
    return httpx.post(f"http://127.0.0.1:{srv.port}{path}", json=body, timeout=120, **kw)


def test_openai_chat_completion_shape_and_routing(server):
    srv, svc = server
    st = {m: svc.services[m].ee.llm.stats for m in svc.models}
    before = st["tiny-gqa4"].decode_tokens
    r = _post(srv, "/v1/chat/completions", {"model": "tiny-gqa4", "max_tokens": 7, "temperature": 0,
                                             "messages": [{"role": "system", "content": "be brief"},
                                                          {"role": "user", "content": "why did my pod crash?"}]})
    assert r.status_code == 200, r.text
    b = r.json()
    assert b["object"] == "chat.completion" and b["model"] == "tiny-gqa4" and b["id"].startswith("chatcmpl-")
    ch = b["choices"][0]
    assert ch["message"]["role"] == "assistant" and isinstance(ch["message"]["content"], str)
    assert ch["finish_reason"] in ("length", "stop")
    u = b["usage"]
    assert 0 < u["completion_tokens"] <= 7 and u["total_tokens"] == u["prompt_tokens"] + u["completion_tokens"]
    assert st["tiny-gqa4"].decode_tokens > before   # the request ran on the engine it named
    # greedy decoding is deterministic: the same request gives the same text
    r2 = _post(srv, "/chat/completions", {"model": "tiny-gqa4", "max_tokens": 7, "temperature": 0,
                                          "messages": [{"role": "system", "content": "be brief"},
                                                       {"role": "user", "content": "why did my pod crash?"}]})
    assert r2.json()["choices"][0]["message"]["content"] == ch["message"]["content"]


def test_openai_completions_models_and_stream(server):
    srv, _ = server
    r = _post(srv, "/v1/completions", {"model": "tiny", "prompt": "OOMKilled means", "max_tokens": 4,
                                       "temperature": 0.7, "seed": 3})
    b = r.json()
    assert r.status_code == 200 and b["object"] == "text_completion" and "text" in b["choices"][0]
    assert b["usage"]["completion_tokens"] <= 4
    m = httpx.get(f"http://127.0.0.1:{srv.port}/v1/models").json()
    assert [d["id"] for d in m["data"]] == ["tiny", "tiny-gqa4"]
    r = _post(srv, "/v1/chat/completions", {"model": "tiny", "stream": True, "max_tokens": 3,
                                            "messages": [{"role": "user", "content": "hi"}]})
    assert r.headers["content-type"].startswith("text/event-stream")
    events = [ln[6:] for ln in r.text.splitlines() if ln.startswith("data: ")]
    assert events[-1] == "[DONE]"
    chunk = json.loads(events[0])
    assert chunk["object"] == "chat.completion.chunk" and "content" in chunk["choices"][0]["delta"]


def test_ollama_generate_and_chat(server):
    srv, _ = server
    r = _post(srv, "/api/generate", {"model": "tiny", "prompt": "CrashLoopBackOff", "stream": False,
                                     "options": {"num_predict": 5, "temperature": 0}})
    b = r.json()
    assert r.status_code == 200 and b["done"] is True and isinstance(b["response"], str)
    assert 0 < b["eval_count"] <= 5 and b["prompt_eval_count"] > 0
    r = _post(srv, "/api/chat", {"model": "tiny", "messages": [{"role": "user", "content": "hi"}],
                                 "options": {"num_predict": 2}})   # Ollama streams unless told not to
    lines = [json.loads(x) for x in r.text.splitlines() if x.strip()]
    assert r.headers["content-type"].startswith("application/x-ndjson")
    assert len(lines) == 1 and lines[0]["done"] and lines[0]["message"]["role"] == "assistant"
    tags = httpx.get(f"http://127.0.0.1:{srv.port}/api/tags").json()
    assert {t["name"] for t in tags["models"]} == {"tiny", "tiny-gqa4"}


def test_bad_requests_are_400(server):
    srv, _ = server
    assert _post(srv, "/v1/chat/completions", {"model": "tiny", "messages": []}).status_code == 400
    assert _post(srv, "/v1/completions", {"model": "tiny", "prompt": 5}).status_code == 400
    assert _post(srv, "/v1/chat/completions", {"n": 2, "messages": [{"role": "user", "content": "x"}]}).status_code == 400
    assert _post(srv, "/v1/completions", {"prompt": "x", "max_tokens": "many"}).status_code == 400
    assert _post(srv, "/api/generate", {"prompt": "x", "options": {"temperature": "hot"}}).status_code == 400
    long = " ".join(["word"] * 2000)   # more tokens than the engine's 512-token context
    r = _post(srv, "/v1/completions", {"model": "tiny", "prompt": long, "max_tokens": 4})
    assert r.status_code == 400 and "max_context" in r.json()["error"]["message"]
    r = httpx.post(f"http://127.0.0.1:{srv.port}/v1/completions", content=b"{not json",
                   headers={"Content-Type": "application/json"})
    assert r.status_code == 400


def test_providers_client_round_trip(server):
    """An AIProvider with providerId openai / ollama whose apiUrl is this server: the
    framework's own external-provider client gets an explanation from the engine."""
    from operator_amd.api.models import AIProviderConfig, AnalysisResult, AnalysisSummary
    from operator_amd.engine.providers import ExternalProviderClient

    srv, _ = server
    res = AnalysisResult(pod_name="p", pod_namespace="default",
                         summary=AnalysisSummary(highest_severity="HIGH", significant_events=1))
    c = ExternalProviderClient()
    for pid, url in (("openai", f"http://127.0.0.1:{srv.port}/v1"), ("ollama", f"http://127.0.0.1:{srv.port}")):
        out = c.explain(res, AIProviderConfig(provider_id=pid, api_url=url, model_id="tiny", max_tokens=4,
                                              temperature=0.0, caching_enabled=False))
        assert isinstance(out.explanation, str) and 0 < out.tokens_generated <= 4


def test_finished_batch_is_detokenized_once_before_waiters_wake(server):
    """The engine loop detokenizes every request a step finished in one decode_batch
    call (LLMEngine.finish_hook), and the text equals per-request decoding."""
    from operator_amd.engine.llm import GenRequest

    _, svc = server
    ee = svc.services["tiny"].ee
    assert ee.llm.finish_hook is not None
    seqs = [[5, 6, 7, 300, 301], [], list(range(40, 90))]
    assert ee.tok.decode_batch(seqs) == [ee.tok.decode(x) for x in seqs]
    reqs = [GenRequest(list(range(3, 3 + n)), max_tokens=5, temperature=0.0, ignore_eos=True) for n in (4, 20)]
    seen = []
    real = ee.llm.finish_hook
    ee.llm.finish_hook = lambda fin: (seen.append([r.event.is_set() for r in fin]), real(fin))
    try:
        for r in reqs:
            ee.llm.submit(r)
        ee.loop.notify()
        for r in reqs:
            assert r.event.wait(60)
    finally:
        ee.llm.finish_hook = real
    assert seen and not any(any(x) for x in seen)          # hook ran before the waiters were released
    assert all(r.text == ee.tok.decode(r.output) for r in reqs)


def test_explain_many_item_failure_keeps_the_others(server):
    """A batch item that cannot be admitted comes back as that item's ExplainError; the
    items already submitted are still waited for (none is left decoding without a waiter)."""
    from operator_amd.api.models import AIProviderConfig, AnalysisResult, AnalysisSummary
    from operator_amd.engine.explain import ExplainError

    _, svc = server
    ee = svc.services["tiny"].ee
    res = AnalysisResult(pod_name="p", pod_namespace="default",
                         summary=AnalysisSummary(highest_severity="HIGH", significant_events=1))
    real, calls = ee._start, {"n": 0}

    def flaky(p, ids, notify=True):
        calls["n"] += 1
        if calls["n"] == 2:
            raise ValueError("prompt exceeds max_context")
        return real(p, ids, notify)

    ee._start = flaky
    try:
        cfg = AIProviderConfig(max_tokens=4, temperature=0.0, caching_enabled=False)
        out = ee.explain_many([(res, cfg)] * 3)
    finally:
        ee._start = real
    assert isinstance(out[1], ExplainError) and "max_context" in str(out[1])
    assert [o.tokens_generated for o in (out[0], out[2])] == [4, 4]
    assert not ee.llm.running and not ee.llm.waiting
