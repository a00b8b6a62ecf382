"""External AIProviders (engine/providers.py): OpenAI-compatible and Ollama
request shapes, auth / extra headers, caching, retries, and the operator path end
to end against a local HTTP stand-in for the provider (no network)."""
import base64
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import httpx
import pytest

from operator_amd.api.models import AIProviderConfig, AnalysisEvent, AnalysisResult, AnalysisSummary, MatchedPattern
from operator_amd.engine.providers import ExternalProviderClient, ProviderError, ProviderRouter, provider_kind


def _result():
    return AnalysisResult(pod_name="api-1", pod_namespace="default",
                          summary=AnalysisSummary(highest_severity="CRITICAL", significant_events=1, total_events=1),
                          events=[AnalysisEvent(line_number=2, score=0.9, matched_line="OOMKilled",
                                                matched_pattern=MatchedPattern(name="OOM", severity="CRITICAL"))])


def _mock(handler):
    seen = []

    def h(req: httpx.Request):
        seen.append(req)
        return handler(req)

    return ExternalProviderClient(transport=httpx.MockTransport(h)), seen


def test_provider_kinds():
    assert provider_kind(None) == "local" and provider_kind("local") == "local"
    assert provider_kind("OpenAI") == "openai" and provider_kind("vllm") == "openai"
    assert provider_kind("ollama") == "ollama" and provider_kind("x") == "unknown"


def test_openai_request_auth_headers_and_cache():
    cli, seen = _mock(lambda r: httpx.Response(200, json={
        "choices": [{"message": {"role": "assistant", "content": "Root Cause: heap. Fix: raise limit."}}],
        "usage": {"completion_tokens": 9}}))
    cfg = AIProviderConfig(provider_id="openai", api_url="https://api.example/v1/", model_id="gpt-x", max_tokens=77,
                           temperature=0.2, auth_token="sk-1", additional_headers={"OpenAI-Organization": "org-9"})
    r = cli.explain(_result(), cfg)
    assert r.explanation.startswith("Root Cause: heap") and r.tokens_generated == 9 and not r.cached
    req = seen[0]
    assert str(req.url) == "https://api.example/v1/chat/completions"
    assert req.headers["authorization"] == "Bearer sk-1" and req.headers["openai-organization"] == "org-9"
    body = json.loads(req.content)
    assert body["model"] == "gpt-x" and body["max_tokens"] == 77 and body["temperature"] == 0.2
    assert body["messages"][-1]["role"] == "user" and "Pod default/api-1 failed" in body["messages"][-1]["content"]
    # cachingEnabled: the same request is answered from the LRU
    assert cli.explain(_result(), cfg).cached and len(seen) == 1
    cli.explain(_result(), cfg.model_copy(update={"caching_enabled": False}))
    assert len(seen) == 2


def test_ollama_request_shape():
    cli, seen = _mock(lambda r: httpx.Response(200, json={"response": "Root Cause: x", "eval_count": 3}))
    cfg = AIProviderConfig(provider_id="ollama", api_url="http://ollama:11434", model_id="llama3", max_tokens=12,
                           caching_enabled=False)
    r = cli.explain(_result(), cfg)
    assert r.explanation == "Root Cause: x" and r.tokens_generated == 3
    body = json.loads(seen[0].content)
    assert str(seen[0].url) == "http://ollama:11434/api/generate"
    assert body["stream"] is False and body["options"] == {"num_predict": 12, "temperature": 0.3}


def test_retries_on_5xx_not_on_4xx():
    codes = iter([503, 502, 200])
    cli, seen = _mock(lambda r: httpx.Response(c, json={"response": "ok"}) if (c := next(codes)) == 200
                      else httpx.Response(c))
    cfg = AIProviderConfig(provider_id="ollama", api_url="http://o", max_retries=3, caching_enabled=False)
    assert cli.explain(_result(), cfg).explanation == "ok" and len(seen) == 3
    cli2, seen2 = _mock(lambda r: httpx.Response(401, text="bad key"))
    with pytest.raises(ProviderError, match="HTTP 401"):
        cli2.explain(_result(), cfg)
    assert len(seen2) == 1
    cli3, seen3 = _mock(lambda r: httpx.Response(500))
    with pytest.raises(ProviderError, match="after 2 attempt"):
        cli3.explain(_result(), cfg.model_copy(update={"max_retries": 1}))


def test_router_keeps_local_providers_local():
    class Local:
        def explain(self, r, c):
            from operator_amd.api.models import AIResponse
            return AIResponse(explanation="local")

    cli, seen = _mock(lambda r: httpx.Response(200, json={"response": "remote"}))
    rt = ProviderRouter(Local(), cli)
    assert rt.explain(_result(), AIProviderConfig(provider_id="local")).explanation == "local"
    assert rt.explain(_result(), AIProviderConfig(provider_id="custom")).explanation == "local"
    assert rt.explain(_result(), AIProviderConfig(provider_id="ollama", api_url="http://o")).explanation == "remote"
    off = ProviderRouter(Local(), cli, enabled=False)
    assert off.explain(_result(), AIProviderConfig(provider_id="ollama", api_url="http://o")).explanation == "local"


class _FakeOpenAI(BaseHTTPRequestHandler):
    requests: list = []

    def do_POST(self):  # noqa: N802
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        type(self).requests.append((self.path, dict(self.headers), body))
        out = json.dumps({"choices": [{"message": {"content": "Root Cause: remote model says OOM. Fix: more memory."}}],
                          "usage": {"completion_tokens": 11}}).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(out)))
        self.end_headers()
        self.wfile.write(out)

    def log_message(self, *a):
        pass


def test_operator_with_openai_provider_end_to_end(tmp_path):
    from operator_amd.config import load_settings
    from operator_amd.controller.operator import Operator
    from operator_amd.engine.match import MatchEngine
    from operator_amd.engine.service import EchoExplainService, LocalMatchService
    from operator_amd.kube.fake import FakeKube, failed_pod, running_pod
    from operator_amd.kube.resources import AIPROVIDERS, PODMORTEMS, PODS, SECRETS
    from operator_amd.patterns.synth import catalog_library
    from tests.test_controller import wait_for

    srv = ThreadingHTTPServer(("127.0.0.1", 0), _FakeOpenAI)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    fk = FakeKube()
    s = load_settings(env={}, overrides={"patterns.cache_dir": str(tmp_path), "health.enabled": False})
    echo = EchoExplainService()
    op = Operator(fk, s, match_service=LocalMatchService(MatchEngine(catalog_library(), device="cpu"), max_wait_ms=1),
                  explain_service=echo)
    op.start(http=False)
    try:
        fk.create(SECRETS, {"metadata": {"name": "openai-credentials", "namespace": "default"},
                            "data": {"api-key": base64.b64encode(b"sk-live").decode()}})
        fk.create(AIPROVIDERS, {"metadata": {"name": "openai-provider", "namespace": "default"},
                                "spec": {"providerId": "openai", "apiUrl": f"http://127.0.0.1:{srv.server_port}/v1",
                                         "modelId": "gpt-3.5-turbo",
                                         "authenticationRef": {"secretName": "openai-credentials",
                                                               "secretKey": "api-key"}}})
        fk.create(PODMORTEMS, {"metadata": {"name": "m", "namespace": "default"},
                               "spec": {"podSelector": {"matchLabels": {"app": "demo"}}, "aiAnalysisEnabled": True,
                                        "aiProviderRef": {"name": "openai-provider"}}})
        wait_for(lambda: op.monitors.list())
        fk.create(PODS, running_pod("api-1", labels={"app": "demo"}))
        fk.set_log("default", "api-1", b"start\nOOMKilled: container exceeded memory limit\n")
        cur = fk.get(PODS, "api-1", "default")
        cur["status"] = failed_pod("api-1", labels={"app": "demo"})["status"]
        fk.replace(PODS, cur)
        pod = wait_for(lambda: (lambda p: p if "podmortem.io/analysis" in (p["metadata"].get("annotations") or {})
                                else None)(fk.get(PODS, "api-1", "default")))
        assert pod["metadata"]["annotations"]["podmortem.io/analysis"].startswith("Root Cause: remote model says OOM")
        assert echo.calls == 0
        path, headers, body = _FakeOpenAI.requests[-1]
        assert path == "/v1/chat/completions" and headers["Authorization"] == "Bearer sk-live"
        assert body["model"] == "gpt-3.5-turbo" and body["max_tokens"] == 500 and body["temperature"] == 0.3
        aip = wait_for(lambda: (lambda o: o if (o.get("status") or {}).get("phase") else None)(
            fk.get(AIPROVIDERS, "openai-provider", "default")))
        assert aip["status"]["phase"] == "Ready" and "external openai API" in aip["status"]["message"]
    finally:
        op.stop()
        srv.shutdown()
