"""Wire-compatible REST front for the on-node engines.

Serves the two contracts the reference operator calls, so an
unmodified podmortem operator (or any other client) can point its
``quarkus.rest-client.{log-parser,ai-interface}.url`` at this process:

  POST /parse                      PodFailureData  -> AnalysisResult   (LogParserRestClient.java:37-39)
  POST /api/v1/analysis/analyze    AnalysisRequest -> AIResponse       (AIInterfaceRestClient.java:37-39)
  GET  /q/health/live | /q/health/ready | /metrics

and the two LLM wire formats the reference's AIProviders name (aiprovider-crd.yaml:21,
"e.g. 'openai', 'ollama'"), so the on-node engine is itself an AIProvider endpoint
for any OpenAI or Ollama client (including engine/providers.py):

  POST [/v1]/chat/completions | [/v1]/completions | GET [/v1]/models   (OpenAI)
  POST /api/generate | /api/chat | GET /api/tags                       (Ollama)

Streaming requests get the whole completion as one chunk (SSE for OpenAI, one
NDJSON line for Ollama). Requests are handed to the batching services
(LocalMatchService / LocalExplainService), so concurrent HTTP callers share GPU
batches with the operator's own explanations.
"""
from __future__ import annotations

import json
import logging
import threading
import time
import uuid
from datetime import datetime, timezone
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from operator_amd.api.models import AnalysisRequest, PodFailureData

log = logging.getLogger(__name__)

COMPLETION_TIMEOUT_S = 600.0


class BadRequest(ValueError):
    pass


def _sampling(body: dict, ollama: bool) -> dict:
    """max_tokens / temperature / seed of an OpenAI body or an Ollama ``options`` map
    (defaults: the AIProvider CRD's 500 tokens at T = 0.3)."""
    src = (body.get("options") or {}) if ollama else body
    if not isinstance(src, dict):
        raise BadRequest("'options' must be an object")
    n = src.get("num_predict") if ollama else (body.get("max_completion_tokens") or body.get("max_tokens"))
    try:
        kw = {"max_tokens": int(n) if n is not None and int(n) > 0 else 500,
              "temperature": float(src.get("temperature", 0.3)), "timeout_s": COMPLETION_TIMEOUT_S}
        if src.get("seed") is not None:
            kw["seed"] = int(src["seed"])
        n_choices = int(body.get("n", 1) or 1)
    except (TypeError, ValueError) as e:
        raise BadRequest(f"bad sampling parameter: {e}") from None
    if not ollama and n_choices != 1:
        raise BadRequest("only n = 1 is supported")
    return kw


def _messages(body: dict) -> list[dict]:
    msgs = body.get("messages")
    if not isinstance(msgs, list) or not msgs:
        raise BadRequest("'messages' must be a non-empty list")
    out = []
    for m in msgs:
        c = m.get("content")
        if isinstance(c, list):   # OpenAI content parts: keep the text ones
            c = "".join(p.get("text", "") for p in c if isinstance(p, dict))
        out.append({"role": m.get("role", "user"), "content": c or ""})
    return out


class CompatServer:
    def __init__(self, matcher, explainer, host: str = "0.0.0.0", port: int = 8080, metrics=None):
        self.matcher, self.explainer, self.metrics = matcher, explainer, metrics
        srv = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, code: int, obj, ctype: str = "application/json") -> None:
                b = obj if isinstance(obj, bytes) else json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def do_GET(self):  # noqa: N802
                if self.path.startswith("/q/health"):
                    return self._send(200, {"status": "UP", "checks": []})
                if self.path.startswith("/metrics") and srv.metrics is not None:
                    return self._send(200, srv.metrics.render(), "text/plain; version=0.0.4")
                path = self.path.split("?")[0].rstrip("/")
                if path in ("/v1/models", "/models"):
                    return self._send(200, {"object": "list", "data": [
                        {"id": m, "object": "model", "created": 0, "owned_by": "operator-amd"} for m in srv.models()]})
                if path == "/api/tags":
                    return self._send(200, {"models": [{"name": m, "model": m} for m in srv.models()]})
                self._send(404, {"error": "not found"})

            def _llm(self, path: str, body: dict) -> bool:
                """OpenAI / Ollama endpoints; False if ``path`` is not one of them."""
                p = path[3:] if path.startswith("/v1/") else path
                if p not in ("/chat/completions", "/completions", "/api/generate", "/api/chat"):
                    return False
                if srv.explainer is None or not hasattr(srv.explainer, "complete"):
                    self._send(503, {"error": "explanation engine not configured"})
                    return True
                ollama = p.startswith("/api/")
                chat = p in ("/chat/completions", "/api/chat")
                kw = _sampling(body, ollama)
                if chat:
                    out = srv.explainer.complete(messages=_messages(body), model=body.get("model"), **kw)
                else:
                    prompt = body.get("prompt")
                    if isinstance(prompt, list):
                        if len(prompt) != 1:
                            raise BadRequest("one prompt per request")
                        prompt = prompt[0]
                    if not isinstance(prompt, str):
                        raise BadRequest("'prompt' must be a string")
                    out = srv.explainer.complete(prompt=prompt, model=body.get("model"), **kw)
                model = body.get("model") or out.get("model")
                if ollama:
                    obj = {"model": model, "created_at": datetime.now(timezone.utc).isoformat(), "done": True,
                           "done_reason": out["finish_reason"], "prompt_eval_count": out["prompt_tokens"],
                           "eval_count": out["completion_tokens"],
                           "total_duration": int(out["latency_ms"] * 1e6)}
                    if chat:
                        obj["message"] = {"role": "assistant", "content": out["text"]}
                    else:
                        obj["response"] = out["text"]
                    if body.get("stream", True):   # Ollama streams by default: one final NDJSON line
                        self._send(200, json.dumps(obj).encode() + b"\n", "application/x-ndjson")
                    else:
                        self._send(200, obj)
                    return True
                usage = {"prompt_tokens": out["prompt_tokens"], "completion_tokens": out["completion_tokens"],
                         "total_tokens": out["prompt_tokens"] + out["completion_tokens"]}
                base = {"id": ("chatcmpl-" if chat else "cmpl-") + uuid.uuid4().hex[:24], "created": int(time.time()),
                        "model": model}
                if body.get("stream"):   # SSE: the whole completion as one chunk, then [DONE]
                    delta = ({"delta": {"role": "assistant", "content": out["text"]}} if chat else {"text": out["text"]})
                    chunk = {**base, "object": "chat.completion.chunk" if chat else "text_completion",
                             "choices": [{"index": 0, **delta, "finish_reason": out["finish_reason"]}]}
                    self._send(200, b"data: " + json.dumps(chunk).encode() + b"\n\ndata: [DONE]\n\n",
                               "text/event-stream")
                    return True
                choice = ({"message": {"role": "assistant", "content": out["text"]}} if chat else {"text": out["text"]})
                self._send(200, {**base, "object": "chat.completion" if chat else "text_completion",
                                 "choices": [{"index": 0, **choice, "finish_reason": out["finish_reason"]}],
                                 "usage": usage})
                return True

            def do_POST(self):  # noqa: N802
                n = int(self.headers.get("Content-Length", "0") or 0)
                try:
                    body = json.loads(self.rfile.read(n) or b"{}")
                    if self.path.rstrip("/") == "/parse":
                        if srv.matcher is None:
                            return self._send(503, {"error": "pattern engine not configured"})
                        res = srv.matcher.analyze(PodFailureData.model_validate(body))
                        return self._send(200, res.to_obj())
                    if self.path.rstrip("/") == "/api/v1/analysis/analyze":
                        if srv.explainer is None:
                            return self._send(503, {"error": "explanation engine not configured"})
                        req = AnalysisRequest.model_validate(body)
                        resp = srv.explainer.explain(req.analysis_result, req.provider_config)
                        return self._send(200, resp.to_obj())
                    if self._llm(self.path.split("?")[0].rstrip("/"), body):
                        return None
                    return self._send(404, {"error": "not found"})
                except (BadRequest, json.JSONDecodeError) as e:
                    return self._send(400, {"error": {"message": str(e), "type": "invalid_request_error"}})
                except Exception as e:  # noqa: BLE001
                    msg = str(e)
                    if "exceeds max_context" in msg:
                        return self._send(400, {"error": {"message": msg, "type": "invalid_request_error"}})
                    log.error("request %s failed: %s", self.path, e)
                    return self._send(504 if "timed out" in msg else 500, {"error": {"message": msg}})

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self._t = threading.Thread(target=self.httpd.serve_forever, name="compat-http", daemon=True)

    def models(self) -> list[str]:
        e = self.explainer
        m = getattr(e, "models", None) if e is not None else None
        return list(m) if m else []

    def start(self) -> "CompatServer":
        self._t.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
