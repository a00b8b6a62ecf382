"""AIProvider routing: the on-node engine for local providers, the provider's own
API for external ones.

In the reference every AIProvider — e.g. ``providerId: openai``,
``apiUrl: https://api.openai.com/v1`` (README.md:54-66; aiprovider-crd.yaml:21
"e.g. 'openai', 'ollama'") — is served by the out-of-repo ai-interface, which
calls that provider. Here the default provider is the local GPU engine, but a
user switching over keeps their external providers working:

* ``providerId`` empty / ``local`` / ``operator-amd`` / ``podmortem`` (or any id
  when ``services.external_providers`` is off) -> the configured explain service
  (the on-node Llama engine, the remote ai-interface shim, or the echo stub);
* ``openai`` (and OpenAI-compatible servers: ``vllm``, ``openai-compatible``,
  ``azure-openai``, ``lmstudio``, ``together``, ``groq``) -> ``POST
  {apiUrl}/chat/completions``;
* ``ollama`` -> ``POST {apiUrl}/api/generate`` (``stream: false``).

The AIProvider fields keep their contract (AIInterfaceClient.java:71-105):
``timeoutSeconds`` per attempt, ``maxRetries`` extra attempts on transport
errors / 429 / 5xx, ``cachingEnabled`` (LRU keyed by provider, model, prompt and
sampling parameters), ``promptTemplate`` (engine/prompt.py placeholders),
``maxTokens``, ``temperature``, ``additionalConfig`` as extra HTTP headers, and
the Secret-held token as ``Authorization: Bearer``.
"""
from __future__ import annotations

import hashlib
import logging
import threading
import time
from collections import OrderedDict

from operator_amd.api.models import AIProviderConfig, AIResponse, AnalysisResult

from . import prompt as prompt_mod

log = logging.getLogger(__name__)

LOCAL_IDS = {"", "local", "operator-amd", "podmortem", "on-node"}
OPENAI_IDS = {"openai", "openai-compatible", "vllm", "azure-openai", "lmstudio", "together", "groq"}
OLLAMA_IDS = {"ollama"}
SYSTEM_PROMPT = "You are Podmortem, a Kubernetes failure analyst."


class ProviderError(RuntimeError):
    pass


def provider_kind(provider_id: str | None) -> str:
    pid = (provider_id or "").strip().lower()
    if pid in LOCAL_IDS:
        return "local"
    if pid in OPENAI_IDS:
        return "openai"
    if pid in OLLAMA_IDS:
        return "ollama"
    return "unknown"


class ExternalProviderClient:
    """HTTP client for OpenAI-compatible and Ollama endpoints."""

    def __init__(self, cache_size: int = 1024, transport=None):
        import httpx

        self._httpx = httpx
        self._transport = transport   # tests inject an httpx transport
        self._cache: OrderedDict[str, AIResponse] = OrderedDict()
        self._cache_size = cache_size
        self._lock = threading.Lock()
        self.calls = 0

    def _client(self, timeout_s: float):
        kw = {"timeout": self._httpx.Timeout(timeout_s)}
        if self._transport is not None:
            kw["transport"] = self._transport
        return self._httpx.Client(**kw)

    @staticmethod
    def _headers(cfg: AIProviderConfig) -> dict[str, str]:
        h = {"Content-Type": "application/json"}
        if cfg.auth_token:
            h["Authorization"] = f"Bearer {cfg.auth_token}"
        for k, v in (cfg.additional_headers or {}).items():
            h[str(k)] = str(v)
        return h

    @staticmethod
    def _request(kind: str, cfg: AIProviderConfig, text: str) -> tuple[str, dict]:
        base = (cfg.api_url or "").rstrip("/")
        if not base:
            raise ProviderError(f"AIProvider {cfg.provider_id!r} has no apiUrl")
        if kind == "openai":
            return base + "/chat/completions", {
                "model": cfg.model_id, "max_tokens": int(cfg.max_tokens), "temperature": float(cfg.temperature),
                "messages": [{"role": "system", "content": SYSTEM_PROMPT}, {"role": "user", "content": text}]}
        return base + "/api/generate", {
            "model": cfg.model_id, "prompt": text, "stream": False,
            "options": {"num_predict": int(cfg.max_tokens), "temperature": float(cfg.temperature)}}

    @staticmethod
    def _parse(kind: str, body: dict) -> tuple[str, int | None]:
        if kind == "openai":
            choices = body.get("choices") or []
            if not choices:
                raise ProviderError("provider response has no choices")
            msg = choices[0].get("message") or {}
            text = msg.get("content") if msg else choices[0].get("text")
            usage = body.get("usage") or {}
            return text or "", usage.get("completion_tokens")
        if "response" not in body:
            raise ProviderError("provider response has no 'response' field")
        return body.get("response") or "", body.get("eval_count")

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        kind = provider_kind(cfg.provider_id)
        if kind not in ("openai", "ollama"):
            raise ProviderError(f"unsupported AI provider {cfg.provider_id!r}")
        text = prompt_mod.render(result, cfg.prompt_template)
        key = None
        if cfg.caching_enabled:
            h = hashlib.sha256(f"{cfg.provider_id}|{cfg.api_url}|{cfg.model_id}|{cfg.max_tokens}|"
                               f"{cfg.temperature}|".encode() + text.encode())
            key = h.hexdigest()
            with self._lock:
                hit = self._cache.get(key)
                if hit is not None:
                    self._cache.move_to_end(key)
                    return hit.model_copy(update={"cached": True})
        url, payload = self._request(kind, cfg, text)
        attempts = 1 + max(0, int(cfg.max_retries or 0))
        last: Exception | None = None
        t0 = time.perf_counter()
        for i in range(attempts):
            try:
                self.calls += 1
                with self._client(float(cfg.timeout_seconds or 30)) as c:
                    r = c.post(url, json=payload, headers=self._headers(cfg))
                if r.status_code == 429 or r.status_code >= 500:
                    raise ProviderError(f"provider returned HTTP {r.status_code}")
                if r.status_code >= 400:   # client errors are not retried
                    raise ProviderError(f"provider returned HTTP {r.status_code}: {r.text[:200]}")
                out, ntok = self._parse(kind, r.json())
                resp = AIResponse(explanation=out, provider_id=cfg.provider_id, model_id=cfg.model_id,
                                  tokens_generated=ntok, latency_ms=round((time.perf_counter() - t0) * 1e3, 3),
                                  cached=False)
                if key is not None:
                    with self._lock:
                        self._cache[key] = resp
                        while len(self._cache) > self._cache_size:
                            self._cache.popitem(last=False)
                return resp
            except ProviderError as e:
                last = e
                if "HTTP 4" in str(e) and "HTTP 429" not in str(e):
                    break
            except Exception as e:  # noqa: BLE001 - transport errors / timeouts: retried
                last = e
            if i + 1 < attempts:
                time.sleep(min(2.0, 0.1 * (2 ** i)))
        raise ProviderError(f"{cfg.provider_id} request failed after {i + 1} attempt(s): {last}")


class ProviderRouter:
    """Explain service that routes each request by its AIProvider's ``providerId``."""

    def __init__(self, local, external: ExternalProviderClient | None = None, enabled: bool = True):
        self.local = local
        self.external = external if external is not None else (ExternalProviderClient() if enabled else None)
        self.enabled = enabled

    def route(self, cfg: AIProviderConfig) -> str:
        kind = provider_kind(cfg.provider_id)
        if not self.enabled or kind in ("local", "unknown") or self.external is None:
            return "local"
        return kind

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        if self.route(cfg) == "local":
            if self.local is None:
                raise ProviderError("no on-node explanation engine is configured")
            return self.local.explain(result, cfg)
        return self.external.explain(result, cfg)

    def explain_many(self, items):
        if all(self.route(c) == "local" for _, c in items) and hasattr(self.local, "explain_many"):
            return self.local.explain_many(items)
        out = []
        for r, c in items:
            try:
                out.append(self.explain(r, c))
            except Exception as e:  # noqa: BLE001 - per-item errors, like ExplainEngine.explain_many
                out.append(e)
        return out

    def ready(self) -> bool:
        return self.local is None or getattr(self.local, "ready", lambda: True)()

    def close(self) -> None:
        close = getattr(self.local, "close", None)
        if close is not None:
            close()

    def __getattr__(self, name):   # ee / pool handles of the wrapped local service
        local = self.__dict__.get("local")
        if local is None:
            raise AttributeError(name)
        return getattr(local, name)
