"""AIProvider lookup and AIProvider CR -> AIProviderConfig conversion.

Mirrors J/service/AIInterfaceClient.java:71-149 and the provider lookup of
J/service/PodFailureWatcher.java:510-559:
* provider namespace defaults to the Podmortem's namespace;
* lookup errors are logged and treated as "not found" (the reference catches
  them inside the lookup and returns Optional.empty());
* defaults timeoutSeconds=30, maxRetries=3, cachingEnabled=true, maxTokens=500,
  temperature=0.3; additionalConfig -> additionalHeaders;
* the auth token is read from the Secret named by authenticationRef in the
  AIProvider's namespace and base64-decoded (null when anything is missing).
"""
from __future__ import annotations

import base64
import logging

from operator_amd.api.models import AIProviderConfig
from operator_amd.kube.resources import AIPROVIDERS, SECRETS

log = logging.getLogger(__name__)

DEFAULTS = {"timeout_seconds": 30, "max_retries": 3, "caching_enabled": True, "max_tokens": 500, "temperature": 0.3}


def provider_ref(monitor: dict) -> tuple[str | None, str | None]:
    spec = (monitor or {}).get("spec") or {}
    ref = spec.get("aiProviderRef")
    if ref is None:
        return None, None
    ns = ref.get("namespace") or (monitor.get("metadata") or {}).get("namespace")
    return ref.get("name"), ns


def ai_enabled(monitor: dict) -> bool:
    """Boolean.TRUE.equals(spec.aiAnalysisEnabled) && spec.aiProviderRef != null (PodFailureWatcher.java:350-351).
    The CRD defaults aiAnalysisEnabled to true at admission; FakeKube objects get the same default here."""
    spec = (monitor or {}).get("spec") or {}
    enabled = spec.get("aiAnalysisEnabled", True)
    return enabled is True and spec.get("aiProviderRef") is not None


def get_provider(kube, monitor: dict, cache=None) -> dict | None:
    """The monitor's AIProvider: from the informer cache when it holds it, else a GET (the
    reference GETs on every analysis, PodFailureWatcher.java:510-559)."""
    name, ns = provider_ref(monitor)
    if name is None:
        return None
    if cache is not None:
        p = cache.get(name, ns)
        if p is not None:
            return p
    try:
        p = kube.get(AIPROVIDERS, name, ns)
        if p is None:
            log.warning("AI provider not found: %s/%s", ns, name)
        return p
    except Exception as e:  # noqa: BLE001 (reference: catch-all -> Optional.empty())
        log.error("Error fetching AI provider: %s", e)
        return None


def load_auth_token(kube, namespace: str | None, secret_name: str | None, secret_key: str | None) -> str | None:
    try:
        sec = kube.get(SECRETS, secret_name, namespace)
        if sec is None:
            log.error("Authentication secret not found: %s/%s", namespace, secret_name)
            return None
        data = sec.get("data")
        if not data or secret_key not in data:
            log.error("Authentication key '%s' not found in secret %s/%s", secret_key, namespace, secret_name)
            return None
        return base64.b64decode(data[secret_key]).decode("utf-8", "replace")
    except Exception as e:  # noqa: BLE001
        log.error("Failed to load auth token from secret %s/%s: %s", namespace, secret_name, e)
        return None


def to_provider_config(kube, provider: dict) -> AIProviderConfig:
    spec = provider.get("spec") or {}

    def pick(key: str, camel: str):
        v = spec.get(camel)
        return DEFAULTS[key] if v is None else v

    cfg = AIProviderConfig(
        provider_id=spec.get("providerId"), api_url=spec.get("apiUrl"), model_id=spec.get("modelId"),
        timeout_seconds=int(pick("timeout_seconds", "timeoutSeconds")),
        max_retries=int(pick("max_retries", "maxRetries")),
        caching_enabled=bool(pick("caching_enabled", "cachingEnabled")),
        prompt_template=spec.get("promptTemplate"),
        max_tokens=int(pick("max_tokens", "maxTokens")),
        temperature=float(pick("temperature", "temperature")),
        additional_headers=dict(spec["additionalConfig"]) if spec.get("additionalConfig") is not None else None,
    )
    auth = spec.get("authenticationRef")
    if auth is not None:
        cfg.auth_token = load_auth_token(kube, (provider.get("metadata") or {}).get("namespace"),
                                         auth.get("secretName"), auth.get("secretKey"))
    return cfg
