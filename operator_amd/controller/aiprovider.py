"""AIProvider reconciler — an extension: the reference has no
controller for AIProvider, so its status (phase Pending/Ready/Failed,
message, lastValidated, observedGeneration; K/aiprovider-crd.yaml:64-77) is
never written. Here the provider is validated against the on-node engine:

* the referenced auth Secret (if any) must exist and contain the key;
* the explain service must be ready (model weights loaded / engine loop alive);
* ``modelId`` picks among the on-node models (``engine.model`` + ``engine.extra_models``);
  one that is not served is mapped to the default model, reported in the message,
  not treated as a failure;
* a provider routed to an external API (``providerId`` openai / ollama, see
  engine/providers.py) is Ready when it names an ``apiUrl``.
"""
from __future__ import annotations

import logging

from operator_amd.kube.resources import SECRETS, ApiError
from operator_amd.utils.timefmt import instant_str

from .runtime import UpdateControl

log = logging.getLogger(__name__)


class AIProviderReconciler:
    def __init__(self, kube, explainer, engine_model: str = "local"):
        self.kube, self.explainer, self.engine_model = kube, explainer, engine_model

    def reconcile(self, provider: dict) -> UpdateControl:
        md = provider.get("metadata") or {}
        spec = provider.get("spec") or {}
        problems = []
        auth = spec.get("authenticationRef")
        if auth:
            try:
                sec = self.kube.get(SECRETS, auth.get("secretName"), md.get("namespace"))
                if sec is None:
                    problems.append(f"secret {auth.get('secretName')} not found")
                elif auth.get("secretKey") not in (sec.get("data") or {}):
                    problems.append(f"key {auth.get('secretKey')} missing in secret {auth.get('secretName')}")
            except ApiError as e:
                problems.append(f"secret lookup failed: {e}")
        from operator_amd.api.models import AIProviderConfig

        route = getattr(self.explainer, "route", lambda c: "local")(AIProviderConfig(provider_id=spec.get("providerId")))
        if route != "local":   # external API (engine/providers.py): needs an endpoint
            if not spec.get("apiUrl"):
                problems.append(f"providerId {spec.get('providerId')} needs spec.apiUrl")
        else:
            ready = self.explainer is not None and getattr(self.explainer, "ready", lambda: True)() \
                and getattr(self.explainer, "local", True) is not None
            if not ready:
                problems.append("explanation engine not ready")
        if problems:
            phase, msg = "Failed", "; ".join(problems)
        elif route != "local":
            phase = "Ready"
            msg = f"Served by the external {route} API at {spec.get('apiUrl')} (model {spec.get('modelId')})"
        else:
            phase = "Ready"
            mid = spec.get("modelId")
            served = list(getattr(getattr(self.explainer, "local", self.explainer), "models", None) or
                          [self.engine_model])
            hit = next((m for m in served if mid and m.lower() == mid.lower()), None)
            msg = f"Served by on-node engine ({hit or self.engine_model})"
            if mid and hit is None:
                msg += f"; requested modelId {mid} is mapped to {self.engine_model}"
        return UpdateControl.patch_status({"phase": phase, "message": msg, "lastValidated": instant_str(),
                                           "observedGeneration": md.get("generation")})
