"""Typed API model: the three CRDs and the analysis DTOs.

The reference takes these classes from its external ``common-lib``
(pom.xml:83-87, not vendored); they are reconstructed here from every call
site and from the CRD schemas
(src/main/kubernetes/{podmortem,patternlibrary,aiprovider}-crd.yaml).
Field names are the Kubernetes/JSON camelCase names; Python attribute names
are snake_case. Unknown fields are preserved (``extra="allow"``) so a
round-trip through the model never drops data another writer put there.
"""
from __future__ import annotations

from typing import Any, Optional

from pydantic import BaseModel, ConfigDict, Field
from pydantic.alias_generators import to_camel

GROUP = "podmortem.redhat.com"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"


_FAST_SPECS: dict[type, list] = {}


class KModel(BaseModel):
    model_config = ConfigDict(alias_generator=to_camel, populate_by_name=True, extra="allow")

    def to_obj(self) -> dict:
        return self.model_dump(by_alias=True, exclude_none=True, mode="json")

    @classmethod
    def fast(cls, **values):
        """``model_construct`` for a producer's own, already-typed values given by field
        name: the same object (defaults and default factories filled in field order,
        ``model_fields_set`` = the names given, empty extras), without model_construct's
        per-call walk over every field's aliases — the match engine builds thousands of
        results per scan batch and that walk was ~70 % of their host time."""
        spec = _FAST_SPECS.get(cls)
        if spec is None:   # every field in definition order (merging keeps that order), factories
            fields = cls.model_fields
            spec = _FAST_SPECS[cls] = ({n: f.default for n, f in fields.items()},
                                       [(n, f.default_factory) for n, f in fields.items() if f.default_factory])
        d = {**spec[0], **values}
        for name, fac in spec[1]:
            if name not in values:
                d[name] = fac()
        m = cls.__new__(cls)
        object.__setattr__(m, "__dict__", d)
        object.__setattr__(m, "__pydantic_fields_set__", set(values))
        object.__setattr__(m, "__pydantic_extra__", {})
        object.__setattr__(m, "__pydantic_private__", None)
        return m


# ---------------------------------------------------------------- kube basics
class OwnerReference(KModel):
    api_version: Optional[str] = None
    kind: str = ""
    name: str = ""
    uid: Optional[str] = None
    controller: Optional[bool] = None


class ObjectMeta(KModel):
    name: str = ""
    namespace: Optional[str] = None
    uid: Optional[str] = None
    resource_version: Optional[str] = None
    generation: Optional[int] = None
    labels: Optional[dict[str, str]] = None
    annotations: Optional[dict[str, str]] = None
    owner_references: Optional[list[OwnerReference]] = None
    creation_timestamp: Optional[str] = None


class LabelSelectorRequirement(KModel):
    key: str
    operator: str
    values: Optional[list[str]] = None


class LabelSelector(KModel):
    match_labels: Optional[dict[str, str]] = None
    match_expressions: Optional[list[LabelSelectorRequirement]] = None


# ---------------------------------------------------------------- Podmortem
class AIProviderRef(KModel):
    name: Optional[str] = None
    namespace: Optional[str] = None


class PodmortemSpec(KModel):
    pod_selector: Optional[LabelSelector] = None
    ai_provider_ref: Optional[AIProviderRef] = None
    ai_analysis_enabled: Optional[bool] = True  # CRD default (podmortem-crd.yaml:49-52)


class PodFailureStatus(KModel):
    pod_name: Optional[str] = None
    pod_namespace: Optional[str] = None
    failure_time: Optional[str] = None
    analysis_status: Optional[str] = None
    explanation: Optional[str] = None


class PodmortemStatus(KModel):
    phase: Optional[str] = None  # Pending | Ready | Processing | Error
    message: Optional[str] = None
    last_update: Optional[str] = None
    observed_generation: Optional[int] = None
    recent_failures: Optional[list[PodFailureStatus]] = None


class Podmortem(KModel):
    api_version: str = API_VERSION
    kind: str = "Podmortem"
    metadata: ObjectMeta = Field(default_factory=ObjectMeta)
    spec: Optional[PodmortemSpec] = None
    status: Optional[PodmortemStatus] = None


# ---------------------------------------------------------------- PatternLibrary
class RepoCredentials(KModel):
    secret_ref: Optional[str] = None


class PatternRepository(KModel):
    name: str
    url: str
    branch: Optional[str] = "main"
    credentials: Optional[RepoCredentials] = None


class PatternLibrarySpec(KModel):
    repositories: Optional[list[PatternRepository]] = None
    refresh_interval: Optional[str] = "1h"
    enabled_libraries: Optional[list[str]] = None


class SyncedRepository(KModel):
    name: Optional[str] = None
    last_commit: Optional[str] = None
    sync_time: Optional[str] = None
    status: Optional[str] = None  # Success | Failed
    error: Optional[str] = None


class PatternLibraryStatus(KModel):
    phase: Optional[str] = None  # Pending | Syncing | Ready | Failed
    message: Optional[str] = None
    last_sync_time: Optional[str] = None
    synced_repositories: Optional[list[SyncedRepository]] = None
    available_libraries: Optional[list[str]] = None
    observed_generation: Optional[int] = None


class PatternLibrary(KModel):
    api_version: str = API_VERSION
    kind: str = "PatternLibrary"
    metadata: ObjectMeta = Field(default_factory=ObjectMeta)
    spec: Optional[PatternLibrarySpec] = None
    status: Optional[PatternLibraryStatus] = None


# ---------------------------------------------------------------- AIProvider
class AuthenticationRef(KModel):
    secret_name: Optional[str] = None
    secret_key: Optional[str] = None


class AIProviderSpec(KModel):
    provider_id: Optional[str] = None
    api_url: Optional[str] = None
    model_id: Optional[str] = None
    authentication_ref: Optional[AuthenticationRef] = None
    timeout_seconds: Optional[int] = None
    max_retries: Optional[int] = None
    caching_enabled: Optional[bool] = None
    prompt_template: Optional[str] = None
    max_tokens: Optional[int] = None
    temperature: Optional[float] = None
    additional_config: Optional[dict[str, str]] = None


class AIProviderStatus(KModel):
    phase: Optional[str] = None  # Pending | Ready | Failed
    message: Optional[str] = None
    last_validated: Optional[str] = None
    observed_generation: Optional[int] = None


class AIProvider(KModel):
    api_version: str = API_VERSION
    kind: str = "AIProvider"
    metadata: ObjectMeta = Field(default_factory=ObjectMeta)
    spec: Optional[AIProviderSpec] = None
    status: Optional[AIProviderStatus] = None


# ---------------------------------------------------------------- analysis DTOs
class MatchedPattern(KModel):
    id: Optional[str] = None
    name: Optional[str] = None
    severity: Optional[str] = None
    category: Optional[str] = None
    library: Optional[str] = None


class AnalysisEvent(KModel):
    line_number: int = 0                         # 1-based line in the pod log
    matched_pattern: Optional[MatchedPattern] = None
    score: float = 0.0
    context: list[str] = Field(default_factory=list)
    matched_line: Optional[str] = None
    remediation: Optional[dict[str, Any]] = None


class AnalysisSummary(KModel):
    highest_severity: Optional[str] = None
    significant_events: int = 0
    total_events: int = 0
    severity_distribution: dict[str, int] = Field(default_factory=dict)


class AnalysisResult(KModel):
    analysis_id: Optional[str] = None
    pod_name: Optional[str] = None
    pod_namespace: Optional[str] = None
    events: Optional[list[AnalysisEvent]] = None
    summary: Optional[AnalysisSummary] = None
    metadata: dict[str, Any] = Field(default_factory=dict)


class PodFailureData(KModel):
    """Body the reference POSTs to the log-parser (J/service/PodFailureWatcher.java:334)."""
    pod: dict[str, Any] = Field(default_factory=dict)
    logs: Optional[str] = None
    events: list[dict[str, Any]] = Field(default_factory=list)


class AIProviderConfig(KModel):
    provider_id: Optional[str] = None
    api_url: Optional[str] = None
    model_id: Optional[str] = None
    timeout_seconds: int = 30
    max_retries: int = 3
    caching_enabled: bool = True
    prompt_template: Optional[str] = None
    max_tokens: int = 500
    temperature: float = 0.3
    additional_headers: Optional[dict[str, str]] = None
    auth_token: Optional[str] = None


class AnalysisRequest(KModel):
    analysis_result: AnalysisResult
    provider_config: AIProviderConfig


class AIResponse(KModel):
    explanation: Optional[str] = None
    provider_id: Optional[str] = None
    model_id: Optional[str] = None
    tokens_generated: Optional[int] = None
    latency_ms: Optional[float] = None
    cached: Optional[bool] = None
    # on-node engine stage timings (absent from remote providers)
    prompt_tokens: Optional[int] = None
    queue_ms: Optional[float] = None      # request -> first token (admission wait + prefill)
    decode_ms: Optional[float] = None     # first token -> last token
