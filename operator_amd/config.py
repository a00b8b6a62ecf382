"""Typed configuration.

Precedence: defaults < YAML file (``--config`` / ``PODMORTEM_CONFIG``) <
environment ``PODMORTEM_<SECTION>__<KEY>`` < explicit overrides.
Every reference config key / hard-coded constant has a home here, with the
reference's default:

reference                                             here
----------------------------------------------------  ---------------------------------------
quarkus.application.name=podmortem-operator           operator.name
pattern.cache.directory=/shared/patterns (ignored!)   patterns.cache_dir (honoured: Q10)
quarkus.rest-client.log-parser.url / timeouts 30/10s  services.log_parser_url / *_timeout_s
quarkus.rest-client.ai-interface.url / 180/120s       services.ai_interface_url / *_timeout_s
podmortem.watch.namespaces                            watch.namespaces
quarkus.kubernetes-client.namespace=default           kube.namespace
MAX_RECENT_FAILURES=10 (AnalysisStorageService:48)    storage.max_recent_failures
5 retries / 100 ms backoff (:75-76)                   storage.max_retries / initial_backoff_s
watch restart 5 s (PodFailureWatcher:574)             watch.restart_delay_s
readiness grace 5 min (ReadinessCheck:26)             health.grace_s
event caps 850 / 900 (EventService:87,117)            (constants, controller/events.py)
refresh default 1h (PatternLibraryReconciler)         (grammar default, controller/patternlibrary.py)
AIProvider defaults 30s/3/true/500/0.3                (controller/ai_client.py DEFAULTS)
"""
from __future__ import annotations

import os
from typing import Any, Optional

import yaml
from pydantic import BaseModel, Field


class OperatorCfg(BaseModel):
    name: str = "podmortem-operator"
    workers: int = 0                  # analysis pipeline threads; 0 = auto: a failure holds one through its
                                      # explanation, so 2 x engine.max_batch x GPUs (+16) keep the engines'
                                      # batches full while the previous batch's results are written
    io_workers: int = 8               # kube write pool (annotations, status, events)
    sink_concurrency: int = 0         # analyses writing their results at once (annotations, status ring,
                                      # Events); 0 = unbounded. A bound keeps a wave of result writes from
                                      # starving the next failures' watch -> collect -> scan -> prompt path
    leader_election: bool = False     # reference: 1 replica, no lease; true = HA replicas behind a Lease
    lease_name: str = "podmortem-operator-leader"
    lease_namespace: str = "podmortem-system"
    lease_duration_s: float = 15.0
    lease_renew_deadline_s: float = 10.0
    lease_retry_period_s: float = 2.0
    # operator shards: shard_count processes split the pods by a stable hash of ns/name
    # (each its own engines and, with leader election, its own lease); 1 = no sharding
    shard_count: int = 1
    shard_index: int = 0


class KubeCfg(BaseModel):
    mode: str = "auto"                # auto | incluster | kubeconfig | fake
    kubeconfig: Optional[str] = None
    namespace: str = "default"
    request_timeout_s: float = 30.0


class WatchCfg(BaseModel):
    namespaces: str = ""
    restart_delay_s: float = 5.0
    include_last_state: bool = False  # treat lastState.terminated (CrashLoopBackOff) as a failure
    include_init_containers: bool = False
    # Q11: the reference fetches the default container's whole current log
    log_container: Optional[str] = None     # a fixed container name instead of the default one
    log_previous: bool = False              # the previous (crashed) instance's log
    log_limit_bytes: Optional[int] = None   # tail bytes cap (None = whole log, as the reference)
    dedupe_max_entries: int = 100_000
    dedupe_ttl_s: float = 7 * 24 * 3600


class StorageCfg(BaseModel):
    max_recent_failures: int = 10
    max_retries: int = 5
    initial_backoff_s: float = 0.1
    # operator.shard_count > 1: N processes prepend to ONE Podmortem's recentFailures ring
    # (GET + PATCH with resourceVersion), so conflicts are N-fold: a larger 409 budget and
    # jittered delays for the status writes (the reference has a single writer)
    sharded_max_retries: int = 12
    sharded_jitter: float = 0.5
    failure_time_from_pod: bool = False  # Q5: reference records now(); true = container finishedAt


class PatternsCfg(BaseModel):
    cache_dir: str = "/shared/patterns"
    builtin_catalog: bool = True      # ship the built-in failure catalog beside synced libraries
    seg_bytes: int = 1024
    max_events: int = 50
    significance_threshold: float = 0.5


class ServicesCfg(BaseModel):
    match: str = "local"              # local | remote | cpu | stub (fixed result: plumbing benchmarks)
    explain: str = "local"            # local | remote | echo | none
    log_parser_url: str = "http://podmortem-log-parser-service.podmortem-system.svc.cluster.local:8080"
    log_parser_read_timeout_s: float = 30.0
    log_parser_connect_timeout_s: float = 10.0
    ai_interface_url: str = "http://podmortem-ai-interface-service.podmortem-system.svc.cluster.local:8080"
    ai_interface_read_timeout_s: float = 180.0
    ai_interface_connect_timeout_s: float = 120.0
    match_batch_wait_ms: float = 2.0
    match_max_batch: int = 1024
    external_providers: bool = True   # AIProviders with providerId openai/ollama call their apiUrl directly


class EngineCfg(BaseModel):
    gpus: int = 1                     # engine processes (one per GPU) behind the controller
    pool: bool = False                # run the engines out of process even with one GPU
    pool_log_arena_mb: float = 64     # per engine worker: shared-memory ring the pod logs travel through
    model: str = "llama3-8b"
    model_path: Optional[str] = None  # HF safetensors dir (its config.json wins over `model`); random init when absent
    chat_template: str = "auto"       # auto = the checkpoint's tokenizer_config.json template; none; a file; Jinja
    extra_models: list[str] = []      # more local models on the same GPU(s): "preset" or "name=/hf/dir"; an
                                      # AIProvider whose modelId names one is served by it (KV budget split)
    seed: int = 0
    weight_cache_dir: str = ""        # ready-to-run weight shards as safetensors, mmapped at start
    dtype: str = "bfloat16"
    weight_dtype: str = "bfloat16"   # bfloat16 | fp8 (W8A8 e4m3fn projections, e.g. Llama-3-70B)
    device: str = "cuda"
    tp: int = 1
    oneshot_allreduce_mb: float = 8.0  # TP all-reduces up to this size use the IPC kernels; 0 = RCCL only
    # one-shot / two-shot / RCCL crossovers: 0 = measured on the node when the TP group starts
    # (custom_ar.OneShotAllReduce.calibrate over the decode buckets' message sizes); > 0 = override:
    # one-shot up to this size, two-shot (reduce-scatter + all-gather) above
    oneshot_max_kb: float = 0.0
    allreduce_calibrate_iters: int = 20
    max_batch: int = 256
    max_prefill_tokens: int = 32768   # tokens per prefill batch (profiles/prefill_batch_sweep_8b.jsonl)
    admit_wait_ms: float = 5.0        # idle engine: gather arrivals this long before a partial prefill (5 vs 20: +0.9 %, profiles/admit_wait_ab_r6.jsonl)
    max_context: int = 4096
    max_prompt_tokens: int = 1536
    kv_cache_gb: float = 64.0
    kv_dtype: str = "auto"            # auto = the compute dtype; fp8 = OCP e4m3fn cache (half the bytes; not the default)
    kv_scale: float = 1.0             # fp8 cache: stored value = x / kv_scale (keys and values)
    # KV page (tokens): 16 lets a shared prompt prefix cover 112 of the explanation prompts'
    # 122 common tokens (64: 64); flagship 31.6 vs 30.6 analyses/s (profiles/bench_prefix_sharing_ab.jsonl)
    page_size: int = 16
    use_graphs: bool = True
    prefill_graphs: bool = True       # full-ish prefill batches replay a captured bucket graph
    prefix_sharing: bool = True       # prompts starting with the same whole KV pages share them (computed once)
    warmup_graphs: bool = True        # engine processes capture their graphs before reporting ready
    multi_step: int = 8
    ignore_eos: bool = False


class HealthCfg(BaseModel):
    port: int = 8080
    host: str = "0.0.0.0"
    grace_s: float = 300.0
    enabled: bool = True


class Settings(BaseModel):
    operator: OperatorCfg = Field(default_factory=OperatorCfg)
    kube: KubeCfg = Field(default_factory=KubeCfg)
    watch: WatchCfg = Field(default_factory=WatchCfg)
    storage: StorageCfg = Field(default_factory=StorageCfg)
    patterns: PatternsCfg = Field(default_factory=PatternsCfg)
    services: ServicesCfg = Field(default_factory=ServicesCfg)
    engine: EngineCfg = Field(default_factory=EngineCfg)
    health: HealthCfg = Field(default_factory=HealthCfg)


def _set_path(d: dict, path: list[str], value: Any) -> None:
    for p in path[:-1]:
        d = d.setdefault(p, {})
    d[path[-1]] = value


def _coerce(v: str) -> Any:
    try:
        return yaml.safe_load(v)
    except yaml.YAMLError:
        return v


def load_settings(path: str | None = None, env: dict[str, str] | None = None,
                  overrides: dict[str, Any] | None = None) -> Settings:
    env = dict(os.environ if env is None else env)
    data: dict = {}
    path = path or env.get("PODMORTEM_CONFIG")
    if path:
        with open(path) as f:
            data = yaml.safe_load(f) or {}
    for k, v in env.items():
        if not k.startswith("PODMORTEM_") or k == "PODMORTEM_CONFIG":
            continue
        parts = [p.lower() for p in k[len("PODMORTEM_"):].split("__")]
        if len(parts) == 2:
            _set_path(data, parts, _coerce(v))
    # the reference's own property name keeps working (PodFailureWatcher.java:52)
    if "PODMORTEM_WATCH_NAMESPACES" in env:
        _set_path(data, ["watch", "namespaces"], env["PODMORTEM_WATCH_NAMESPACES"])
    for k, v in (overrides or {}).items():
        _set_path(data, k.split("."), v)
    return Settings.model_validate(data)
