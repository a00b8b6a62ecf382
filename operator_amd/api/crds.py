"""CRD + deployment manifests, generated from Python.

The three CRDs are schema-equivalent to the reference's
(src/main/kubernetes/{podmortem,patternlibrary,aiprovider}-crd.yaml: same
group/version/kind/plural/shortNames/scope, same properties, types, enums,
defaults, required fields and status subresource; descriptions are ours).
tests/test_crds.py checks the equivalence against the reference files when
they are present.

Deployment shape (ours): the operator and its GPU engines are ONE pod per
node-GPU group (no separate log-parser / ai-interface services),
requesting ``amd.com/gpu``. RBAC adds ``apps`` get/list for the owner lookup of
Events (the reference's ClusterRole lacks it: SURVEY.md Q9).
"""
from __future__ import annotations

from typing import Any

import yaml

from .models import GROUP, VERSION


def _s(desc: str | None = None, **kw) -> dict:
    d: dict[str, Any] = {"type": "string", **kw}
    if desc:
        d["description"] = desc
    return d


def _i(desc: str | None = None, **kw) -> dict:
    d: dict[str, Any] = {"type": "integer", **kw}
    if desc:
        d["description"] = desc
    return d


def _b(desc: str | None = None, **kw) -> dict:
    d: dict[str, Any] = {"type": "boolean", **kw}
    if desc:
        d["description"] = desc
    return d


def _o(props: dict | None = None, desc: str | None = None, **kw) -> dict:
    d: dict[str, Any] = {"type": "object"}
    if props is not None:
        d["properties"] = props
    d.update(kw)
    if desc:
        d["description"] = desc
    return d


def _a(items: dict, desc: str | None = None) -> dict:
    d: dict[str, Any] = {"type": "array", "items": items}
    if desc:
        d["description"] = desc
    return d


def _ts(desc: str | None = None) -> dict:
    return _s(desc, format="date-time")


def _gen() -> dict:
    return _i(format="int64")


def _crd(kind: str, plural: str, short: str, spec: dict, status: dict) -> dict:
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{plural}.{GROUP}"},
        "spec": {
            "group": GROUP,
            "versions": [{"name": VERSION, "served": True, "storage": True,
                          "schema": {"openAPIV3Schema": _o({"spec": spec, "status": status})},
                          "subresources": {"status": {}}}],
            "scope": "Namespaced",
            "names": {"plural": plural, "singular": kind.lower(), "kind": kind, "shortNames": [short]},
        },
    }


def podmortem_crd() -> dict:
    selector = _o({
        "matchLabels": _o(additionalProperties=_s()),
        "matchExpressions": _a(_o({"key": _s(), "operator": _s(), "values": _a(_s())})),
    }, "Selects the pods whose failures this monitor analyses")
    spec = _o({
        "podSelector": selector,
        "aiProviderRef": _o({"name": _s("AIProvider name"),
                             "namespace": _s("AIProvider namespace (default: this monitor's namespace)")},
                            "AIProvider used for explanations"),
        "aiAnalysisEnabled": _b("Generate an explanation for each analysed failure", default=True),
    })
    failure = _o({"podName": _s(), "podNamespace": _s(), "failureTime": _ts(), "analysisStatus": _s(),
                  "explanation": _s()})
    status = _o({
        "phase": _s(enum=["Pending", "Ready", "Processing", "Error"]),
        "message": _s(), "lastUpdate": _ts(), "observedGeneration": _gen(),
        "recentFailures": _a(failure),
    })
    return _crd("Podmortem", "podmortems", "pm", spec, status)


def patternlibrary_crd() -> dict:
    repo = _o({
        "name": _s("Repository identifier"),
        "url": _s("Git URL of the pattern repository"),
        "branch": _s("Branch to track", default="main"),
        "credentials": _o({"secretRef": _s("Secret with git credentials (key 'token')")}, "HTTPS credentials"),
    }, required=["name", "url"])
    spec = _o({
        "repositories": _a(repo),
        "refreshInterval": _s("Sync period, e.g. 30m, 1h, 1h30m", default="1h"),
        "enabledLibraries": _a(_s(), "Library ids to load (default: all)"),
    })
    synced = _o({"name": _s(), "lastCommit": _s(), "syncTime": _ts(),
                 "status": _s(enum=["Success", "Failed"]), "error": _s()})
    status = _o({
        "phase": _s("Sync state", enum=["Pending", "Syncing", "Ready", "Failed"]),
        "message": _s("Human readable state"),
        "lastSyncTime": _ts("Last synchronisation"),
        "syncedRepositories": _a(synced, "Per-repository sync result"),
        "availableLibraries": _a(_s(), "Pattern libraries found in the synced repositories"),
        "observedGeneration": _gen(),
    })
    return _crd("PatternLibrary", "patternlibraries", "pl", spec, status)


def aiprovider_crd() -> dict:
    spec = _o({
        "providerId": _s("Provider identifier (e.g. local, openai, ollama)"),
        "apiUrl": _s("Provider base URL (informational for the on-node engine)"),
        "modelId": _s("Model identifier"),
        "authenticationRef": _o({"secretName": _s(), "secretKey": _s()}, "Secret holding the API token"),
        "timeoutSeconds": _i("Per-attempt timeout", default=30),
        "maxRetries": _i("Retries after a failed attempt", default=3),
        "cachingEnabled": _b("Cache responses for identical prompts", default=True),
        "promptTemplate": _s("Prompt template with {placeholders}"),
        "maxTokens": _i("Generation cap", default=500),
        "temperature": {"type": "number", "default": 0.3, "description": "Sampling temperature"},
        "additionalConfig": _o(additionalProperties=_s(), desc="Provider specific settings"),
    })
    status = _o({"phase": _s(enum=["Pending", "Ready", "Failed"]), "message": _s(), "lastValidated": _ts(),
                 "observedGeneration": _gen()})
    return _crd("AIProvider", "aiproviders", "aip", spec, status)


def crds() -> list[dict]:
    return [podmortem_crd(), patternlibrary_crd(), aiprovider_crd()]


def rbac(namespace: str = "podmortem-system", name: str = "podmortem-operator") -> list[dict]:
    return [
        {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": name, "namespace": namespace}},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole", "metadata": {"name": name},
         "rules": [
             {"apiGroups": [GROUP], "resources": ["aiproviders", "podmortems", "patternlibraries"],
              "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]},
             {"apiGroups": [GROUP], "resources": ["aiproviders/status", "podmortems/status",
                                                  "patternlibraries/status"], "verbs": ["get", "update", "patch"]},
             {"apiGroups": [""], "resources": ["pods", "configmaps", "secrets", "events"],
              "verbs": ["get", "list", "watch", "create", "patch"]},
             {"apiGroups": [""], "resources": ["pods/log"], "verbs": ["get"]},
             {"apiGroups": ["events.k8s.io"], "resources": ["events"],
              "verbs": ["get", "list", "watch", "create", "patch"]},
             {"apiGroups": ["apps"], "resources": ["replicasets", "deployments"], "verbs": ["get", "list"]},
             {"apiGroups": ["coordination.k8s.io"], "resources": ["leases"],
              "verbs": ["get", "create", "update", "patch"]},
         ]},
        {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding", "metadata": {"name": name},
         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": name},
         "subjects": [{"kind": "ServiceAccount", "name": name, "namespace": namespace}]},
    ]


def deployment(namespace: str = "podmortem-system", image: str = "ghcr.io/podmortem/operator-amd:latest",
               gpus: int = 1, name: str = "podmortem-operator", replicas: int = 1, shards: int = 1,
               shard_per_gpu: bool = False) -> list[dict]:
    """PVC + operator Deployment + Service. ``replicas`` > 1 turns on Lease leader
    election (one active replica, the others warm standbys); ``shards`` > 1 runs that
    many operator processes in the pod, splitting the pods between them, each with
    its own engines on the pod's GPUs (``run --shards``); ``shard_per_gpu`` runs one
    operator process per GPU, each owning its GPU and its slice of the pods
    (``run --shard-per-gpu``, the multi-GPU topology ``bench.py --gpus N`` measures)."""
    if shard_per_gpu:
        shards = max(1, gpus)
    labels = {"app.kubernetes.io/name": name}
    env = [{"name": "PODMORTEM_PATTERNS__CACHE_DIR", "value": "/shared/patterns"},
           {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]
    if replicas > 1:
        env += [{"name": "PODMORTEM_OPERATOR__LEADER_ELECTION", "value": "true"},
                {"name": "PODMORTEM_OPERATOR__LEASE_NAMESPACE", "value": namespace}]
    probe = lambda path, d: {"httpGet": {"path": path, "port": 8080}, "initialDelaySeconds": d,  # noqa: E731
                             "periodSeconds": 10}
    return [
        {"apiVersion": "v1", "kind": "PersistentVolumeClaim",
         "metadata": {"name": "pattern-cache-pvc", "namespace": namespace},
         "spec": {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "5Gi"}}}},
        {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "namespace": namespace,
                                                                     "labels": labels},
         "spec": {"replicas": replicas, "selector": {"matchLabels": labels},
                  "template": {"metadata": {"labels": labels}, "spec": {
                      "serviceAccountName": name,
                      "securityContext": {"runAsNonRoot": True, "runAsUser": 1001},
                      "containers": [{
                          "name": "operator", "image": image,
                          "command": ["python", "-m", "operator_amd", "run", "--gpus", str(gpus)] +
                                     (["--shard-per-gpu"] if shard_per_gpu else
                                      ["--shards", str(shards)] if shards > 1 else []),
                          "env": env,
                          "ports": [{"containerPort": 8080, "name": "http"}],
                          "resources": {"limits": {"amd.com/gpu": gpus, "memory": f"{64 * max(1, shards)}Gi"},
                                        "requests": {"cpu": str(4 * max(1, shards)),
                                                     "memory": f"{32 * max(1, shards)}Gi"}},
                          "livenessProbe": probe("/q/health/live", 30),
                          "readinessProbe": probe("/q/health/ready", 30),
                          "volumeMounts": [{"name": "pattern-cache", "mountPath": "/shared/patterns"},
                                           {"name": "dshm", "mountPath": "/dev/shm"}]}],
                      "volumes": [{"name": "pattern-cache", "persistentVolumeClaim": {"claimName": "pattern-cache-pvc"}},
                                  {"name": "dshm", "emptyDir": {"medium": "Memory"}}]}}}},
        {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "namespace": namespace, "labels": labels},
         "spec": {"selector": labels, "ports": [{"name": "http", "port": 8080, "targetPort": 8080}]}},
    ]


def compat_services(namespace: str = "podmortem-system", image: str = "ghcr.io/podmortem/operator-amd:latest",
                    gpus: int = 1) -> list[dict]:
    """The on-node engines behind the reference's two service names
    (K/log-parser-deployment.yaml + K/log-parser-service.yaml,
    K/ai-interface-deployment.yaml + K/ai-interface-service.yaml): an unmodified
    reference operator pointed at these Services gets GPU pattern analysis and
    local-LLM explanations (``operator_amd serve-compat``)."""
    out = []
    for svc, role in (("podmortem-log-parser", "match"), ("podmortem-ai-interface", "explain")):
        labels = {"app.kubernetes.io/name": svc}
        env = [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
               {"name": "PODMORTEM_SERVICES__EXPLAIN", "value": "local" if role == "explain" else "none"}]
        res = {"limits": {"amd.com/gpu": gpus, "memory": "64Gi"}, "requests": {"cpu": "4", "memory": "16Gi"}}
        out += [
            {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": svc, "namespace": namespace,
                                                                         "labels": labels},
             "spec": {"replicas": 1, "selector": {"matchLabels": labels},
                      "template": {"metadata": {"labels": labels}, "spec": {
                          "securityContext": {"runAsNonRoot": True, "runAsUser": 1001},
                          "containers": [{"name": svc, "image": image,
                                          "command": ["python", "-m", "operator_amd", "serve-compat", "--port", "8080"],
                                          "env": env, "ports": [{"containerPort": 8080, "name": "http"}],
                                          "resources": res,
                                          "readinessProbe": {"httpGet": {"path": "/q/health/ready", "port": 8080},
                                                             "initialDelaySeconds": 30, "periodSeconds": 10}}]}}}},
            {"apiVersion": "v1", "kind": "Service", "metadata": {"name": f"{svc}-service", "namespace": namespace},
             "spec": {"selector": labels, "ports": [{"name": "http", "port": 8080, "targetPort": 8080}]}},
        ]
    return out


def render_all(**kw) -> str:
    compat = kw.pop("compat", False)
    docs = crds() + rbac(kw.get("namespace", "podmortem-system")) + deployment(**kw)
    if compat:
        docs += compat_services(kw.get("namespace", "podmortem-system"), kw.get("image", "ghcr.io/podmortem/operator-amd:latest"),
                                kw.get("gpus", 1))
    return yaml.safe_dump_all(docs, sort_keys=False)
