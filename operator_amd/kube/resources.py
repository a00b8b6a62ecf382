"""Resource descriptors, API errors, label/field selectors.

Every kube verb the reference issues goes through one
of these descriptors, for both the in-memory FakeKube and the HTTPS client.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Any, Iterable, Mapping


@dataclass(frozen=True)
class Resource:
    group: str
    version: str
    plural: str
    kind: str
    namespaced: bool = True

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    def base_path(self, namespace: str | None) -> str:
        root = f"/apis/{self.group}/{self.version}" if self.group else f"/api/{self.version}"
        if self.namespaced and namespace:
            return f"{root}/namespaces/{namespace}/{self.plural}"
        return f"{root}/{self.plural}"


PODS = Resource("", "v1", "pods", "Pod")
CORE_EVENTS = Resource("", "v1", "events", "Event")
EVENTS = Resource("events.k8s.io", "v1", "events", "Event")
SECRETS = Resource("", "v1", "secrets", "Secret")
CONFIGMAPS = Resource("", "v1", "configmaps", "ConfigMap")
NAMESPACES = Resource("", "v1", "namespaces", "Namespace", namespaced=False)
REPLICASETS = Resource("apps", "v1", "replicasets", "ReplicaSet")
DEPLOYMENTS = Resource("apps", "v1", "deployments", "Deployment")
LEASES = Resource("coordination.k8s.io", "v1", "leases", "Lease")
PODMORTEMS = Resource("podmortem.redhat.com", "v1alpha1", "podmortems", "Podmortem")
PATTERNLIBRARIES = Resource("podmortem.redhat.com", "v1alpha1", "patternlibraries", "PatternLibrary")
AIPROVIDERS = Resource("podmortem.redhat.com", "v1alpha1", "aiproviders", "AIProvider")

ALL = [PODS, CORE_EVENTS, EVENTS, SECRETS, CONFIGMAPS, NAMESPACES, REPLICASETS, DEPLOYMENTS, LEASES, PODMORTEMS,
       PATTERNLIBRARIES, AIPROVIDERS]
BY_KIND = {(r.api_version, r.kind): r for r in ALL}


class ApiError(Exception):
    """A Kubernetes API failure with its HTTP status code (409 conflict, 403 forbidden, ...)."""

    def __init__(self, code: int, message: str = "", reason: str = ""):
        super().__init__(f"{code} {reason}: {message}".strip())
        self.code = code
        self.reason = reason
        self.message = message


class WatchClosed(Exception):
    """Raised by a watch iterator when the stream closes with an error.

    ``code`` is the status of the apiserver's ERROR event when there was one:
    410 (Gone / Expired) means the requested resourceVersion has been compacted
    away, so resuming from it can never succeed: the caller must relist."""

    def __init__(self, message: str = "", code: int | None = None):
        super().__init__(message)
        self.code = code

    @property
    def expired(self) -> bool:
        return self.code == 410


# ---------------------------------------------------------------- label selectors
def match_labels(selector: Mapping[str, str] | None, labels: Mapping[str, str] | None) -> bool:
    """All selector pairs present & equal (J/service/PodFailureWatcher.java:263-264)."""
    labels = labels or {}
    return all(labels.get(k) == v for k, v in (selector or {}).items())


def _expr_ok(expr: Mapping[str, Any], labels: Mapping[str, str]) -> bool:
    key, op = expr.get("key"), str(expr.get("operator", ""))
    vals = list(expr.get("values") or [])
    has = key in labels
    if op == "In":
        return has and labels[key] in vals
    if op == "NotIn":
        return not has or labels[key] not in vals
    if op == "Exists":
        return has
    if op == "DoesNotExist":
        return not has
    raise ValueError(f"unknown label selector operator {op!r}")


def selector_is_empty(sel: Mapping[str, Any] | None) -> bool:
    return not sel or (not sel.get("matchLabels") and not sel.get("matchExpressions"))


def as_selector(sel: Mapping[str, Any] | None) -> Mapping[str, Any] | None:
    """A LabelSelector as is; a plain {label: value} map as its matchLabels."""
    if sel and "matchLabels" not in sel and "matchExpressions" not in sel:
        return {"matchLabels": dict(sel)}
    return sel


def match_selector(sel: Mapping[str, Any] | None, labels: Mapping[str, str] | None) -> bool:
    """Full metav1.LabelSelector semantics (matchLabels AND matchExpressions).
    An empty/absent selector matches everything here; callers decide policy."""
    labels = labels or {}
    sel = as_selector(sel)
    if not sel:
        return True
    if not match_labels(sel.get("matchLabels"), labels):
        return False
    return all(_expr_ok(e, labels) for e in (sel.get("matchExpressions") or []))


_SET_RE = re.compile(r"^\s*([A-Za-z0-9_./-]+)\s+(in|notin)\s+\(([^)]*)\)\s*$")


def selector_to_string(sel: Mapping[str, Any] | None) -> str:
    sel = as_selector(sel)
    if not sel:
        return ""
    parts = [f"{k}={v}" for k, v in sorted((sel.get("matchLabels") or {}).items())]
    for e in sel.get("matchExpressions") or []:
        op, k, vals = e["operator"], e["key"], ",".join(e.get("values") or [])
        parts.append({"In": f"{k} in ({vals})", "NotIn": f"{k} notin ({vals})", "Exists": k,
                      "DoesNotExist": f"!{k}"}[op])
    return ",".join(parts)


def parse_selector(s: str | None) -> dict:
    """Parse a string label selector ('a=b,c!=d,e in (x,y),!f,g') into LabelSelector form."""
    sel: dict[str, Any] = {"matchLabels": {}, "matchExpressions": []}
    if not s:
        return sel
    depth, cur, items = 0, "", []
    for ch in s:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            items.append(cur)
            cur = ""
        else:
            cur += ch
    items.append(cur)
    for it in (i.strip() for i in items):
        if not it:
            continue
        m = _SET_RE.match(it)
        if m:
            sel["matchExpressions"].append({"key": m.group(1), "operator": "In" if m.group(2) == "in" else "NotIn",
                                            "values": [v.strip() for v in m.group(3).split(",") if v.strip()]})
        elif "!=" in it:
            k, v = it.split("!=", 1)
            sel["matchExpressions"].append({"key": k.strip(), "operator": "NotIn", "values": [v.strip()]})
        elif "==" in it or "=" in it:
            k, v = it.split("==", 1) if "==" in it else it.split("=", 1)
            sel["matchLabels"][k.strip()] = v.strip()
        elif it.startswith("!"):
            sel["matchExpressions"].append({"key": it[1:].strip(), "operator": "DoesNotExist"})
        else:
            sel["matchExpressions"].append({"key": it, "operator": "Exists"})
    return sel


# ---------------------------------------------------------------- field selectors
def _dig(obj: Mapping[str, Any], path: str) -> Any:
    cur: Any = obj
    for p in path.split("."):
        if not isinstance(cur, Mapping):
            return None
        cur = cur.get(p)
    return cur


def match_fields(field_selector: str | None, obj: Mapping[str, Any]) -> bool:
    if not field_selector:
        return True
    for term in field_selector.split(","):
        term = term.strip()
        if not term:
            continue
        if "!=" in term:
            k, v = term.split("!=", 1)
            if str(_dig(obj, k.strip())) == v.strip():
                return False
        else:
            k, v = term.split("==", 1) if "==" in term else term.split("=", 1)
            got = _dig(obj, k.strip())
            if got is None or str(got) != v.strip():
                return False
    return True


def iter_containers_terminated(pod: Mapping[str, Any]) -> Iterable[Mapping[str, Any]]:
    st = (pod or {}).get("status") or {}
    for cs in st.get("containerStatuses") or []:
        term = ((cs or {}).get("state") or {}).get("terminated")
        if term:
            yield term
