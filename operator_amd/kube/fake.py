"""FakeKube: an in-memory Kubernetes API server for tests and the plumbing
benchmark (SURVEY.md §4.2 "Controller integration, CPU"; BASELINE config 1).

The reference has no test double at all. FakeKube models the
behaviour the controllers depend on:

* namespaced objects with uid / resourceVersion / generation / creationTimestamp;
  optimistic concurrency: a write carrying a stale resourceVersion -> 409;
* JSON merge patch (RFC 7386) on objects and on the ``status`` subresource
  (status writes never touch spec and do not bump generation);
* list with label + field selectors; ``pods/log`` subresource;
* watches (ADDED / MODIFIED / DELETED / BOOKMARK) with resourceVersion resume,
  close-with-error injection, server-side clean close (``end_watches``: the
  apiserver ends every watch after its min-request-timeout) and history
  compaction (``compact``: a watch from a compacted resourceVersion fails with
  410 Gone, as etcd compaction makes it on a real apiserver);
* a fault matrix: ``inject(verb, plural, code, times)`` makes the next N
  matching calls raise ApiError(code) (409 / 403 / 500 ...);
* a call journal (``calls``) so tests can assert on the exact verbs issued.

Thread-safe; every read returns a deep copy.
"""
from __future__ import annotations

import itertools
import json
import queue
import threading
import uuid
from collections import defaultdict
from typing import Any, Iterator

from operator_amd.utils.timefmt import instant_str

from .resources import (ALL, PODS, ApiError, Resource, WatchClosed, match_fields, match_selector, parse_selector)


_KEYS: dict[int, tuple[Resource, str]] = {}


def _res_key(res: Resource) -> str:
    """Store key of a resource, computed once per Resource object (every verb needs it;
    the dataclass property + f-string per call showed in the API server's profile)."""
    e = _KEYS.get(id(res))
    if e is None or e[0] is not res:
        e = _KEYS[id(res)] = (res, f"{res.api_version}/{res.plural}")
    return e[1]


def _jcopy(o: Any) -> Any:
    """Deep copy of a JSON value (dicts, lists, scalars): what copy.deepcopy does for
    API objects, without its memo bookkeeping (several times faster; API objects
    have neither cycles nor shared sub-objects that must stay shared)."""
    t = type(o)
    if t is dict:
        return {k: _jcopy(v) for k, v in o.items()}
    if t is list:
        return [_jcopy(v) for v in o]
    return o


def merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return _jcopy(patch)
    out = _jcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


class FakeWatch:
    """Iterator of (type, obj) events; ``close()`` ends it normally."""

    _END = object()

    def __init__(self, fk: "FakeKube", res: Resource, namespace: str | None, sink=None):
        self.fk, self.res, self.namespace = fk, res, namespace
        self.rkey = _res_key(res)   # events match by key (the REST server builds a Resource per request)
        self.q: queue.Queue = queue.Queue()
        # sink(item): deliver events / end / failure markers somewhere else than self.q
        # (the asyncio REST server feeds its watch coroutines this way)
        self._put = sink if sink is not None else self.q.put
        self.closed = False
        self._held = None   # an end / failure marker met while draining (next_events)

    def push(self, typ: str, obj: dict, ev: "_Event | None" = None) -> None:
        if not self.closed:
            self._put(ev if ev is not None else _Event(typ, obj))

    def fail(self, message: str = "watch stream error", code: int | None = None) -> None:
        self._put(WatchClosed(message, code))

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            self._put(self._END)
            self.fk._drop_watch(self)

    def __iter__(self) -> Iterator[tuple[str, dict]]:
        return self

    def next_event(self) -> "_Event":
        """The next event as shared by every watch it went to (the REST server sends its
        memoised wire bytes instead of copying and serialising the object per watcher)."""
        item, self._held = (self._held, None) if self._held is not None else (self.q.get(), None)
        if item is self._END:
            raise StopIteration
        if isinstance(item, WatchClosed):
            self.closed = True
            self.fk._drop_watch(self)
            raise item
        return item

    def next_events(self, max_n: int = 64) -> list["_Event"]:
        """The next event (blocking) plus every one already queued behind it, up to
        ``max_n``: the REST server writes them with one flush."""
        out = [self.next_event()]
        while len(out) < max_n:
            try:
                item = self.q.get_nowait()
            except queue.Empty:
                break
            if item is self._END or isinstance(item, WatchClosed):
                self._held = item   # delivered by the next call
                break
            out.append(item)
        return out

    def __next__(self) -> tuple[str, dict]:
        ev = self.next_event()
        # events carry the stored (never mutated) object; each consumer gets its own
        # copy, made here on its thread rather than under the store's lock
        return ev.typ, _jcopy(ev.obj)


class _Event:
    """One watch event, shared by every watch it is delivered to; ``wire()`` is its
    serialised form, computed once (by whichever consumer asks first)."""
    __slots__ = ("typ", "obj", "_wire")

    def __init__(self, typ: str, obj: dict):
        self.typ, self.obj, self._wire = typ, obj, None

    def wire(self) -> bytes:
        b = self._wire
        if b is None:
            b = self._wire = json.dumps({"type": self.typ, "object": self.obj}, separators=(",", ":")).encode() + b"\n"
        return b


class FakeKube:
    def __init__(self, record_calls: bool = True):
        self.record_calls = record_calls   # off for a long-running API server process (unbounded list)
        self._lock = threading.RLock()
        self._objs: dict[tuple[str, str, str], dict] = {}  # (plural-key, ns, name) -> obj
        self._by_kind: dict[str, dict[tuple[str, str], dict]] = {}
        self._rv = itertools.count(1)
        self._history: list[tuple[int, str, str, dict]] = []  # (rv, plural-key, type, obj)
        self._watches: list[FakeWatch] = []
        self._faults: dict[tuple[str, str], list[int]] = defaultdict(list)
        self._logs: dict[tuple[str, str, str | None], str] = {}
        self._compacted = 0
        self._last_rv = 0
        self.calls: list[tuple[str, str, str | None, str | None]] = []

    # ------------------------------------------------------------------ faults
    def inject(self, verb: str, plural: str, code: int, times: int = 1) -> None:
        """Next ``times`` calls of verb ('get','list','create','patch','patch_status','delete','watch','log')
        on ``plural`` raise ApiError(code)."""
        with self._lock:
            self._faults[(verb, plural)].extend([code] * times)

    def clear_faults(self) -> None:
        with self._lock:
            self._faults.clear()

    def _fault(self, verb: str, res: Resource) -> None:
        if not self._faults.get((verb, res.plural)):   # fast path: nothing injected (no lock round trip)
            return
        with self._lock:
            lst = self._faults.get((verb, res.plural))
            if lst:
                code = lst.pop(0)
                raise ApiError(code, f"injected {verb} {res.plural} failure", {409: "Conflict", 403: "Forbidden",
                                                                                404: "NotFound"}.get(code, "Error"))

    def _log_call(self, verb, res, ns, name) -> None:
        if self.record_calls:
            self.calls.append((verb, res.plural, ns, name))

    # ------------------------------------------------------------------ helpers
    _key = staticmethod(_res_key)

    def _kind(self, key: str) -> dict:
        """Per-resource index {(ns, name): obj} over the same objects as ``_objs``."""
        d = self._by_kind.get(key)
        if d is None:
            d = self._by_kind[key] = {}
        return d

    def _store(self, k: tuple[str, str, str], obj: dict) -> None:
        self._objs[k] = obj
        self._kind(k[0])[k[1:]] = obj

    def _emit(self, res: Resource, typ: str, obj: dict) -> None:
        rv = int(obj["metadata"]["resourceVersion"])
        # stored objects are never mutated after they are stored (every update stores a
        # new dict), so the history can hold them by reference
        k = self._key(res)
        self._history.append((rv, k, typ, obj))
        self._last_rv = rv
        ev = None
        ns = obj["metadata"].get("namespace")
        for w in list(self._watches):
            if w.rkey == k and (w.namespace is None or w.namespace == ns):
                if ev is None:
                    ev = _Event(typ, obj)
                w.push(typ, obj, ev)

    def _drop_watch(self, w: FakeWatch) -> None:
        with self._lock:
            if w in self._watches:
                self._watches.remove(w)

    def current_resource_version(self) -> str:
        with self._lock:
            # the last resourceVersion handed out (deletions included), like etcd's revision
            return str(self._last_rv)

    # ------------------------------------------------------------------ verbs
    def list_rv(self, res: Resource, namespace: str | None = None, label_selector: dict | str | None = None,
                field_selector: str | None = None) -> tuple[list[dict], str]:
        """``list`` plus the list's resourceVersion (the store's current one), atomically."""
        with self._lock:
            return self.list(res, namespace, label_selector, field_selector), self.current_resource_version()

    def get(self, res: Resource, name: str, namespace: str | None = None, *, copy: bool = True) -> dict | None:
        self._log_call("get", res, namespace, name)
        self._fault("get", res)
        with self._lock:
            o = self._objs.get((self._key(res), namespace or "", name))
        # stored objects are immutable: copy unlocked (copy=False: the REST server only encodes it)
        return _jcopy(o) if o is not None and copy else o

    def list(self, res: Resource, namespace: str | None = None, label_selector: dict | str | None = None,
             field_selector: str | None = None, *, copy: bool = True) -> list[dict]:
        self._log_call("list", res, namespace, None)
        self._fault("list", res)
        sel = parse_selector(label_selector) if isinstance(label_selector, str) else label_selector
        key = self._key(res)
        with self._lock:
            out = []
            for (ns, _), o in sorted(self._kind(key).items()):
                if namespace is not None and ns != namespace:
                    continue
                if sel is not None and not match_selector(sel, o["metadata"].get("labels")):
                    continue
                if not match_fields(field_selector, o):
                    continue
                out.append(o)
        return [_jcopy(o) for o in out] if copy else out

    def create(self, res: Resource, obj: dict, namespace: str | None = None, *, copy: bool = True,
               owned: bool = False) -> dict:
        """``owned``: the caller hands ``obj`` over (a freshly decoded request body, the REST
        server) -- it is stored as is instead of deep-copied first."""
        ns = namespace or obj.get("metadata", {}).get("namespace") or ("default" if res.namespaced else "")
        name = obj.get("metadata", {}).get("name")
        self._log_call("create", res, ns, name)
        self._fault("create", res)
        if not name:
            gen = obj.get("metadata", {}).get("generateName")
            if not gen:
                raise ApiError(422, "metadata.name is required", "Invalid")
            name = gen + uuid.uuid4().hex[:5]
        with self._lock:
            k = (self._key(res), ns if res.namespaced else "", name)
            if k in self._objs:
                raise ApiError(409, f"{res.plural} {name} already exists", "AlreadyExists")
            o = obj if owned else _jcopy(obj)
            md = o.setdefault("metadata", {})
            md["name"] = name
            if res.namespaced:
                md["namespace"] = ns
            md["uid"] = str(uuid.uuid4())
            md["resourceVersion"] = str(next(self._rv))
            md["generation"] = 1
            md.setdefault("creationTimestamp", instant_str())
            o.setdefault("apiVersion", res.api_version)
            o.setdefault("kind", res.kind)
            self._store(k, o)
            self._emit(res, "ADDED", o)
        return _jcopy(o) if copy else o

    def _update(self, res: Resource, name: str, namespace: str | None, fn, resource_version: str | None,
                status: bool, copy: bool = True) -> dict:
        with self._lock:
            k = (self._key(res), namespace or "", name)
            cur = self._objs.get(k)
            if cur is None:
                raise ApiError(404, f"{res.plural} {name} not found", "NotFound")
            if resource_version is not None and str(resource_version) != cur["metadata"]["resourceVersion"]:
                raise ApiError(409, f"the object has been modified; resourceVersion {resource_version} is stale",
                               "Conflict")
            if status:
                # only status may change: copy status deeply, share the rest (never mutated)
                base = dict(cur)
                base["metadata"] = dict(cur["metadata"])
                if "status" in cur:
                    base["status"] = _jcopy(cur["status"])
                new = fn(base)
            else:
                new = fn(_jcopy(cur))
            new["metadata"]["uid"] = cur["metadata"]["uid"]
            new["metadata"]["name"] = name
            if res.namespaced:
                new["metadata"]["namespace"] = namespace
            if status:
                # status subresource: only status may change
                kept = dict(cur)
                kept["metadata"] = dict(cur["metadata"])
                kept["status"] = new.get("status")
                if kept["status"] is None:
                    kept.pop("status", None)
                new = kept
            elif new.get("spec") != cur.get("spec"):
                new["metadata"]["generation"] = int(cur["metadata"].get("generation", 1)) + 1
            else:
                new["metadata"]["generation"] = cur["metadata"].get("generation", 1)
            new["metadata"]["resourceVersion"] = str(next(self._rv))
            self._store(k, new)
            self._emit(res, "MODIFIED", new)
        return _jcopy(new) if copy else new

    def patch(self, res: Resource, name: str, namespace: str | None, patch: dict,
              resource_version: str | None = None, *, copy: bool = True) -> dict:
        self._log_call("patch", res, namespace, name)
        self._fault("patch", res)
        rv = resource_version or (patch.get("metadata") or {}).get("resourceVersion")
        return self._update(res, name, namespace, lambda o: merge_patch(o, patch), rv, status=False, copy=copy)

    def replace(self, res: Resource, obj: dict, namespace: str | None = None, *, copy: bool = True) -> dict:
        name = obj["metadata"]["name"]
        ns = namespace or obj["metadata"].get("namespace")
        self._log_call("replace", res, ns, name)
        self._fault("replace", res)
        rv = obj["metadata"].get("resourceVersion")
        return self._update(res, name, ns, lambda o: _jcopy(obj), rv, status=False, copy=copy)

    def patch_status(self, res: Resource, name: str, namespace: str | None, status_patch: dict,
                     resource_version: str | None = None, *, copy: bool = True) -> dict:
        self._log_call("patch_status", res, namespace, name)
        self._fault("patch_status", res)
        return self._update(res, name, namespace, lambda o: merge_patch(o, {"status": status_patch}),
                            resource_version, status=True, copy=copy)

    def replace_status(self, res: Resource, obj: dict, namespace: str | None = None, *, copy: bool = True) -> dict:
        name = obj["metadata"]["name"]
        ns = namespace or obj["metadata"].get("namespace")
        self._log_call("replace_status", res, ns, name)
        self._fault("patch_status", res)
        rv = obj["metadata"].get("resourceVersion")

        def fn(o):
            o["status"] = _jcopy(obj.get("status"))
            return o

        return self._update(res, name, ns, fn, rv, status=True, copy=copy)

    def delete(self, res: Resource, name: str, namespace: str | None = None) -> bool:
        self._log_call("delete", res, namespace, name)
        self._fault("delete", res)
        with self._lock:
            k = (self._key(res), namespace or "", name)
            o = self._objs.pop(k, None)
            if o is None:
                return False
            self._kind(k[0]).pop(k[1:], None)
            o = dict(o)
            o["metadata"] = dict(o["metadata"])
            o["metadata"]["resourceVersion"] = str(next(self._rv))
            self._emit(res, "DELETED", o)
            return True

    def watch(self, res: Resource, namespace: str | None = None, resource_version: str | None = None,
              sink=None) -> FakeWatch:
        self._log_call("watch", res, namespace, None)
        self._fault("watch", res)
        with self._lock:
            w = FakeWatch(self, res, namespace, sink)
            if resource_version and int(resource_version) < self._compacted:
                w.fail(f"too old resource version: {resource_version} ({self._compacted})", 410)
                return w
            if resource_version:
                key = self._key(res)
                for rv, k, typ, o in self._history:
                    if k == key and rv > int(resource_version) and \
                            (namespace is None or o["metadata"].get("namespace") == namespace):
                        w.push(typ, o)
            self._watches.append(w)
            return w

    def fail_watches(self, message: str = "injected watch failure", res: Resource | None = None) -> int:
        """Close every open watch (optionally of one resource) with an error."""
        with self._lock:
            ws = [w for w in self._watches if res is None or w.res == res]
        for w in ws:
            w.fail(message)
        return len(ws)

    def end_watches(self, res: Resource | None = None) -> int:
        """End every open watch cleanly from the server side (no ERROR event), as a
        real apiserver does when a watch reaches its timeout (30-60 min)."""
        with self._lock:
            ws = [w for w in self._watches if res is None or w.res == res]
        for w in ws:
            w.close()
        return len(ws)

    def bookmark(self, res: Resource | None = None) -> int:
        """Send a BOOKMARK (current resourceVersion only) to every open watch."""
        with self._lock:
            rv = self.current_resource_version()
            ws = [w for w in self._watches if res is None or w.res == res]
        for w in ws:
            w.push("BOOKMARK", {"apiVersion": w.res.api_version, "kind": w.res.kind,
                                "metadata": {"resourceVersion": rv}})
        return len(ws)

    def compact(self, resource_version: str | int | None = None) -> int:
        """Forget the event history up to ``resource_version`` (default: everything so far);
        later watches from an older resourceVersion fail with 410 Gone."""
        with self._lock:
            upto = int(resource_version) if resource_version is not None else int(self.current_resource_version())
            self._history = [h for h in self._history if h[0] > upto]
            self._compacted = max(self._compacted, upto)
            return self._compacted

    def open_watches(self, res: Resource | None = None) -> int:
        with self._lock:
            return sum(1 for w in self._watches if res is None or w.res == res)

    # ------------------------------------------------------------------ pods/log
    def set_log(self, namespace: str, pod: str, text: str | bytes, container: str | None = None) -> None:
        if isinstance(text, bytes):
            text = text.decode("utf-8", "replace")
        with self._lock:
            self._logs[(namespace, pod, container)] = text

    def pod_log(self, name: str, namespace: str, container: str | None = None, previous: bool = False,
                tail_lines: int | None = None, limit_bytes: int | None = None) -> str:
        self._log_call("log", PODS, namespace, name)
        self._fault("log", PODS)
        with self._lock:
            if (self._key(PODS), namespace, name) not in self._objs:
                raise ApiError(404, f"pod {name} not found", "NotFound")
            text = self._logs.get((namespace, name, container))
            if text is None:
                text = self._logs.get((namespace, name, None), "")
        if tail_lines is not None:
            text = "\n".join(text.split("\n")[-tail_lines:])
        if limit_bytes is not None:
            text = text.encode()[:limit_bytes].decode("utf-8", "ignore")
        return text

    # ------------------------------------------------------------------ conveniences for tests
    def objects(self, res: Resource) -> list[dict]:
        return self.list(res)

    def reset_calls(self) -> None:
        self.calls.clear()


def failed_pod(name: str, namespace: str = "default", labels: dict | None = None, exit_code: int = 1,
               finished_at: str | None = None, reason: str = "Error", owner_rs: str | None = None) -> dict:
    """A pod whose single container terminated with ``exit_code``."""
    md: dict[str, Any] = {"name": name, "namespace": namespace, "labels": labels or {}}
    if owner_rs:
        md["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": owner_rs,
                                  "uid": str(uuid.uuid4()), "controller": True}]
    return {
        "apiVersion": "v1", "kind": "Pod", "metadata": md,
        "spec": {"containers": [{"name": "app", "image": "registry.example/app:1.0"}]},
        "status": {"phase": "Running", "containerStatuses": [{
            "name": "app", "ready": False, "restartCount": 1,
            "state": {"terminated": {"exitCode": exit_code, "reason": reason,
                                     "finishedAt": finished_at or instant_str().split(".")[0] + "Z"}}}]},
    }


def running_pod(name: str, namespace: str = "default", labels: dict | None = None) -> dict:
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": name, "namespace": namespace, "labels": labels or {}},
            "spec": {"containers": [{"name": "app", "image": "registry.example/app:1.0"}]},
            "status": {"phase": "Running", "containerStatuses": [{"name": "app", "ready": True,
                                                                  "state": {"running": {"startedAt": instant_str()}}}]}}


__all__ = ["FakeKube", "FakeWatch", "merge_patch", "failed_pod", "running_pod", "ALL"]
