"""Resumable list/watch loop: the one piece of informer machinery shared by the
pod-failure watcher, the Podmortem cache and the controller runtime.

fabric8 (the reference's client, J/service/PodFailureWatcher.java:102-137)
reconnects a watch the apiserver ends on its own and only reports ``onClose``
for errors; here every consumer gets the same contract from one loop:

* resume from the last resourceVersion seen — object events AND ``BOOKMARK``
  events (requested with ``allowWatchBookmarks``) advance it, so a quiet
  resource does not keep a resourceVersion that compaction will expire;
* a stream the server ends cleanly (the apiserver's min-request-timeout closes
  every watch after 30-60 min) is reopened at once from that resourceVersion —
  only ``stop()`` ends the loop;
* a watch that fails with **410 Gone / Expired** (the resourceVersion was
  compacted away) is never retried with the same resourceVersion: the loop
  relists, takes the LIST's own ``metadata.resourceVersion`` (an opaque string,
  never the maximum of the items') and hands the listed objects to ``relist``
  so the consumer can catch up on what it missed;
* other errors restart after ``restart_delay_s`` (5 s, PodFailureWatcher.java:574)
  with doubling backoff up to ``max_delay_s``.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Callable

from .resources import ApiError, Resource, WatchClosed

log = logging.getLogger(__name__)


def list_with_rv(kube, res: Resource, namespace: str | None = None) -> tuple[list[dict], str | None]:
    """(items, list resourceVersion); clients without ``list_rv`` give no resourceVersion."""
    fn = getattr(kube, "list_rv", None)
    if fn is not None:
        return fn(res, namespace)
    return kube.list(res, namespace), None


class WatchLoop:
    def __init__(self, kube, res: Resource, namespace: str | None, on_event: Callable[[str, dict], None],
                 relist: Callable[[list[dict]], None] | None = None, name: str = "",
                 restart_delay_s: float = 5.0, max_delay_s: float = 60.0, stop: threading.Event | None = None):
        self.kube, self.res, self.namespace = kube, res, namespace
        self.on_event, self.relist = on_event, relist
        self.name = name or f"{res.plural}-watch"
        self.restart_delay_s, self.max_delay_s = restart_delay_s, max_delay_s
        self.stop_event = stop or threading.Event()
        self.rv: str | None = None
        self._need_relist = False
        self._lock = threading.Lock()
        self._open: list = []
        self.restarts = 0        # reopen after an error
        self.reconnects = 0      # reopen after a clean server-side end
        self.relists = 0         # relist after 410 Gone

    # ------------------------------------------------------------------ pieces
    def list_now(self) -> list[dict]:
        """LIST and adopt the list's resourceVersion as the resume point."""
        items, rv = list_with_rv(self.kube, self.res, self.namespace)
        self.rv = rv
        self._need_relist = False
        return items

    def open(self):
        w = self.kube.watch(self.res, self.namespace, resource_version=self.rv)
        with self._lock:
            self._open.append(w)
        return w

    def _forget(self, w) -> None:
        with self._lock:
            if w in self._open:
                self._open.remove(w)

    def _do_relist(self) -> None:
        items = self.list_now()
        self.relists += 1
        if self.relist is not None:
            self.relist(items)

    def stop(self) -> None:
        self.stop_event.set()
        with self._lock:
            ws = list(self._open)
        for w in ws:
            try:
                w.close()
            except Exception:  # noqa: BLE001
                pass

    # ------------------------------------------------------------------ loop
    def run(self, first=None) -> None:
        delay = self.restart_delay_s
        stop = self.stop_event
        while not stop.is_set():
            w, first = first, None
            events, t0 = 0, time.monotonic()
            failed = False
            try:
                if w is None:
                    if self._need_relist:
                        self._do_relist()
                    w = self.open()
                for typ, obj in w:
                    rv = (obj.get("metadata") or {}).get("resourceVersion")
                    if rv:
                        self.rv = rv
                    if typ == "BOOKMARK":
                        continue
                    events += 1
                    delay = self.restart_delay_s
                    self.on_event(typ, obj)
                if stop.is_set():
                    return
                # clean end from the server: reopen from self.rv (no event is lost)
                self.reconnects += 1
                log.info("%s: watch stream ended; reconnecting from resourceVersion %s", self.name, self.rv)
                if events == 0 and time.monotonic() - t0 < 1.0 and stop.wait(1.0):   # no hot loop
                    return
                continue
            except WatchClosed as e:
                if stop.is_set():
                    return
                if e.expired:
                    log.warning("%s: resourceVersion %s expired (410 Gone); relisting", self.name, self.rv)
                    self.rv, self._need_relist = None, True
                else:
                    log.error("%s: watch closed due to error: %s", self.name, e)
                    failed = True
            except (ApiError, OSError) as e:
                if stop.is_set():
                    return
                if getattr(e, "code", None) == 410:
                    log.warning("%s: resourceVersion %s expired (410 Gone); relisting", self.name, self.rv)
                    self.rv, self._need_relist = None, True
                else:
                    log.error("%s: watch failed: %s", self.name, e)
                    failed = True
            except Exception as e:  # noqa: BLE001 - a consumer bug must not kill the loop
                log.exception("%s: watch handler failure: %s", self.name, e)
                failed = True
            finally:
                if w is not None:
                    self._forget(w)
            if failed:
                if stop.wait(delay):
                    return
                self.restarts += 1
                log.info("%s: restarting watch", self.name)
                delay = min(delay * 2, self.max_delay_s)
            elif stop.is_set():
                return
