"""Health + metrics HTTP endpoints.

Readiness check ``pattern-library-sync`` (J/health/PatternLibraryReadinessCheck.java:33-85):
UP if no PatternLibrary CRs exist; else UP if the pattern cache holds >= 1
*.yaml/*.yml file; else DOWN until ``grace_s`` (5 min) after startup, then UP;
any error -> DOWN. Served at the paths the reference's Deployment probes
(K/operator-deployment.yaml:61-78): ``/q/health/live`` and ``/q/health/ready``
(SmallRye Health JSON), plus ``/q/health`` and Prometheus ``/metrics``.
Additional readiness check ``analysis-engine``: the on-node GPU engines loaded.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path
from typing import Callable

from operator_amd.kube.resources import PATTERNLIBRARIES

from .sync import yaml_files

log = logging.getLogger(__name__)


class PatternLibraryReadiness:
    NAME = "pattern-library-sync"

    def __init__(self, kube, cache_dir: str, grace_s: float = 300.0, clock=time.monotonic):
        self.kube, self.cache_dir, self.grace_s, self.clock = kube, Path(cache_dir), grace_s, clock
        self.startup = clock()

    def __call__(self) -> tuple[str, bool]:
        try:
            if not self.kube.list(PATTERNLIBRARIES):
                return self.NAME, True
            past_grace = self.clock() - self.startup > self.grace_s
            if not self.cache_dir.exists():
                if past_grace:
                    log.warning("Pattern library sync grace period exceeded (no cache dir), reporting ready anyway")
                return self.NAME, past_grace
            if yaml_files(self.cache_dir):
                return self.NAME, True
            if past_grace:
                log.warning("Pattern library sync grace period exceeded (no patterns found), reporting ready anyway")
            return self.NAME, past_grace
        except Exception as e:  # noqa: BLE001
            log.error("Error during pattern library readiness check: %s", e)
            return self.NAME, False


def health_body(checks: list[tuple[str, bool]]) -> tuple[int, dict]:
    up = all(ok for _, ok in checks)
    body = {"status": "UP" if up else "DOWN",
            "checks": [{"name": n, "status": "UP" if ok else "DOWN"} for n, ok in checks]}
    return (200 if up else 503), body


class HealthServer:
    def __init__(self, host: str, port: int, readiness: list[Callable[[], tuple[str, bool]]],
                 liveness: list[Callable[[], tuple[str, bool]]] | None = None, metrics=None):
        self.readiness, self.liveness, self.metrics = readiness, liveness or [], metrics
        srv = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def _send(self, code: int, body: bytes, ctype: str) -> None:
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):  # noqa: N802
                path = self.path.split("?")[0]
                if path == "/metrics" and srv.metrics is not None:
                    return self._send(200, srv.metrics.render(), "text/plain; version=0.0.4")
                if path in ("/q/health/live", "/q/health/ready", "/q/health"):
                    checks = []
                    if path in ("/q/health/live", "/q/health"):
                        checks += [c() for c in srv.liveness]
                    if path in ("/q/health/ready", "/q/health"):
                        checks += [c() for c in srv.readiness]
                    code, body = health_body(checks)
                    return self._send(code, json.dumps(body).encode(), "application/json")
                self._send(404, b'{"error":"not found"}', "application/json")

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.port = self.httpd.server_address[1]
        self._t: threading.Thread | None = None

    def start(self) -> None:
        self._t = threading.Thread(target=self.httpd.serve_forever, name="health-http", daemon=True)
        self._t.start()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
