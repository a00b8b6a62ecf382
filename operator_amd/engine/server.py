"""Wire-compatible REST front for the on-node engines.

Serves the two contracts the reference operator calls, so an
unmodified podmortem operator (or any other client) can point its
``quarkus.rest-client.{log-parser,ai-interface}.url`` at this process:

  POST /parse                      PodFailureData  -> AnalysisResult   (LogParserRestClient.java:37-39)
  POST /api/v1/analysis/analyze    AnalysisRequest -> AIResponse       (AIInterfaceRestClient.java:37-39)
  GET  /q/health/live | /q/health/ready | /metrics

Requests are handed to the batching services (LocalMatchService /
LocalExplainService), so concurrent HTTP callers share GPU batches.
"""
from __future__ import annotations

import json
import logging
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from operator_amd.api.models import AnalysisRequest, PodFailureData

log = logging.getLogger(__name__)


class CompatServer:
    def __init__(self, matcher, explainer, host: str = "0.0.0.0", port: int = 8080, metrics=None):
        self.matcher, self.explainer, self.metrics = matcher, explainer, metrics
        srv = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, code: int, obj, ctype: str = "application/json") -> None:
                b = obj if isinstance(obj, bytes) else json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def do_GET(self):  # noqa: N802
                if self.path.startswith("/q/health"):
                    return self._send(200, {"status": "UP", "checks": []})
                if self.path.startswith("/metrics") and srv.metrics is not None:
                    return self._send(200, srv.metrics.render(), "text/plain; version=0.0.4")
                self._send(404, {"error": "not found"})

            def do_POST(self):  # noqa: N802
                n = int(self.headers.get("Content-Length", "0") or 0)
                try:
                    body = json.loads(self.rfile.read(n) or b"{}")
                    if self.path.rstrip("/") == "/parse":
                        if srv.matcher is None:
                            return self._send(503, {"error": "pattern engine not configured"})
                        res = srv.matcher.analyze(PodFailureData.model_validate(body))
                        return self._send(200, res.to_obj())
                    if self.path.rstrip("/") == "/api/v1/analysis/analyze":
                        if srv.explainer is None:
                            return self._send(503, {"error": "explanation engine not configured"})
                        req = AnalysisRequest.model_validate(body)
                        resp = srv.explainer.explain(req.analysis_result, req.provider_config)
                        return self._send(200, resp.to_obj())
                    return self._send(404, {"error": "not found"})
                except Exception as e:  # noqa: BLE001
                    log.error("request %s failed: %s", self.path, e)
                    return self._send(500, {"error": str(e)})

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self._t = threading.Thread(target=self.httpd.serve_forever, name="compat-http", daemon=True)

    def start(self) -> "CompatServer":
        self._t.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
