"""Serve a FakeKube over the Kubernetes REST paths (HTTP), so the real
KubeClient is exercised end-to-end without a cluster (tests, local demos).

Supported: GET/LIST (label & field selectors), POST, PUT, PATCH
(merge-patch, with metadata.resourceVersion -> 409), DELETE, the ``status``
subresource, ``pods/{name}/log``, and ``?watch=1`` streaming.
"""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

from .fake import FakeKube
from .resources import ALL, ApiError, Resource, WatchClosed


def _route(path: str) -> tuple[Resource, str | None, str | None, str | None] | None:
    parts = [p for p in path.split("/") if p]
    if not parts:
        return None
    if parts[0] == "api":
        group, version, rest = "", parts[1], parts[2:]
    elif parts[0] == "apis":
        group, version, rest = parts[1], parts[2], parts[3:]
    else:
        return None
    ns = None
    if len(rest) >= 2 and rest[0] == "namespaces" and len(rest) > 2:
        ns, rest = rest[1], rest[2:]
    plural, name, sub = rest[0], (rest[1] if len(rest) > 1 else None), (rest[2] if len(rest) > 2 else None)
    for r in ALL:
        if r.group == group and r.version == version and r.plural == plural:
            return r, ns, name, sub
    return None


class FakeKubeServer:
    def __init__(self, fk: FakeKube, host: str = "127.0.0.1", port: int = 0):
        self.fk = fk
        srv = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _json(self, code: int, obj) -> None:
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def _err(self, e: ApiError) -> None:
                self._json(e.code, {"kind": "Status", "code": e.code, "reason": e.reason, "message": e.message})

            def _body(self) -> dict:
                n = int(self.headers.get("Content-Length", "0") or 0)
                return json.loads(self.rfile.read(n) or b"{}")

            def _dispatch(self, method: str) -> None:
                u = urlparse(self.path)
                q = {k: v[0] for k, v in parse_qs(u.query).items()}
                rt = _route(u.path)
                if rt is None:
                    return self._json(404, {"message": "not found", "reason": "NotFound", "code": 404})
                res, ns, name, sub = rt
                try:
                    if method == "GET" and sub == "log":
                        text = srv.fk.pod_log(name, ns, q.get("container"), q.get("previous") == "true",
                                              int(q["tailLines"]) if "tailLines" in q else None,
                                              int(q["limitBytes"]) if "limitBytes" in q else None).encode()
                        self.send_response(200)
                        self.send_header("Content-Type", "text/plain")
                        self.send_header("Content-Length", str(len(text)))
                        self.end_headers()
                        self.wfile.write(text)
                        return
                    if method == "GET" and name is None and q.get("watch") in ("1", "true"):
                        return self._watch(res, ns, q.get("resourceVersion"))
                    if method == "GET" and name is None:
                        items = srv.fk.list(res, ns, q.get("labelSelector"), q.get("fieldSelector"))
                        return self._json(200, {"kind": res.kind + "List", "apiVersion": res.api_version,
                                                "metadata": {"resourceVersion": srv.fk.current_resource_version()},
                                                "items": items})
                    if method == "GET":
                        o = srv.fk.get(res, name, ns)
                        if o is None:
                            raise ApiError(404, f"{res.plural} {name} not found", "NotFound")
                        return self._json(200, o)
                    if method == "POST":
                        return self._json(201, srv.fk.create(res, self._body(), ns))
                    if method == "PUT":
                        body = self._body()
                        if sub == "status":
                            return self._json(200, srv.fk.replace_status(res, body, ns))
                        return self._json(200, srv.fk.replace(res, body, ns))
                    if method == "PATCH":
                        body = self._body()
                        rv = (body.get("metadata") or {}).get("resourceVersion")
                        if sub == "status":
                            return self._json(200, srv.fk.patch_status(res, name, ns, body.get("status") or {}, rv))
                        return self._json(200, srv.fk.patch(res, name, ns, body, rv))
                    if method == "DELETE":
                        if not srv.fk.delete(res, name, ns):
                            raise ApiError(404, f"{res.plural} {name} not found", "NotFound")
                        return self._json(200, {"kind": "Status", "status": "Success"})
                except ApiError as e:
                    return self._err(e)
                self._json(405, {"message": "method not allowed", "code": 405})

            def _watch(self, res, ns, rv) -> None:
                w = srv.fk.watch(res, ns, rv)
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Transfer-Encoding", "chunked")
                self.end_headers()

                def chunk(b: bytes) -> None:
                    self.wfile.write(f"{len(b):x}\r\n".encode() + b + b"\r\n")
                    self.wfile.flush()

                try:
                    for typ, obj in w:
                        chunk(json.dumps({"type": typ, "object": obj}).encode() + b"\n")
                except WatchClosed as e:
                    try:
                        chunk(json.dumps({"type": "ERROR", "object": {"code": e.code or 500, "message": str(e),
                                                                      "reason": "Expired" if e.code == 410 else "Error"}}
                                         ).encode() + b"\n")
                    except OSError:
                        pass
                except OSError:
                    w.close()
                    return
                try:
                    self.wfile.write(b"0\r\n\r\n")
                except OSError:
                    pass

            def do_GET(self):  # noqa: N802
                self._dispatch("GET")

            def do_POST(self):  # noqa: N802
                self._dispatch("POST")

            def do_PUT(self):  # noqa: N802
                self._dispatch("PUT")

            def do_PATCH(self):  # noqa: N802
                self._dispatch("PATCH")

            def do_DELETE(self):  # noqa: N802
                self._dispatch("DELETE")

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.url = f"http://{host}:{self.httpd.server_address[1]}"
        self._t = threading.Thread(target=self.httpd.serve_forever, name="fakekube-http", daemon=True)

    def start(self) -> "FakeKubeServer":
        self._t.start()
        return self

    def stop(self) -> None:
        self.fk.fail_watches("server shutdown")
        self.httpd.shutdown()
        self.httpd.server_close()
