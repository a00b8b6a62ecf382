"""Serve a FakeKube over the Kubernetes REST paths (HTTP), so the real
KubeClient is exercised end-to-end without a cluster (tests, local demos).

Supported: GET/LIST (label & field selectors), POST, PUT, PATCH
(merge-patch, with metadata.resourceVersion -> 409), DELETE, the ``status``
subresource, ``pods/{name}/log``, and ``?watch=1`` streaming. One extension a
real apiserver does not have: ``PUT pods/{name}/log`` sets a pod's log text (what
the container would have written), so a test or benchmark in another process can
seed logs.

Run standalone (the one API server several operator shard processes share, e.g.
``bench.py --gpus N``): ``python -m operator_amd.kube.fake_server --port 0
--port-file F`` writes its URL to F once it is listening. Each watch event is
serialised once and the same bytes go to every watcher.
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
            # one buffered write per response and TCP_NODELAY: unbuffered header lines under
            # Nagle + the client's delayed ACK cost ~40 ms per keep-alive request
            disable_nagle_algorithm = True
            wbufsize = 1 << 16

            def log_message(self, *a):
                pass

            def _json(self, code: int, obj) -> None:
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)
                self.wfile.flush()

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
                    if method == "PUT" and sub == "log":
                        n = int(self.headers.get("Content-Length", "0") or 0)
                        srv.fk.set_log(ns or "default", name, self.rfile.read(n), q.get("container"))
                        return self._json(200, {"kind": "Status", "status": "Success"})
                    if method == "GET" and sub == "log":
                        text = srv.fk.pod_log(name, ns, q.get("container"), q.get("previous") == "true",
                                              int(q["tailLines"]) if "tailLines" in q else None,
                                              int(q["limitBytes"]) if "limitBytes" in q else None).encode()
                        self.send_response(200)
                        self.send_header("Content-Type", "text/plain")
                        self.send_header("Content-Length", str(len(text)))
                        self.end_headers()
                        self.wfile.write(text)
                        self.wfile.flush()
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
                self.wfile.flush()

                def chunk(b: bytes) -> None:
                    self.wfile.write(f"{len(b):x}\r\n".encode() + b + b"\r\n")
                    self.wfile.flush()

                try:
                    while True:
                        try:
                            ev = w.next_event()
                        except StopIteration:
                            break
                        chunk(ev.wire())
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
                    self.wfile.flush()
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

        class Server(ThreadingHTTPServer):
            def handle_error(self, request, client_address):   # a client gone mid-stream is not an error
                import sys

                if not isinstance(sys.exc_info()[1], (BrokenPipeError, ConnectionResetError)):
                    super().handle_error(request, client_address)

        self.httpd = Server((host, port), H)
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


def main(argv: list[str] | None = None) -> int:
    """A standalone FakeKube API server process (until SIGTERM / SIGINT)."""
    import argparse
    import os
    import signal

    ap = argparse.ArgumentParser(description="in-memory Kubernetes API server (test double)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--port-file", default=None, help="write the URL here once listening")
    a = ap.parse_args(argv)
    if hasattr(os, "getppid"):   # exit with the process that started it
        try:
            import ctypes

            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))   # PR_SET_PDEATHSIG
        except OSError:
            pass
    srv = FakeKubeServer(FakeKube(record_calls=False), a.host, a.port).start()
    if a.port_file:
        tmp = a.port_file + ".tmp"
        with open(tmp, "w") as f:
            f.write(srv.url)
        os.replace(tmp, a.port_file)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    srv.stop()
    return 0


def write_kubeconfig(url: str, path: str, namespace: str = "default") -> str:
    """A kubeconfig (no credentials) for the API server at ``url``: what ``run`` /
    ``KubeClient.auto`` read to reach a FakeKubeServer from another process."""
    import yaml

    doc = {"apiVersion": "v1", "kind": "Config", "current-context": "fake",
           "clusters": [{"name": "fake", "cluster": {"server": url}}],
           "users": [{"name": "fake", "user": {}}],
           "contexts": [{"name": "fake", "context": {"cluster": "fake", "user": "fake", "namespace": namespace}}]}
    with open(path, "w") as f:
        yaml.safe_dump(doc, f)
    return path


def spawn(port_file: str, timeout_s: float = 60.0):
    """Start ``main`` as a child process; returns (process, url) once it listens."""
    import os
    import subprocess
    import sys
    import time

    if os.path.exists(port_file):
        os.unlink(port_file)
    p = subprocess.Popen([sys.executable, "-m", "operator_amd.kube.fake_server", "--port-file", port_file])
    t0 = time.monotonic()
    while not os.path.exists(port_file):
        if p.poll() is not None or time.monotonic() - t0 > timeout_s:
            p.kill()
            raise RuntimeError(f"fake API server did not start (exit {p.poll()})")
        time.sleep(0.05)
    with open(port_file) as f:
        return p, f.read().strip()


if __name__ == "__main__":
    raise SystemExit(main())
