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
import socketserver
import threading
from urllib.parse import parse_qsl

from .fake import FakeKube
from .resources import ALL, ApiError, Resource, WatchClosed


_BY_PATH = {(r.group, r.version, r.plural): r for r in ALL}


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
    if not rest:
        return None
    plural, name, sub = rest[0], (rest[1] if len(rest) > 1 else None), (rest[2] if len(rest) > 2 else None)
    r = _BY_PATH.get((group, version, plural))
    return None if r is None else (r, ns, name, sub)


_REASONS = {200: b"OK", 201: b"Created", 400: b"Bad Request", 403: b"Forbidden", 404: b"Not Found",
            405: b"Method Not Allowed", 409: b"Conflict", 410: b"Gone", 422: b"Unprocessable Entity",
            500: b"Internal Server Error"}


class _Conn(socketserver.StreamRequestHandler):
    """One keep-alive HTTP/1.1 connection, parsed by hand: request line, headers up to the
    blank line, a Content-Length body. http.server's handler parses every header block
    with the email package, which made the fake API server the bottleneck of an 8-shard
    run (~3.6k requests/s); a response is one buffered write (TCP_NODELAY: a header line
    per segment under Nagle + delayed ACK cost ~40 ms per request)."""
    disable_nagle_algorithm = True
    wbufsize = 1 << 16
    server: "_Server"

    def handle(self) -> None:
        rf = self.rfile
        while True:
            line = rf.readline(65537)
            if not line:
                return
            if line in (b"\r\n", b"\n"):
                continue
            try:
                method, target, _ = line.split(b" ", 2)
            except ValueError:
                return
            hdrs = {}
            while True:
                h = rf.readline(65537)
                if h in (b"\r\n", b"\n", b""):
                    break
                k, _, v = h.partition(b":")
                hdrs[k.strip().lower()] = v.strip()
            n = int(hdrs.get(b"content-length", b"0") or 0)
            body = rf.read(n) if n else b""
            self.server.app.dispatch(self, method.decode(), target.decode(), body)
            if hdrs.get(b"connection", b"").lower() == b"close":
                return

    def respond(self, code: int, body: bytes, ctype: bytes = b"application/json") -> None:
        self.wfile.write(b"HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %d\r\n\r\n"
                         % (code, _REASONS.get(code, b"Status"), ctype, len(body)) + body)
        self.wfile.flush()

    def json(self, code: int, obj) -> None:
        self.respond(code, json.dumps(obj, separators=(",", ":")).encode())


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True
    # listen backlog: eight operator shards' worker pools plus bursts of failing pods connect
    # at once (the socketserver default of 5 resets connections under that load)
    request_queue_size = 1024

    def handle_error(self, request, client_address):   # a client gone mid-stream is not an error
        import sys

        if not isinstance(sys.exc_info()[1], (BrokenPipeError, ConnectionResetError)):
            super().handle_error(request, client_address)


class FakeKubeServer:
    def __init__(self, fk: FakeKube, host: str = "127.0.0.1", port: int = 0):
        self.fk = fk
        self.httpd = _Server((host, port), _Conn)
        self.httpd.app = self
        self.url = f"http://{host}:{self.httpd.server_address[1]}"
        self._t = threading.Thread(target=self.httpd.serve_forever, name="fakekube-http", daemon=True)

    def dispatch(self, c: _Conn, method: str, target: str, raw: bytes) -> None:
        w = self.route(c, method, target, raw)
        if w is not None:
            self._watch(c, *w)

    def route(self, c, method: str, target: str, raw: bytes):
        """Serve one unary request into ``c`` (``respond`` / ``json``); a watch request
        is returned as (resource, namespace, resourceVersion) for the caller to stream."""
        fk = self.fk
        path, _, query = target.partition("?")
        q = {}
        if query:
            for k, v in parse_qsl(query.partition("#")[0]):
                q.setdefault(k, v)   # the first value of a repeated key, as parse_qs()[k][0]
        rt = _route(path.partition("#")[0])
        if rt is None:
            return c.json(404, {"message": "not found", "reason": "NotFound", "code": 404})
        res, ns, name, sub = rt
        body = lambda: json.loads(raw or b"{}")  # noqa: E731
        try:
            if method == "PUT" and sub == "log":
                fk.set_log(ns or "default", name, raw, q.get("container"))
                return c.json(200, {"kind": "Status", "status": "Success"})
            if method == "GET" and sub == "log":
                text = fk.pod_log(name, ns, q.get("container"), q.get("previous") == "true",
                                  int(q["tailLines"]) if "tailLines" in q else None,
                                  int(q["limitBytes"]) if "limitBytes" in q else None).encode()
                return c.respond(200, text, b"text/plain")
            if method == "GET" and name is None and q.get("watch") in ("1", "true"):
                return res, ns, q.get("resourceVersion")
            if method == "GET" and name is None:
                items = fk.list(res, ns, q.get("labelSelector"), q.get("fieldSelector"), copy=False)
                return c.json(200, {"kind": res.kind + "List", "apiVersion": res.api_version,
                                    "metadata": {"resourceVersion": fk.current_resource_version()},
                                    "items": items})
            if method == "GET":
                o = fk.get(res, name, ns, copy=False)
                if o is None:
                    raise ApiError(404, f"{res.plural} {name} not found", "NotFound")
                return c.json(200, o)
            if method == "POST":
                return c.json(201, fk.create(res, body(), ns, copy=False, owned=True))
            if method == "PUT":
                if sub == "status":
                    return c.json(200, fk.replace_status(res, body(), ns, copy=False))
                return c.json(200, fk.replace(res, body(), ns, copy=False))
            if method == "PATCH":
                b = body()
                rv = (b.get("metadata") or {}).get("resourceVersion")
                if sub == "status":
                    return c.json(200, fk.patch_status(res, name, ns, b.get("status") or {}, rv, copy=False))
                return c.json(200, fk.patch(res, name, ns, b, rv, copy=False))
            if method == "DELETE":
                if not fk.delete(res, name, ns):
                    raise ApiError(404, f"{res.plural} {name} not found", "NotFound")
                return c.json(200, {"kind": "Status", "status": "Success"})
        except ApiError as e:
            return c.json(e.code, {"kind": "Status", "code": e.code, "reason": e.reason, "message": e.message})
        c.json(405, {"message": "method not allowed", "code": 405})

    def _watch(self, c: _Conn, res, ns, rv) -> None:
        w = self.fk.watch(res, ns, rv)
        wf = c.wfile
        wf.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n")
        wf.flush()

        def chunk(b: bytes) -> None:
            wf.write(b"%x\r\n%s\r\n" % (len(b), b))
            wf.flush()

        try:
            while True:
                try:
                    evs = w.next_events()
                except StopIteration:
                    break
                # every event already queued goes out in one write + flush (under load one
                # wake-up and one syscall per burst instead of per event)
                wf.write(b"".join(b"%x\r\n%s\r\n" % (len(b), b) for b in (ev.wire() for ev in evs)))
                wf.flush()
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
            wf.write(b"0\r\n\r\n")
            wf.flush()
        except OSError:
            pass

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
    ap.add_argument("--threaded", action="store_true", help="one thread per connection (the in-process server)")
    a = ap.parse_args(argv)
    try:   # exit with the process that started it
        import ctypes

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))   # PR_SET_PDEATHSIG
    except OSError:
        pass
    if a.threaded:
        srv = FakeKubeServer(FakeKube(record_calls=False), a.host, a.port).start()
    else:
        from .fake_aserver import AsyncFakeKubeServer

        srv = AsyncFakeKubeServer(FakeKube(record_calls=False), a.host, a.port).start()
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
