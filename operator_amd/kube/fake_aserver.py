"""The FakeKube REST server on one asyncio event loop (the standalone API server that
several operator shard processes share: ``python -m operator_amd.kube.fake_server``).

Same routes and wire format as the threaded ``FakeKubeServer`` (it reuses its request
routing); the difference is the process model. The threaded server runs one thread per
keep-alive connection — with eight operator shards that is ~500 threads taking turns on
one GIL, and a pod update wakes eight watch threads. Here one thread parses every
request, runs the (non-blocking) store operation and writes the response, and a watch is
a coroutine fed by the store's event fan-out: no thread switches, one write per burst of
queued events. An 8-shard plumbing run is bound by this process (tools/bench_plumbing.py).
"""
from __future__ import annotations

import asyncio
import os
import json
import threading

from .fake import FakeKube, FakeWatch
from .fake_server import _REASONS, FakeKubeServer
from .resources import WatchClosed


class _Sink:
    """Collects one response (the ``respond`` / ``json`` interface ``FakeKubeServer.route`` writes to)."""
    __slots__ = ("out",)

    def __init__(self):
        self.out = b""

    def respond(self, code: int, body: bytes, ctype: bytes = b"application/json") -> None:
        self.out = (b"HTTP/1.1 %d %s\r\nContent-Type: %s\r\nContent-Length: %d\r\n\r\n"
                    % (code, _REASONS.get(code, b"Status"), ctype, len(body)) + body)

    def json(self, code: int, obj) -> None:
        self.respond(code, _ENC.encode(obj).encode())


# one encoder for every response (json.dumps with arguments builds a new one per call)
_ENC = json.JSONEncoder(separators=(",", ":"), check_circular=False)


def _chunk(b: bytes) -> bytes:
    return b"%x\r\n%s\r\n" % (len(b), b)


class AsyncFakeKubeServer:
    def __init__(self, fk: FakeKube, host: str = "127.0.0.1", port: int = 0):
        self.fk = fk
        self._router = FakeKubeServer.__new__(FakeKubeServer)   # routing only, no sockets
        self._router.fk = fk
        self.loop = asyncio.new_event_loop()
        self._server = self.loop.run_until_complete(
            asyncio.start_server(self._client, host, port, backlog=1024, limit=1 << 20))
        self.url = f"http://{host}:{self._server.sockets[0].getsockname()[1]}"
        self._t = threading.Thread(target=self._run, name="fakekube-aio", daemon=True)

    def _run(self) -> None:
        prof_path = os.environ.get("OAMD_APISERVER_PROFILE")   # cProfile of the serving loop (tools)
        if not prof_path:
            self.loop.run_forever()
            return
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
        try:
            self.loop.run_forever()
        finally:
            prof.disable()
            prof.dump_stats(prof_path)

    def start(self) -> "AsyncFakeKubeServer":
        self._t.start()
        return self

    def stop(self) -> None:
        async def _shutdown():   # end every connection coroutine before the loop stops
            self._server.close()
            tasks = [t for t in asyncio.all_tasks() if t is not asyncio.current_task()]
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)

        if self._t.is_alive():
            try:
                asyncio.run_coroutine_threadsafe(_shutdown(), self.loop).result(timeout=5)
            except Exception:  # noqa: BLE001 - stopping anyway
                pass
            self.loop.call_soon_threadsafe(self.loop.stop)
            self._t.join(timeout=5)
        if not self._t.is_alive():
            self.loop.close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------------ connections
    async def _client(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            while True:
                # the request line and every header in one read (a readline per header line
                # was ~8 coroutine round trips per request)
                try:
                    head = await reader.readuntil(b"\r\n\r\n")
                except asyncio.IncompleteReadError:   # the client closed the connection
                    return
                lines = head.split(b"\r\n")
                while lines and not lines[0]:   # stray CRLFs between keep-alive requests
                    lines.pop(0)
                if not lines:
                    continue
                try:
                    method, target, _ = lines[0].split(b" ", 2)
                except ValueError:
                    return
                hdrs = {}
                for h in lines[1:]:
                    if h:
                        k, _, v = h.partition(b":")
                        hdrs[k.strip().lower()] = v.strip()
                n = int(hdrs.get(b"content-length", b"0") or 0)
                body = await reader.readexactly(n) if n else b""
                sink = _Sink()
                try:
                    w = self._router.route(sink, method.decode(), target.decode(), body)
                except Exception as e:  # noqa: BLE001 - a malformed request must not end the server
                    w = None
                    sink.json(500, {"kind": "Status", "code": 500, "message": f"{type(e).__name__}: {e}"})
                if w is not None:   # a watch owns the connection until it ends; then keep-alive
                    # goes on (a client pool reuses the connection: closing it here would
                    # reset the next request sent on it)
                    await self._watch(writer, *w)
                    continue
                writer.write(sink.out)
                if writer.transport.get_write_buffer_size() > (1 << 20):
                    await writer.drain()
                if hdrs.get(b"connection", b"").lower() == b"close":
                    await writer.drain()
                    return
        except (ConnectionError, asyncio.IncompleteReadError):
            pass
        finally:
            writer.close()

    async def _watch(self, writer: asyncio.StreamWriter, res, ns, rv) -> None:
        loop = self.loop
        aq: asyncio.Queue = asyncio.Queue()
        on_loop = threading.get_ident

        def sink(item) -> None:   # the store's fan-out: on this loop, or from an in-process thread
            if on_loop() == self._t.ident:
                aq.put_nowait(item)
            else:
                loop.call_soon_threadsafe(aq.put_nowait, item)

        w = self.fk.watch(res, ns, rv, sink=sink)
        writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n")
        try:
            while True:
                items = [await aq.get()]
                while len(items) < 256 and not aq.empty():
                    items.append(aq.get_nowait())
                out, end = [], None
                for it in items:
                    if it is FakeWatch._END or isinstance(it, WatchClosed):
                        end = it
                        break
                    out.append(_chunk(it.wire()))
                if end is not None:
                    if isinstance(end, WatchClosed):
                        out.append(_chunk(json.dumps({"type": "ERROR", "object": {
                            "code": end.code or 500, "message": str(end),
                            "reason": "Expired" if end.code == 410 else "Error"}}).encode() + b"\n"))
                    out.append(b"0\r\n\r\n")
                    writer.write(b"".join(out))
                    await writer.drain()
                    return
                writer.write(b"".join(out))
                await writer.drain()
        except (ConnectionError, RuntimeError):
            pass
        finally:
            w.close()
