"""Multi-GPU engine pool: one engine process per GPU behind the CPU controller.

SURVEY.md §5.8 "Process model": the controller (kube watches, reconcilers,
sinks) is a CPU process; each GPU gets its own engine process holding the
log-scan DFA and a TP=1 explanation model (P1 / P2: data parallel over
failures and over explanation requests). The reference's two single-replica
REST services (``K/log-parser-deployment.yaml:8``,
``K/ai-interface-deployment.yaml:8``) become these workers, reached over
local pipes instead of HTTP.

* Routing: least outstanding requests among live, ready workers — every
  worker holds the full pattern set and model, so any worker can serve any
  failure; batching happens inside the worker (LocalMatchService micro-batches
  scans, the LLM engine continuously batches explanations).
* Health loop (SURVEY.md §5.3 "GPU-worker health loop"): a worker that exits
  (GPU fault, OOM kill) or stops heart-beating is drained — its in-flight
  requests are re-queued to the surviving workers — and respawned up to
  ``max_restarts`` times.
* Fault injection: ``inject_crash(i)`` makes worker i exit abruptly, for the
  recovery tests (the engine-side half of the §5.3 fault matrix).
* Pattern updates (PatternLibrary sync) are broadcast to every worker.
* Pod logs travel through a per-worker shared-memory arena (``_LogArena``): the
  controller copies the log's bytes into the worker's ring once and sends only
  (offset, length) with the log-less request; the worker hands those bytes to its
  scan batcher without a str round trip. Logs that do not fit the free ring space
  fall back to the pickled request.

Workers are started with the ``spawn`` method before the controller touches
any GPU, so no process ever forks a GPU-initialised parent.
"""
from __future__ import annotations

import itertools
import logging
import multiprocessing as mp
import os
import queue
import threading
import time
from concurrent.futures import Future

from operator_amd.api.models import AIProviderConfig, AIResponse, AnalysisResult, PodFailureData

log = logging.getLogger(__name__)


class WorkerDied(RuntimeError):
    pass


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


# ---------------------------------------------------------------- worker process
def _tp_init(tp_rank: int, tp_world: int, tp_port: int, device: str):
    """Process group of one TP replica (its own rendezvous port; RCCL on GPUs, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    from operator_amd.parallel.comm import Group

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(tp_port)
    backend = "nccl" if device.startswith("cuda") else "gloo"
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(torch.device(device))
        kw["device_id"] = torch.device(device)
    dist.init_process_group(backend, rank=tp_rank, world_size=tp_world, **kw)
    return Group()


class _LogArena:
    """Ring allocator over one worker's shared-memory log buffer (controller side).
    Allocations are released when their request's reply (or the worker's death)
    arrives; space is reclaimed in allocation order, so one slow request holds back
    at most the ring behind it, and a full ring only means the pickled path."""

    def __init__(self, size: int):
        from multiprocessing import shared_memory

        self.shm = shared_memory.SharedMemory(create=True, size=size)
        self.size = size
        self._live: dict[int, list] = {}       # rid -> [start, end, released]
        self._order: list[int] = []            # rids in allocation order
        self.head = self.tail = 0              # next free byte / oldest live byte
        self.copied = self.fallbacks = 0

    def reset(self) -> None:   # the worker died: nothing it read is in flight any more
        self._live.clear()
        self._order.clear()
        self.head = self.tail = 0

    def put(self, rid: int, data: bytes) -> int | None:
        n = len(data)
        if n == 0 or n > self.size // 4:
            self.fallbacks += 1
            return None
        if not self._live:
            self.head = self.tail = 0
        if self.head >= self.tail:                       # free: [head, size) and [0, tail)
            if self.head + n <= self.size:
                off = self.head
            elif n < self.tail:
                off = 0
            else:
                self.fallbacks += 1
                return None
        elif self.head + n < self.tail:                  # free: [head, tail)
            off = self.head
        else:
            self.fallbacks += 1
            return None
        self.shm.buf[off:off + n] = data
        self.head = off + n
        self._live[rid] = [off, off + n, False]
        self._order.append(rid)
        self.copied += 1
        return off

    def release(self, rid: int) -> None:
        a = self._live.get(rid)
        if a is None:
            return
        a[2] = True
        while self._order and self._live[self._order[0]][2]:
            del self._live[self._order.pop(0)]
        if self._order:
            self.tail = self._live[self._order[0]][0]
        else:
            self.head = self.tail = 0

    def close(self) -> None:
        try:
            self.shm.close()
            self.shm.unlink()
        except (FileNotFoundError, OSError):
            pass


def _follower_main(idx: int, device: str, settings_obj: dict, tp_rank: int, tp_world: int, tp_port: int,
                   outq) -> None:
    """Non-leader rank of a TP replica: holds its model shard and mirrors the leader's steps."""
    logging.basicConfig(level=os.environ.get("PODMORTEM_LOG_LEVEL", "WARNING"))
    from operator_amd.config import Settings
    from operator_amd.engine import factory

    s = Settings.model_validate(settings_obj)
    s.engine.device = device
    try:
        tp = _tp_init(tp_rank, tp_world, tp_port, device)
        _, _, llm, _ = factory.build_llm(s, device=device, tp=tp)
    except Exception as e:  # noqa: BLE001
        outq.put(("fatal", idx, f"TP rank {tp_rank}: {type(e).__name__}: {e}"))
        return
    llm.follow()


def _worker_main(idx: int, device: str, settings_obj: dict, patterns, roles: tuple[str, ...], inq, outq,
                 heartbeat_s: float, tp_world: int = 1, tp_port: int = 0, arena_name: str | None = None) -> None:
    logging.basicConfig(level=os.environ.get("PODMORTEM_LOG_LEVEL", "WARNING"))
    from concurrent.futures import ThreadPoolExecutor

    from operator_amd.config import Settings
    from operator_amd.engine import factory, service

    s = Settings.model_validate(settings_obj)
    s.engine.device = device
    if device == "cpu" and s.services.match != "stub":
        s.services.match = "cpu"
    matcher = explainer = None
    try:
        tp = _tp_init(0, tp_world, tp_port, device) if tp_world > 1 else None
        if "match" in roles and s.services.match == "stub":
            matcher = service.StubMatchService()
        elif "match" in roles:
            matcher = service.LocalMatchService(factory.build_match_engine(s, patterns, device=device),
                                                s.services.match_max_batch, s.services.match_batch_wait_ms)
        if "explain" in roles:
            explainer = factory.build_explain_service(s, tp=tp)
            llm = getattr(getattr(explainer, "ee", None), "llm", None)
            if llm is not None and tp is None and s.engine.warmup_graphs:
                llm.warmup()   # capture the decode / prefill graphs before reporting ready
    except Exception as e:  # noqa: BLE001 - reported to the controller, which marks the worker dead
        outq.put(("fatal", idx, f"{type(e).__name__}: {e}"))
        return
    stop = threading.Event()

    loop = getattr(getattr(explainer, "ee", None), "loop", None)

    def beat():
        while not stop.wait(heartbeat_s):
            if loop is not None and getattr(loop, "fatal", None) is not None:
                # unrecoverable engine state (a TP collective timed out): die like a GPU
                # fault so the health loop re-queues the in-flight work and respawns us
                outq.put(("fatal", idx, f"engine failed: {loop.fatal}"))
                os._exit(70)
            outq.put(("hb", idx, time.time()))

    threading.Thread(target=beat, daemon=True).start()
    outq.put(("ready", idx, {"device": device, "pid": os.getpid(), "roles": list(roles)}))
    # one thread per in-flight request (an explain blocks its thread until generated):
    # as many as the engine can batch, twice, like the controller's own pipeline pool
    pool = ThreadPoolExecutor(max_workers=max(4, s.operator.workers or 2 * s.engine.max_batch + 16))

    arena = None
    if arena_name:
        from multiprocessing import shared_memory

        # the controller owns and unlinks the segment (spawned workers share its
        # resource tracker, which already holds the one registration of this name)
        arena = shared_memory.SharedMemory(name=arena_name)

    def run_shm(rid, payload, off, n):
        log_bytes = bytes(arena.buf[off:off + n])   # copied out before the reply frees the slot
        try:
            fut = matcher.submit(payload, log_bytes)
            outq.put(("ok", idx, rid, fut.result()))
        except Exception as e:  # noqa: BLE001
            outq.put(("err", idx, rid, f"{type(e).__name__}: {e}"))

    def run(rid, kind, payload):
        # requests and results cross the process boundary as the pydantic objects
        # themselves (pickled by the queue): no dict round trip, no re-validation of a
        # whole AnalysisResult on the controller's GIL per failure
        try:
            if kind == "match":
                res = matcher.analyze(payload)
            else:
                res = explainer.explain(payload[0], payload[1])
            outq.put(("ok", idx, rid, res))
        except Exception as e:  # noqa: BLE001 - per-request failure, worker stays up
            outq.put(("err", idx, rid, f"{type(e).__name__}: {e}"))

    while True:
        msg = inq.get()
        kind = msg[0]
        if kind == "stop":
            break
        if kind == "crash":           # fault injection: die like a GPU fault would
            os._exit(int(msg[1]))
        if kind == "hang":            # fault injection: stop heart-beating and serving
            stop.set()
            time.sleep(3600)
        if kind == "patterns":
            if matcher is not None:
                matcher.swap_engine(factory.build_match_engine(s, msg[1], device=device))
            continue
        if kind == "stats":          # engine counters for the controller (bench, metrics)
            outq.put(("ok", idx, msg[1], _worker_stats(matcher, explainer)))
            continue
        if kind in ("match", "explain"):
            pool.submit(run, msg[1], kind, msg[2])
        elif kind == "match_shm":
            pool.submit(run_shm, msg[1], msg[2], msg[3], msg[4])
    stop.set()
    pool.shutdown(wait=True)
    if matcher is not None:
        matcher.close()
    ee = getattr(explainer, "ee", None)
    if ee is not None:   # stops the engine loop (a TP leader releases its followers)
        ee.close(join_s=30.0)


def _worker_stats(matcher, explainer) -> dict:
    from dataclasses import asdict

    out: dict = {}
    llm = getattr(getattr(explainer, "ee", None), "llm", None)
    if llm is not None:
        out["llm"] = asdict(llm.stats)
        out["prefill_graph_buckets"] = sorted(getattr(llm, "_prefill_g", {}))
        out["use_graphs"] = bool(getattr(llm, "use_graphs", False))
    eng = getattr(matcher, "engine", None)
    if eng is not None:
        out["dfa_states"] = getattr(eng, "dfa_states", None)
    return out


# ---------------------------------------------------------------- controller side
class _Worker:
    """One engine replica: a single process, or a TP group (leader = ``proc``, + ``followers``)."""

    def __init__(self, idx: int, device: str, follower_devices: list[str] | None = None):
        self.idx, self.device = idx, device
        self.follower_devices = list(follower_devices or [])
        self.proc = None
        self.followers: list = []
        self.inq = None
        self.ready = False
        self.alive = False
        self.last_beat = 0.0
        self.restarts = 0
        self.inflight: dict[int, tuple] = {}
        self.info: dict = {}
        self.arena: _LogArena | None = None


class EnginePool:
    def __init__(self, settings, patterns, devices: list[str], roles: tuple[str, ...] = ("match", "explain"),
                 heartbeat_s: float = 2.0, heartbeat_timeout_s: float = 30.0, max_restarts: int = 3,
                 log_arena_mb: float | None = None):
        self.settings, self.patterns, self.roles = settings, patterns, roles
        mb = getattr(settings.engine, "pool_log_arena_mb", 64) if log_arena_mb is None else log_arena_mb
        self.log_arena_bytes = int(mb * (1 << 20)) if "match" in roles else 0
        self.heartbeat_s, self.heartbeat_timeout_s = heartbeat_s, heartbeat_timeout_s
        self.max_restarts = max_restarts
        self._ctx = mp.get_context("spawn")
        self._outq = self._ctx.Queue()
        self._lock = threading.Lock()
        self._ready_cv = threading.Condition(self._lock)
        self._ids = itertools.count()
        self._closing = False
        self.tp = max(1, int(getattr(settings.engine, "tp", 1)))
        if len(devices) % self.tp:
            raise ValueError(f"{len(devices)} devices cannot be split into TP groups of {self.tp}")
        groups = [devices[i:i + self.tp] for i in range(0, len(devices), self.tp)]
        self.workers = [_Worker(i, g[0], g[1:]) for i, g in enumerate(groups)]
        self.stats = {"requeued": 0, "restarts": 0, "deaths": 0}
        for w in self.workers:
            self._spawn(w)
        self._reader = threading.Thread(target=self._read_loop, name="pool-reader", daemon=True)
        self._reader.start()
        self._monitor = threading.Thread(target=self._monitor_loop, name="pool-monitor", daemon=True)
        self._monitor.start()

    # ---------------------------------------------------------------- lifecycle
    def _spawn(self, w: _Worker) -> None:
        # under the pool lock: _handle may still release() a late reply of the killed
        # process into this arena and _dispatch put() into it as soon as alive is set,
        # so the ring reset and the alive/ready transition must not interleave with either
        with self._lock:
            if self.log_arena_bytes and w.arena is None:
                w.arena = _LogArena(self.log_arena_bytes)
            if w.arena is not None:
                w.arena.reset()
            w.inq = self._ctx.Queue()
            w.ready, w.alive, w.last_beat = False, True, time.time()
        world = 1 + len(w.follower_devices)
        port = _free_port() if world > 1 else 0
        settings = self.settings.model_dump()
        w.proc = self._ctx.Process(
            target=_worker_main, name=f"engine-{w.idx}",
            args=(w.idx, w.device, settings, self.patterns, self.roles, w.inq, self._outq,
                  self.heartbeat_s, world, port, w.arena.shm.name if w.arena is not None else None), daemon=True)
        w.followers = [self._ctx.Process(target=_follower_main, name=f"engine-{w.idx}-tp{r}",
                                         args=(w.idx, d, settings, r, world, port, self._outq), daemon=True)
                       for r, d in enumerate(w.follower_devices, start=1)]
        w.proc.start()
        for f in w.followers:
            f.start()

    @staticmethod
    def _procs(w: _Worker) -> list:
        return [p for p in [w.proc, *w.followers] if p is not None]

    def wait_ready(self, timeout: float = 600.0, n: int | None = None) -> int:
        """Block until ``n`` (default: all) workers are ready; returns the ready count."""
        need = len(self.workers) if n is None else n
        deadline = time.time() + timeout
        with self._ready_cv:
            while sum(w.ready for w in self.workers) < need:
                left = deadline - time.time()
                if left <= 0 or not any(w.alive for w in self.workers):
                    break
                self._ready_cv.wait(min(left, 1.0))
            return sum(w.ready for w in self.workers)

    def close(self, timeout: float = 30.0) -> None:
        self._closing = True
        for w in self.workers:
            if w.alive:
                try:
                    w.inq.put(("stop",))
                except (OSError, ValueError):
                    pass
        for w in self.workers:
            for p in self._procs(w):
                p.join(timeout)
                if p.is_alive():
                    p.kill()
                    p.join(5)
        with self._lock:
            for w in self.workers:
                for rid, (kind, payload, fut) in list(w.inflight.items()):
                    if not fut.done():
                        fut.set_exception(WorkerDied("engine pool closed"))
                w.inflight.clear()
                if w.arena is not None:
                    w.arena.close()
                    w.arena = None

    # ---------------------------------------------------------------- requests
    def _pick(self) -> _Worker | None:
        live = [w for w in self.workers if w.alive and w.ready]
        if not live:
            return None
        return min(live, key=lambda w: (len(w.inflight), w.idx))

    def _dispatch(self, kind: str, payload, fut: Future, rid: int | None = None) -> None:
        with self._lock:
            w = self._pick()
            if w is None:
                if any(x.alive for x in self.workers):   # still starting: wait for one
                    self._ready_cv.wait_for(lambda: self._pick() is not None or self._closing, timeout=600)
                    w = self._pick()
                if w is None:
                    fut.set_exception(WorkerDied("no live engine worker"))
                    return
            rid = next(self._ids) if rid is None else rid
            w.inflight[rid] = (kind, payload, fut)
            if kind == "match" and w.arena is not None and payload.logs:
                off = w.arena.put(rid, payload.logs.encode("utf-8", "replace"))
                if off is not None:   # the log rides the shared-memory ring; the request carries none
                    w.inq.put(("match_shm", rid, payload.model_copy(update={"logs": None}), off,
                               w.arena._live[rid][1] - off))   # noqa: SLF001
                    return
            w.inq.put((kind, rid, payload))

    def submit_match(self, data: PodFailureData) -> Future:
        fut: Future = Future()
        self._dispatch("match", data, fut)
        return fut

    def submit_explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> Future:
        fut: Future = Future()
        self._dispatch("explain", (result, cfg), fut)
        return fut

    def worker_stats(self, timeout: float = 30.0) -> list[dict]:
        """Engine counters of every live worker (LLM EngineStats, prefill graph buckets,
        DFA size), one dict per worker."""
        futs = []
        with self._lock:
            for w in self.workers:
                if w.alive and w.ready:
                    fut: Future = Future()
                    rid = next(self._ids)
                    w.inflight[rid] = ("stats", None, fut)
                    w.inq.put(("stats", rid))
                    futs.append(fut)
        return [f.result(timeout) for f in futs]

    def set_patterns(self, patterns) -> None:
        self.patterns = patterns
        with self._lock:
            for w in self.workers:
                if w.alive:
                    w.inq.put(("patterns", patterns))

    def inject_crash(self, idx: int, code: int = 139) -> None:
        self.workers[idx].inq.put(("crash", code))

    def inject_hang(self, idx: int) -> None:
        self.workers[idx].inq.put(("hang",))

    # ---------------------------------------------------------------- background loops
    def _read_loop(self) -> None:
        while True:
            try:
                msg = self._outq.get(timeout=0.5)
            except queue.Empty:
                if self._closing:
                    return
                continue
            except (EOFError, OSError):
                return
            if msg[0] == "batch":
                for m in msg[2]:
                    self._handle(m)
            else:
                self._handle(msg)

    def _handle(self, msg) -> None:
        kind, idx = msg[0], msg[1]
        w = self.workers[idx]
        item = None
        with self._lock:
            if kind == "hb":
                w.last_beat = time.time()
            elif kind == "ready":
                w.ready, w.info, w.last_beat = True, msg[2], time.time()
                self._ready_cv.notify_all()
            elif kind == "fatal":
                log.error("engine worker %d failed to start: %s", idx, msg[2])
                w.info["fatal"] = msg[2]
                w.restarts = self.max_restarts  # a start-up failure is not transient
            elif kind in ("ok", "err"):
                if w.arena is not None:
                    w.arena.release(msg[2])
                item = w.inflight.pop(msg[2], None)
        if item is not None and not item[2].done():   # waiters wake outside the pool lock
            if kind == "ok":
                item[2].set_result(msg[3])
            else:
                item[2].set_exception(RuntimeError(msg[3]))

    def _monitor_loop(self) -> None:
        while not self._closing:
            time.sleep(min(0.5, self.heartbeat_s))
            now = time.time()
            for w in self.workers:
                if not w.alive or self._closing:
                    continue
                gone = [p for p in self._procs(w) if not p.is_alive()]
                hung = w.ready and now - w.last_beat > self.heartbeat_timeout_s
                if gone or hung:
                    for p in self._procs(w):   # a TP replica lives and dies as a whole
                        if p.is_alive():
                            p.kill()
                    self._on_death(w, f"{gone[0].name} exited with {gone[0].exitcode}" if gone
                                   else "stopped heart-beating")

    def _on_death(self, w: _Worker, why: str) -> None:
        with self._lock:
            w.alive, w.ready = False, False
            orphans = list(w.inflight.items())
            w.inflight.clear()
            self.stats["deaths"] += 1
        log.error("engine worker %d (%s) %s; re-queueing %d in-flight requests", w.idx, w.device, why,
                  len(orphans))
        if w.restarts < self.max_restarts and not self._closing:
            w.restarts += 1
            self.stats["restarts"] += 1
            self._spawn(w)
        live = [(rid, item) for rid, item in orphans if not item[2].done()]
        self.stats["requeued"] += len(live)
        if live:  # re-dispatch off the monitor thread (it may wait for a worker to become ready)
            threading.Thread(target=lambda: [self._dispatch(k, p, f, rid) for rid, (k, p, f) in live],
                             name="pool-requeue", daemon=True).start()

    def health(self) -> dict:
        with self._lock:
            return {"workers": [{"idx": w.idx, "device": w.device, "tp_devices": [w.device, *w.follower_devices],
                                 "alive": w.alive, "ready": w.ready,
                                 "inflight": len(w.inflight), "restarts": w.restarts,
                                 "shm_logs": w.arena.copied if w.arena else 0,
                                 "shm_fallbacks": w.arena.fallbacks if w.arena else 0} for w in self.workers],
                    **self.stats}


class PoolMatchService:
    """LocalMatchService-compatible front for an EnginePool."""

    def __init__(self, pool: EnginePool, timeout_s: float = 600.0):
        self.pool, self.timeout_s = pool, timeout_s

    def analyze(self, data: PodFailureData) -> AnalysisResult:
        return self.pool.submit_match(data).result(self.timeout_s)

    def swap_engine(self, patterns) -> None:  # the pool rebuilds the DFA inside each worker
        self.pool.set_patterns(patterns)

    def close(self) -> None:
        pass


class PoolExplainService:
    """LocalExplainService-compatible front for an EnginePool."""

    def __init__(self, pool: EnginePool, timeout_s: float = 3600.0):
        self.pool, self.timeout_s = pool, timeout_s

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        return self.pool.submit_explain(result, cfg).result(self.timeout_s)

    def explain_many(self, items):
        futs = [self.pool.submit_explain(r, c) for r, c in items]
        return [f.result(self.timeout_s) for f in futs]

    def ready(self) -> bool:
        return any(w.ready for w in self.pool.workers)
