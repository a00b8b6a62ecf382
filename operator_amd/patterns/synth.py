"""Synthetic pattern libraries and pod logs (tests + benchmarks).

There is no network, so neither the reference's pattern repos
(``podmortem-patterns.git``, reference README.md:43-47) nor real pod logs are
available. This module generates both deterministically from a seed:

* ``catalog_library()``  — ~30 hand-written signatures of common container
  failures (OOM, crash loops, connection errors, JVM/Go/Python crashes...).
* ``synthetic_library(n)`` — the catalog plus generated signatures up to n
  patterns (literal and regex primaries, shared secondary phrases), sized like
  BASELINE.json config 2 ("1k patterns").
* ``LogFactory`` — fast log synthesis: a pool of benign lines is sampled with
  numpy and failure lines (matching primaries, with secondaries nearby) are
  injected; returns the bytes plus the ground-truth injected pattern ids.
"""
from __future__ import annotations

import random

import numpy as np
import yaml

from .schema import PatternSet

CATALOG = [
    ("oom-killed", "Container OOMKilled", "CRITICAL", "memory", {"literal": "OOMKilled"},
     [{"literal": "memory limit", "weight": 0.5, "proximity_window": 20}], "OOMKilled: container exceeded memory limit"),
    ("java-oom", "Java OutOfMemoryError", "CRITICAL", "memory",
     {"regex": r"java\.lang\.OutOfMemoryError: (Java heap space|GC overhead limit exceeded|Metaspace)"},
     [{"literal": "at java.util", "weight": 0.3, "proximity_window": 10}],
     "Exception in thread \"main\" java.lang.OutOfMemoryError: Java heap space"),
    ("conn-refused", "Connection refused", "HIGH", "network", {"literal": "Connection refused"},
     [{"regex": r"retry(ing)? in \d+", "weight": 0.4, "proximity_window": 5}], "dial tcp 10.0.0.12:5432: connect: Connection refused"),
    ("dns-fail", "DNS resolution failure", "HIGH", "network", {"regex": r"no such host|Temporary failure in name resolution"},
     [], "lookup db.internal on 10.96.0.10:53: no such host"),
    ("go-panic", "Go panic", "CRITICAL", "runtime", {"regex": r"^panic: "},
     [{"literal": "goroutine", "weight": 0.6, "proximity_window": 5}], "panic: runtime error: invalid memory address or nil pointer dereference"),
    ("segfault", "Segmentation fault", "CRITICAL", "runtime", {"regex": r"[Ss]egmentation fault|SIGSEGV"},
     [{"literal": "core dumped", "weight": 0.3, "proximity_window": 3}], "Segmentation fault (core dumped)"),
    ("py-traceback", "Python unhandled exception", "HIGH", "runtime", {"literal": "Traceback (most recent call last)"},
     [{"regex": r"^\w+(Error|Exception): ", "weight": 0.6, "proximity_window": 30}], "Traceback (most recent call last):"),
    ("tls-handshake", "TLS handshake failure", "HIGH", "security", {"regex": r"tls: (handshake failure|bad certificate)"},
     [{"literal": "x509", "weight": 0.5, "proximity_window": 10}], "remote error: tls: bad certificate"),
    ("x509-expired", "Certificate expired", "HIGH", "security", {"literal": "x509: certificate has expired"}, [],
     "x509: certificate has expired or is not yet valid"),
    ("perm-denied", "Permission denied", "MEDIUM", "filesystem", {"literal": "Permission denied"}, [],
     "open /var/lib/app/data.db: Permission denied"),
    ("disk-full", "No space left on device", "CRITICAL", "filesystem", {"literal": "No space left on device"}, [],
     "write /data/wal/000001.log: No space left on device"),
    ("readonly-fs", "Read-only file system", "HIGH", "filesystem", {"literal": "Read-only file system"}, [],
     "mkdir /etc/app: Read-only file system"),
    ("db-auth", "Database authentication failed", "HIGH", "database",
     {"regex": r"password authentication failed for user \"?\w+"}, [], "FATAL: password authentication failed for user \"app\""),
    ("db-too-many", "Too many connections", "HIGH", "database", {"literal": "too many connections"}, [],
     "pq: sorry, too many connections for role \"app\""),
    ("deadlock", "Deadlock detected", "MEDIUM", "database", {"literal": "deadlock detected"}, [],
     "ERROR: deadlock detected"),
    ("liveness", "Liveness probe failed", "MEDIUM", "kubernetes", {"literal": "Liveness probe failed"},
     [{"literal": "Back-off restarting failed container", "weight": 0.5, "proximity_window": 50}],
     "Liveness probe failed: HTTP probe failed with statuscode: 503"),
    ("crashloop", "CrashLoopBackOff", "HIGH", "kubernetes", {"literal": "Back-off restarting failed container"}, [],
     "Back-off restarting failed container app in pod app-7d9f"),
    ("image-pull", "Image pull failure", "HIGH", "kubernetes", {"regex": r"(ErrImagePull|ImagePullBackOff)"}, [],
     "Failed to pull image \"registry/app:1.2\": ErrImagePull"),
    ("config-missing", "Missing configuration", "MEDIUM", "config", {"regex": r"(missing|required) (config|configuration|environment variable)"},
     [], "error: required environment variable DATABASE_URL is not set"),
    ("quarkus-fail", "Quarkus startup failure", "HIGH", "framework", {"literal": "Failed to start application"},
     [{"literal": "Caused by:", "weight": 0.5, "proximity_window": 40}], "ERROR [io.quarkus.runtime.Application] Failed to start application"),
    ("spring-fail", "Spring context failure", "HIGH", "framework", {"literal": "APPLICATION FAILED TO START"},
     [{"literal": "Description:", "weight": 0.3, "proximity_window": 10}], "APPLICATION FAILED TO START"),
    ("port-in-use", "Address already in use", "MEDIUM", "network", {"literal": "address already in use"}, [],
     "listen tcp :8080: bind: address already in use"),
    ("timeout", "Upstream timeout", "MEDIUM", "network", {"regex": r"(context deadline exceeded|i/o timeout|timed out after \d+)"},
     [], "rpc error: code = DeadlineExceeded desc = context deadline exceeded"),
    ("node-unreachable", "Broken pipe / reset", "LOW", "network", {"regex": r"(broken pipe|connection reset by peer)"}, [],
     "write tcp 10.1.2.3:443: broken pipe"),
    ("npe", "NullPointerException", "HIGH", "runtime", {"literal": "java.lang.NullPointerException"},
     [{"literal": "at com.", "weight": 0.3, "proximity_window": 10}], "java.lang.NullPointerException: Cannot invoke \"String.length()\""),
    ("killed-137", "Killed (exit 137)", "HIGH", "memory", {"regex": r"exit(ed)? (code|status) 137"}, [],
     "process exited with exit code 137"),
    ("assert-fail", "Assertion failure", "MEDIUM", "runtime", {"literal": "Assertion failed"}, [],
     "Assertion failed: (ptr != NULL), function main"),
    ("rate-limit", "Rate limited", "LOW", "network", {"regex": r"(429 Too Many Requests|rate limit exceeded)"}, [],
     "received 429 Too Many Requests from api.example.com"),
    ("kafka-leader", "Kafka leader not available", "MEDIUM", "messaging", {"literal": "LEADER_NOT_AVAILABLE"}, [],
     "Error while fetching metadata with correlation id 42 : {orders=LEADER_NOT_AVAILABLE}"),
    ("fatal-generic", "Fatal error", "HIGH", "runtime", {"regex": r"\bFATAL\b"}, [], "FATAL: unrecoverable state, shutting down"),
]

_SYL = ["ka", "lo", "mi", "ra", "ten", "vo", "zu", "shi", "pre", "dor", "gan", "bel", "quin", "tro", "fex", "nor",
        "cal", "dri", "hul", "sem", "par", "vin", "jor", "lek"]
_COMPONENTS = ["http-server", "db-pool", "scheduler", "auth", "cache", "worker", "grpc", "kafka-consumer", "ingest",
               "billing", "search", "gateway", "metrics", "session", "queue", "storage"]
_MSGS = ["request completed", "processing batch", "heartbeat ok", "cache hit ratio", "flushed segment",
         "accepted connection", "scheduled job", "checkpoint written", "GET /api/v1/items", "POST /api/v1/orders",
         "rebalanced partitions", "config reloaded", "health check passed", "compaction finished", "token refreshed"]


def catalog_library() -> PatternSet:
    items = []
    for pid, name, sev, cat, prim, secs, _ex in CATALOG:
        items.append({"id": pid, "name": name, "severity": sev, "category": cat,
                      "primary_pattern": dict(prim, confidence=0.9), "secondary_patterns": secs,
                      "remediation": {"description": f"See runbook for {name}."}})
    return PatternSet.from_dicts(items, "catalog")


def _words(rng: random.Random, n: int) -> list[str]:
    out, seen = [], set()
    while len(out) < n:
        w = "".join(rng.choice(_SYL) for _ in range(rng.randint(2, 3)))
        if w not in seen:
            seen.add(w)
            out.append(w)
    return out


def _gen_items(n: int, seed: int) -> tuple[list[dict], dict[str, list[str]]]:
    rng = random.Random(seed)
    words = _words(rng, 600)
    shared_secs = [("retrying request", 0.3, 10), ("circuit breaker open", 0.5, 20), ("rolling back transaction", 0.4, 15),
                   ("upstream unhealthy", 0.3, 8)]
    items, examples = [], {}
    sevs = ["CRITICAL", "HIGH", "HIGH", "MEDIUM", "MEDIUM", "LOW", "INFO"]
    for i in range(n):
        w1, w2, w3, w4 = rng.sample(words, 4)
        pid = f"gen-{i:05d}"
        if rng.random() < 0.7:
            lit = f"E{i:05d} {w1} {w2} {w3} failure"
            prim = {"literal": lit, "confidence": round(rng.uniform(0.6, 0.95), 2)}
            ex = [f"{rng.choice(_COMPONENTS)}: {lit} (component={w4})"]
        else:
            prim = {"regex": rf"{w1}-{w2} worker \d+ crashed: {w3} {w4} unavailable",
                    "confidence": round(rng.uniform(0.6, 0.95), 2)}
            ex = [f"[{rng.choice(_COMPONENTS)}] {w1}-{w2} worker {rng.randint(1, 999)} crashed: {w3} {w4} unavailable"]
        secs = []
        for s, w, win in rng.sample(shared_secs, rng.randint(0, 2)):
            secs.append({"literal": s, "weight": w, "proximity_window": win})
        items.append({"id": pid, "name": f"{w1.title()} {w2} failure", "severity": rng.choice(sevs),
                      "category": rng.choice(["runtime", "network", "storage", "config"]),
                      "primary_pattern": prim, "secondary_patterns": secs})
        examples[pid] = ex
    return items, examples


def synthetic_library(n_patterns: int = 1000, seed: int = 0) -> PatternSet:
    base = catalog_library()
    items, _ = _gen_items(max(0, n_patterns - len(base)), seed)
    return base.merged(PatternSet.from_dicts(items, "generated"))


def library_yaml(n_patterns: int = 1000, seed: int = 0, library_id: str = "synthetic") -> str:
    items, _ = _gen_items(n_patterns, seed)
    return yaml.safe_dump({"metadata": {"library_id": library_id, "version": "1.0"}, "patterns": items},
                          sort_keys=False)


class LogFactory:
    """Deterministic pod-log synthesizer with injected failure signatures."""

    def __init__(self, n_patterns: int = 1000, seed: int = 0, pool_lines: int = 8192, library_seed: int = 0):
        """``seed`` varies the background lines; the injected failure signatures are the
        examples of ``synthetic_library(n_patterns, seed=library_seed)`` — the library
        the logs are scanned with — whatever ``seed`` is. (They once followed ``seed``,
        so a factory seeded differently from its library injected signatures that the
        library does not contain: bench.py's extra shards and ranks got lighter logs.)"""
        self.seed = seed
        rng = random.Random(seed + 1)
        gen_items, gen_examples = _gen_items(max(0, n_patterns - len(CATALOG)), library_seed)
        self.examples: dict[str, list[str]] = {c[0]: [c[6]] for c in CATALOG}
        self.examples.update(gen_examples)
        self.secondary_examples = {
            "oom-killed": "container memory limit reached (512Mi)",
            "java-oom": "\tat java.util.Arrays.copyOf(Arrays.java:3332)",
            "conn-refused": "retrying in 5 seconds",
            "go-panic": "goroutine 1 [running]:",
            "py-traceback": "ValueError: invalid literal for int() with base 10: 'x'",
            "liveness": "Back-off restarting failed container",
            "quarkus-fail": "Caused by: java.lang.IllegalStateException: boom",
        }
        self.ids = list(self.examples)
        pool = []
        for i in range(pool_lines):
            ts = f"2025-08-29T{rng.randint(0, 23):02d}:{rng.randint(0, 59):02d}:{rng.randint(0, 59):02d}.{rng.randint(0, 999):03d}Z"
            lvl = rng.choice(["INFO", "INFO", "INFO", "DEBUG", "WARN"])
            comp = rng.choice(_COMPONENTS)
            msg = rng.choice(_MSGS)
            extra = f"id={rng.randint(1, 10**9):x} latency_ms={rng.randint(1, 900)} user=u{rng.randint(1, 99999)}"
            pool.append(f"{ts} {lvl:5s} [{comp}] {msg} {extra}".encode())
        self.pool = np.array(pool, dtype=object)

    def log(self, rng: np.random.Generator, approx_bytes: int, n_failures: int = 3) -> tuple[bytes, list[str]]:
        n_lines = max(4, approx_bytes // 88)
        idx = rng.integers(0, len(self.pool), n_lines)
        lines = list(self.pool[idx])
        injected = []
        inserts = []
        for _ in range(n_failures):
            pid = self.ids[int(rng.integers(0, len(self.ids)))]
            at = int(rng.integers(0, len(lines) + 1))
            ex = self.examples[pid]
            block = [ex[int(rng.integers(0, len(ex)))].encode()]
            sec = self.secondary_examples.get(pid)
            if sec:
                block += [lines[int(rng.integers(0, len(lines)))], sec.encode()]
            inserts.append((at, block))
            injected.append(pid)
        # insert (never overwrite) so every injected signature survives
        for at, block in sorted(inserts, key=lambda t: -t[0]):
            lines[at:at] = block
        return b"\n".join(lines) + b"\n", injected

    def batch(self, n_docs: int, approx_bytes: int, n_failures: int = 3, seed: int | None = None):
        rng = np.random.default_rng(self.seed if seed is None else seed)
        docs, truth = [], []
        for _ in range(n_docs):
            d, t = self.log(rng, approx_bytes, n_failures)
            docs.append(d)
            truth.append(t)
        return docs, truth
