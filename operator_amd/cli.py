"""Command line: ``python -m operator_amd <command>``.

  run            start the operator (kube watch + reconcilers + GPU engines + health)
  manifests      print / write CRDs, RBAC and the Deployment (kubectl apply -f -)
  scan           pattern-analyse log files -> AnalysisResult JSON
  explain        scan + explain log files with the local LLM -> AIResponse JSON
  serve-compat   REST server speaking the reference's log-parser / ai-interface contracts
  bench          run bench.py (flagship benchmark)
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import signal
import sys
import threading
import time


def _settings(args):
    from operator_amd.config import load_settings

    ov = {}
    for kv in args.set or []:
        k, _, v = kv.partition("=")
        import yaml

        ov[k] = yaml.safe_load(v)
    return load_settings(getattr(args, "config", None), overrides=ov)


def _patterns(s, paths: list[str] | None):
    from operator_amd.patterns.schema import PatternSet
    from operator_amd.patterns.synth import catalog_library

    ps = catalog_library() if s.patterns.builtin_catalog else PatternSet([], [])
    for p in paths or []:
        ps = ps.merged(PatternSet.load_dir(p) if os.path.isdir(p) else PatternSet.from_yaml_text(open(p).read()))
    return ps


def cmd_manifests(args) -> int:
    from operator_amd.api.crds import render_all

    text = render_all(namespace=args.namespace, image=args.image, gpus=args.gpus, replicas=args.replicas,
                      shards=args.shards, shard_per_gpu=args.shard_per_gpu, compat=args.compat_services)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text)
    return 0


def cmd_scan(args) -> int:
    from operator_amd.engine.factory import build_match_engine

    s = _settings(args)
    if args.device:
        s.engine.device = args.device
        s.services.match = "cpu" if args.device == "cpu" else "local"
    eng = build_match_engine(s, _patterns(s, args.patterns), device=args.device)
    docs = [open(p, "rb").read() for p in args.logs]
    res = eng.analyze(docs, [(os.path.basename(p), None) for p in args.logs])
    print(json.dumps([r.to_obj() for r in res], indent=1))
    return 0


def cmd_explain(args) -> int:
    from operator_amd.api.models import AIProviderConfig
    from operator_amd.engine.explain import ExplainEngine
    from operator_amd.engine.factory import build_llm, build_match_engine

    s = _settings(args)
    eng = build_match_engine(s, _patterns(s, args.patterns))
    _, _, llm, tok = build_llm(s)
    ee = ExplainEngine(llm, tok, model_id=s.engine.model, max_prompt_tokens=s.engine.max_prompt_tokens)
    docs = [open(p, "rb").read() for p in args.logs]
    res = eng.analyze(docs, [(os.path.basename(p), None) for p in args.logs])
    cfg = AIProviderConfig(max_tokens=args.max_tokens, temperature=args.temperature)
    outs = ee.explain_many([(r, cfg) for r in res])
    print(json.dumps([o.to_obj() if hasattr(o, "to_obj") else {"error": str(o)} for o in outs], indent=1))
    ee.close()
    return 0


def _build_pool(s, patterns):
    """One engine process per GPU: the controller stays a CPU process."""
    from operator_amd.engine.pool import EnginePool, PoolExplainService, PoolMatchService

    if s.engine.device == "cpu":
        devices = ["cpu"] * max(1, s.engine.gpus)
    else:
        import torch

        n = torch.cuda.device_count()  # counts devices without initialising the GPU
        devices = [f"cuda:{i}" for i in range(min(max(1, s.engine.gpus), max(1, n)))]
    roles = tuple(r for r, on in (("match", s.services.match in ("local", "cpu", "stub")),
                                  ("explain", s.services.explain == "local")) if on)
    pool = EnginePool(s, patterns, devices, roles=roles)
    return pool, PoolMatchService(pool), PoolExplainService(pool)


def _build_services(s, metrics):
    from operator_amd.engine.factory import build_explain_service, build_match_engine
    from operator_amd.engine.service import LocalMatchService, RemoteLogParser, StubMatchService

    if s.services.match == "remote":
        matcher = RemoteLogParser(s.services.log_parser_url, s.services.log_parser_read_timeout_s,
                                  s.services.log_parser_connect_timeout_s)
        factory = None
    elif s.services.match == "stub":
        matcher, factory = StubMatchService(), None
    else:
        factory = lambda ps: build_match_engine(s, ps)  # noqa: E731
        matcher = None
    explainer = build_explain_service(s, metrics)
    return matcher, factory, explainer


def shard_env(base: dict, index: int, count: int, health_port: int, device: str | None = None) -> dict:
    """Environment of operator shard ``index`` of ``count`` started by ``run --shards`` /
    ``run --shard-per-gpu``: its slice of the pods, its own health/metrics port and, per
    GPU, the one device its engines own (applied over the config and the --set overrides
    by ``apply_shard_env``)."""
    env = dict(base)
    env.update({"OAMD_SHARD_CHILD": "1", "OAMD_SHARD_INDEX": str(index), "OAMD_SHARD_COUNT": str(count),
                "OAMD_SHARD_PORT": str(health_port + index)})
    if device is not None:
        env["OAMD_SHARD_DEVICE"] = device
    return env


def apply_shard_env(s, env: dict) -> None:
    if env.get("OAMD_SHARD_CHILD"):
        s.operator.shard_index = int(env["OAMD_SHARD_INDEX"])
        s.operator.shard_count = int(env["OAMD_SHARD_COUNT"])
        s.health.port = int(env["OAMD_SHARD_PORT"])
        if env.get("OAMD_SHARD_DEVICE"):   # shard-per-GPU: this shard's engines on one device
            s.engine.device = env["OAMD_SHARD_DEVICE"]
            s.engine.gpus = 1


def shard_device(base_device: str, index: int) -> str:
    """The device shard ``index`` owns in shard-per-GPU mode (CPU stays CPU: tests)."""
    return "cpu" if base_device == "cpu" else f"cuda:{index}"


class ShardSupervisor:
    """``run --shards K``: K-1 more operator processes on the same GPUs (K engine sets
    per GPU), started before this process touches a GPU. Shards scale the operator's
    host side (watch, collection, sinks: one Python process per shard). On one GPU
    they do not raise GPU throughput: 2 x 128 measured 26.6 analyses/s vs 28.2 for one
    operator with equal work (profiles/shards_equal_work_8b.jsonl).

    A shard that exits is started again (its slice of the pods would otherwise go
    unanalysed); more than ``max_restarts`` restarts within ``window_s`` makes
    ``poll`` return False so the whole pod fails and Kubernetes restarts it."""

    def __init__(self, argv: list[str], count: int, health_port: int, max_restarts: int = 5,
                 window_s: float = 300.0, clock=time.monotonic, devices: list[str] | None = None):
        self.argv, self.count, self.health_port = list(argv), count, health_port
        self.max_restarts, self.window_s, self.clock = max_restarts, window_s, clock
        self.devices = devices   # shard-per-GPU: shard i's device (None: every shard on every GPU)
        self.restarts: list[float] = []
        self.kids = {i: self._start(i) for i in range(1, count)}

    def _start(self, index: int):
        import subprocess

        return subprocess.Popen([sys.executable, "-m", "operator_amd", *self.argv],
                                env=shard_env(os.environ, index, self.count, self.health_port,
                                              self.devices[index] if self.devices else None))

    def poll(self) -> bool:
        """Restart exited shards; False once they crash-loop."""
        for i, k in list(self.kids.items()):
            rc = k.poll()
            if rc is None:
                continue
            now = self.clock()
            self.restarts = [t for t in self.restarts if now - t < self.window_s] + [now]
            if len(self.restarts) > self.max_restarts:
                logging.getLogger(__name__).error("operator shard %d exited (code %s): %d restarts in %.0f s, "
                                                  "giving up", i, rc, len(self.restarts) - 1, self.window_s)
                return False
            logging.getLogger(__name__).error("operator shard %d exited (code %s); starting it again", i, rc)
            self.kids[i] = self._start(i)
        return True

    def stop(self, timeout_s: float = 60.0) -> None:
        for k in self.kids.values():
            if k.poll() is None:
                k.terminate()
        for k in self.kids.values():
            try:
                k.wait(timeout_s)
            except Exception:  # noqa: BLE001 - a shard that ignores SIGTERM is killed
                k.kill()


def shard_sizing(s, count: int) -> None:
    """Per-shard engine sizing: the GPU's batch and KV budget split over the shards."""
    s.engine.max_batch = max(1, s.engine.max_batch // count)
    s.engine.kv_cache_gb = s.engine.kv_cache_gb / count


def cmd_run(args) -> int:
    from operator_amd.controller.operator import Operator
    from operator_amd.kube.client import KubeClient
    from operator_amd.kube.fake import FakeKube
    from operator_amd.utils.metrics import Metrics

    s = _settings(args)
    apply_shard_env(s, os.environ)
    if os.environ.get("OAMD_SHARD_CHILD"):
        try:   # a shard started by `run --shards` exits with the process that started it
            import ctypes

            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))   # PR_SET_PDEATHSIG
        except OSError:
            pass
    sup = None
    child = bool(os.environ.get("OAMD_SHARD_CHILD"))
    if args.shard_per_gpu:
        # production multi-GPU topology: one operator shard process per GPU, each owning
        # that GPU's engines in-process and its hash slice of the pods, all against the
        # same API server; the first process supervises (restarts) the others
        n = max(1, args.gpus or s.engine.gpus)
        if args.shards and args.shards > 1:
            raise SystemExit("--shard-per-gpu and --shards are exclusive")
        if not child:
            devs = [shard_device(s.engine.device, i) for i in range(n)]
            if n > 1:
                sup = ShardSupervisor(sys.argv[1:], n, s.health.port, devices=devs)
            s.operator.shard_count, s.operator.shard_index = n, 0
            s.engine.device, s.engine.gpus = devs[0], 1
    elif args.shards and args.shards > 1:   # shards of this process's GPUs (config-only sharding: one pod each)
        if not child:
            sup = ShardSupervisor(sys.argv[1:], args.shards, s.health.port)
            s.operator.shard_count, s.operator.shard_index = args.shards, 0
        shard_sizing(s, args.shards)
    if args.gpus and args.gpus > 1 and not args.shard_per_gpu:
        s.engine.gpus = args.gpus
    if args.tp and args.tp > 1:
        s.engine.tp = args.tp
        s.engine.gpus = max(s.engine.gpus, args.tp)
    pool = None
    metrics = Metrics()
    if s.kube.mode == "fake" or args.fake:
        kube = FakeKube()
    else:
        kube = KubeClient.auto(s.kube.mode, s.kube.kubeconfig, s.kube.request_timeout_s)
    if s.engine.gpus > 1 or s.engine.pool or s.engine.tp > 1:
        # engines first, before anything in this process could initialise a GPU
        from operator_amd.controller.operator import load_patterns

        pool, matcher, pool_explainer = _build_pool(s, load_patterns(s, kube))
        explainer = pool_explainer if "explain" in pool.roles else None
        if "match" not in pool.roles:
            matcher, factory, _ = _build_services(s, metrics)
        else:
            factory = lambda ps: ps  # noqa: E731 - the pool rebuilds the DFA in every worker
    else:
        matcher, factory, explainer = _build_services(s, metrics)
    op = Operator(kube, s, match_service=matcher, explain_service=explainer, metrics=metrics,
                  match_engine_factory=factory)
    op.start()
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    logging.getLogger(__name__).info("running; health on :%d", s.health.port)
    rc = 0
    while not stop.wait(1.0):
        if sup is not None and not sup.poll():
            rc = 1
            break
    op.stop()
    if pool is not None:
        pool.close()
    if sup is not None:   # the other shards stop with this one
        sup.stop()
    return rc


def cmd_serve_compat(args) -> int:
    from operator_amd.engine.server import CompatServer
    from operator_amd.engine.service import LocalMatchService
    from operator_amd.utils.metrics import Metrics

    s = _settings(args)
    metrics = Metrics()
    matcher, factory, explainer = _build_services(s, metrics)
    if matcher is None:
        matcher = LocalMatchService(factory(_patterns(s, args.patterns)), metrics=metrics)
    srv = CompatServer(matcher, explainer, s.health.host, args.port or s.health.port, metrics).start()
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    srv.stop()
    return 0


def cmd_bench(args, rest) -> int:
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.call([sys.executable, os.path.join(root, "bench.py"), *rest])


def main(argv: list[str] | None = None) -> int:
    logging.basicConfig(level=os.environ.get("PODMORTEM_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    ap = argparse.ArgumentParser(prog="operator_amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)

    def common(p):
        p.add_argument("--config", default=None)
        p.add_argument("--set", action="append", help="override, e.g. --set engine.model=tiny")

    p = sub.add_parser("run")
    common(p)
    p.add_argument("--fake", action="store_true", help="in-memory FakeKube instead of a cluster")
    p.add_argument("--gpus", type=int, default=0, help="engine processes, one per GPU (engine.gpus)")
    p.add_argument("--tp", type=int, default=0,
                   help="GPUs per explanation-model replica (engine.tp); --gpus 8 --tp 8 = one 70B replica")
    p.add_argument("--shards", type=int, default=0,
                   help="operator shards (processes splitting the pods, each with its own engines on the same "
                        "GPUs; operator.shard_count)")
    p.add_argument("--shard-per-gpu", action="store_true",
                   help="one operator shard process per GPU (--gpus N): shard i owns cuda:i and the pods hashing "
                        "to it, all shards on the same API server (the multi-GPU production topology)")
    p = sub.add_parser("manifests")
    p.add_argument("--namespace", default="podmortem-system")
    p.add_argument("--image", default="ghcr.io/podmortem/operator-amd:latest")
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--replicas", type=int, default=1, help=">1 enables Lease leader election")
    p.add_argument("--shards", type=int, default=1, help="operator shards per pod (run --shards)")
    p.add_argument("--shard-per-gpu", action="store_true", help="one operator shard per GPU (run --shard-per-gpu)")
    p.add_argument("--compat-services", action="store_true",
                   help="also emit log-parser / ai-interface Deployments+Services backed by serve-compat")
    p.add_argument("--out", default=None)
    p = sub.add_parser("scan")
    common(p)
    p.add_argument("logs", nargs="+")
    p.add_argument("--patterns", action="append", help="pattern YAML file or directory")
    p.add_argument("--device", default=None)
    p = sub.add_parser("explain")
    common(p)
    p.add_argument("logs", nargs="+")
    p.add_argument("--patterns", action="append")
    p.add_argument("--max-tokens", type=int, default=500)
    p.add_argument("--temperature", type=float, default=0.3)
    p = sub.add_parser("serve-compat")
    common(p)
    p.add_argument("--patterns", action="append")
    p.add_argument("--port", type=int, default=None)
    sub.add_parser("bench", add_help=False)
    args, rest = ap.parse_known_args(argv)
    if args.cmd == "bench":
        return cmd_bench(args, rest)
    if rest:
        ap.error(f"unrecognized arguments: {rest}")
    return {"run": cmd_run, "manifests": cmd_manifests, "scan": cmd_scan, "explain": cmd_explain,
            "serve-compat": cmd_serve_compat}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
