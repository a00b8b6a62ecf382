#!/usr/bin/env python3
"""Flagship benchmark: pod-failure analyses/sec (whole node) + p50 explanation
latency, Llama-3-8B explanation model at TP=1 per GPU, data-parallel over GPUs
(BASELINE.json metric; config 4 "End-to-end: synthetic pod failures -> pattern
match + 8B explanation, DP across 8xMI355X").

One process per GPU (torchrun / ``python -m torch.distributed.run``), RCCL
process group for the barrier + max-over-ranks timing. Each rank runs the
full operator — FakeKube (in-memory API server) + pod watcher + analysis
pipeline + GPU log scan (1k-pattern Aho-Corasick DFA) + Llama-3-8B bf16
explanation on the gfx950 kernels (continuous batching, hipGraph decode) +
result sinks (pod annotations, Podmortem status ring, Events).

A *step* is one wave of ``--batch`` failures per GPU: the failed pods are
written to FakeKube (MODIFIED events), the watcher picks them up, and the step
ends when every failure's analysis + explanation is stored. Weak scaling:
per-GPU work is fixed as N grows. Work per failure: one synthetic ~``--log-kb``
KiB pod log scanned against the pattern library, a <= ``--prompt-tokens``
prompt, ``--max-tokens`` (AIProvider default 500) generated tokens at
temperature 0.3. Random-init weights (no checkpoints offline) => EOS is not
meaningful, so generation always runs to maxTokens (``ignore_eos``).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "pod-failure analyses/sec (whole node) + p50 explanation latency, 8B TP=1"


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, help="failures per GPU per step")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--max-tokens", type=int, default=500)
    ap.add_argument("--prompt-tokens", type=int, default=1024, help="prompt budget (tokens)")
    ap.add_argument("--log-kb", type=int, default=64)
    ap.add_argument("--patterns", type=int, default=1000)
    ap.add_argument("--max-batch", type=int, default=256, help="LLM continuous-batching width")
    ap.add_argument("--prefill-tokens", type=int, default=32768,
                    help="max tokens per prefill batch (16k / 32k / 64k: 27.9 / 28.2-28.4 / 28.0 analyses/s)")
    ap.add_argument("--mode", choices=["pipeline", "engine"], default="pipeline")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--serial-waves", action="store_true",
                    help="wait for every sink write of a wave before writing the next one")
    ap.add_argument("--kv-gb", type=float, default=None, help="KV-cache budget (default 96 GB on GPU, 1 GB on CPU)")
    ap.add_argument("--page-size", type=int, default=16, help="KV page size in tokens (engine.page_size)")
    ap.add_argument("--no-prefix-sharing", action="store_true",
                    help="prefill every prompt whole (engine.prefix_sharing off: no shared prompt-prefix pages)")
    ap.add_argument("--kv-dtype", choices=["auto", "fp8"], default="auto",
                    help="fp8: e4m3fn KV cache (reduced precision: not the headline configuration)")
    ap.add_argument("--engine-procs", type=int, default=1,
                    help="engine processes per GPU (EnginePool workers holding the scan + LLM engines, "
                         "--max-batch split over them); 1 = engines inside this process")
    ap.add_argument("--shards", type=int, default=None,
                    help="operator shards per GPU (default 1): independent operator "
                         "processes (own API-server shard, controller and engines), each failing --batch / shards "
                         "pods per step on its own closed loop; the rank process runs shard 0 and starts the "
                         "others as child processes")
    ap.add_argument("--shard-index", type=int, default=None, help=argparse.SUPPRESS)  # internal: child shard
    ap.add_argument("--multi-step", type=int, default=8, help="decode steps per graph window (engine.multi_step)")
    ap.add_argument("--admit-wait-ms", type=float, default=None,
                    help="idle engine: gather arrivals this long before a partial prefill (engine.admit_wait_ms)")
    ap.add_argument("--sink-concurrency", type=int, default=16,
                    help="operator.sink_concurrency: analyses writing results at once (0 = unbounded); a bound "
                         "keeps a finished wave's 256 result writers from starving the next wave's ramp "
                         "(GPU gap before its first prefill 230-440 -> 140-170 ms, profiles/wave_timeline_sinks_8b.jsonl)")
    ap.add_argument("--ranks-per-apiserver", type=int, default=4,
                    help="rest: ranks sharing one API server process (ranks g*R .. g*R+R-1 = the operator shards "
                         "of server g). One Python API server costs ~2.8 ms of CPU per analysis (~357/s), below "
                         "2x the ~260/s an 8-GPU node asks of it: 4 ranks per server keeps >= 2x headroom")
    ap.add_argument("--apiserver", choices=["auto", "inproc", "rest"], default="auto",
                    help="rest: ONE API server process (the REST FakeKube, kube/fake_server.py) that every rank's "
                         "operator shard talks to over HTTP, each rank owning the pods that hash to it "
                         "(`run --shard-per-gpu`); inproc: an in-memory FakeKube inside the rank process; "
                         "auto: rest when --gpus > 1")
    ap.add_argument("--handoff", choices=["generated", "explained"], default="generated",
                    help="pipelined waves: wave w+1 fails when wave w's explanations are generated (the "
                         "engine's finish hook) or once every pipeline thread has its explanation back")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--cpu", action="store_true",
                    help="CPU rehearsal (gloo, tiny models): allows --gpus N > 1 on a host without N GPUs")
    return ap.parse_args()


def launch_ranks(a) -> int:
    """``--gpus N`` with no outer torchrun (WORLD_SIZE unset): start N rank processes
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* on 127.0.0.1) as plain children of this
    process, which never touches the GPU itself (device_count() does not initialise HIP
    here, and nothing is exec'd). Rank 0 prints the JSON line on the inherited stdout;
    the exit code is the first non-zero rank exit code."""
    import socket
    import subprocess

    if not a.cpu:
        import torch

        have = torch.cuda.device_count()
        if have < a.gpus:
            print(f"bench.py: --gpus {a.gpus} needs {a.gpus} visible GPUs, found {have} "
                  "(--cpu for a gloo CPU rehearsal)", file=sys.stderr, flush=True)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    kids = []
    for r in range(a.gpus):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OAMD_BENCH_LAUNCHED="1")
        kids.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    for k in kids:
        c = k.wait()
        if c != 0 and rc == 0:
            rc = c
            for o in kids:   # one rank failed: the others would block in a collective
                if o.poll() is None:
                    o.terminate()
    return rc


SHARD_TAG = "OAMD_SHARD"  # protocol lines on a child shard's stdout


def spawn_shards(a) -> list:
    """Child shard processes 1..shards-1 of this rank, started before this process
    touches the GPU (plain child processes, no exec from a GPU-initialised process)."""
    import subprocess

    kids = []
    for i in range(1, a.shards):
        env = dict(os.environ)
        env.update(OAMD_BENCH_RANK=os.environ.get("RANK", "0"), OAMD_BENCH_WORLD=os.environ.get("WORLD_SIZE", "1"),
                   OAMD_BENCH_LOCAL=os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")),
                   WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
        kids.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *sys.argv[1:],
                                      "--shard-index", str(i)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                     env=env, text=True, bufsize=1))
    return kids


def shard_read(kid, what: str) -> str:
    """Next protocol line ``OAMD_SHARD <what> ...`` of a child shard (other stdout lines skipped)."""
    while True:
        line = kid.stdout.readline()
        if not line:
            raise SystemExit(f"shard process {kid.pid} exited (code {kid.poll()}) before {what}")
        if line.startswith(f"{SHARD_TAG} {what}"):
            return line[len(SHARD_TAG) + len(what) + 2:].strip()


def main() -> int:
    a = parse_args()
    child = a.shard_index is not None
    if not child and a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(a)
    if child:   # a child shard dies with its rank process (torchrun only signals its own workers)
        try:
            import ctypes
            import signal

            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGTERM))   # PR_SET_PDEATHSIG
        except OSError:
            pass
        if os.getppid() == 1:
            return 1
    if a.shards is None:
        # one operator per GPU: with every shard's logs equally heavy, 1 x 256 measured
        # 28.2 analyses/s at p50 9.0 s vs 26.6 / 9.5 s for 2 x 128 and 26.8 / 14.1 s for
        # 3 x 128 (profiles/shards_equal_work_8b.jsonl)
        a.shards = 1
    a.shards = max(1, a.shards)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rest = a.mode == "pipeline" and (a.apiserver == "rest" or (a.apiserver == "auto" and world_env > 1))
    if rest and a.shards > 1:
        raise SystemExit("--apiserver rest runs one operator shard per rank (no --shards)")
    apisrvs: list = []
    apiurls: list = []
    rpa = max(1, a.ranks_per_apiserver)
    if rest and int(os.environ.get("RANK", "0")) == 0:
        # the node's API servers (one per `rpa` ranks): their own processes, started before this
        # rank touches the GPU; the URLs reach the other ranks over the process group
        from operator_amd.kube.fake_server import spawn as spawn_apiserver

        for g in range(-(-world_env // rpa)):
            p_, u_ = spawn_apiserver(f"/tmp/oamd-bench-apiserver-{os.getpid()}-{g}.url")
            apisrvs.append(p_)
            apiurls.append(u_)
    kids = spawn_shards(a) if (a.shards > 1 and not child) else []
    shard = a.shard_index or 0
    a.batch = max(1, a.batch // a.shards)   # this shard's wave (--batch is per GPU, over all shards)
    a.max_batch = max(1, a.max_batch // a.shards)
    # host thread pools sized to this rank's share of the node (N ranks on one host):
    # the tokenizer's Rust pool and torch's intra-op pool default to every CPU each
    procs_on_host = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))) * a.shards
    share_cpus = max(2, min(16, (os.cpu_count() or 16) // procs_on_host))
    os.environ.setdefault("RAYON_RS_NUM_CPUS", str(share_cpus))
    import torch

    torch.set_num_threads(min(torch.get_num_threads(), share_cpus))
    import torch.distributed as dist

    from operator_amd.parallel.comm import init_from_env

    # OAMD_BENCH_SHARE_GPU=1: rehearsal of the multi-rank launch on a one-GPU box —
    # every rank on cuda:0, gloo for the timing collectives (RCCL refuses two ranks
    # on one device), KV budget split so the ranks fit one card. Not a scaling number.
    share = os.environ.get("OAMD_BENCH_SHARE_GPU") == "1"
    procs = max(1, a.engine_procs)
    if procs > 1 and a.mode != "pipeline":
        raise SystemExit("--engine-procs > 1 runs the operator pipeline (--mode pipeline)")

    from operator_amd.config import load_settings
    from operator_amd.patterns.synth import LogFactory, synthetic_library

    def settings(dev: str, max_batch: int, world_: int):
        on_gpu = procs * a.shards * (world_ if share else 1)   # operator / engine processes on this GPU
        # each holds 16 GB of weights and up to ~8 GB of prefill workspace beside its KV
        kv = a.kv_gb or (1.0 if dev == "cpu" else 96.0 / on_gpu if not share else max(8.0, 240.0 / on_gpu - 24))
        return load_settings(env={}, overrides={
            "engine.model": a.model, "engine.device": dev, "engine.max_batch": max_batch,
            "engine.max_prefill_tokens": a.prefill_tokens,
            "engine.max_context": a.prompt_tokens + a.max_tokens + 64, "engine.max_prompt_tokens": a.prompt_tokens,
            "engine.kv_cache_gb": kv, "engine.kv_dtype": a.kv_dtype, "engine.use_graphs": not a.no_graphs,
            "engine.ignore_eos": True,
            "engine.multi_step": a.multi_step, "engine.page_size": a.page_size,
            **({} if a.admit_wait_ms is None else {"engine.admit_wait_ms": a.admit_wait_ms}),
            "engine.prefix_sharing": not a.no_prefix_sharing,
            "engine.seed": 0, "health.enabled": False, "operator.workers": 2 * a.batch + 16, "operator.io_workers": 16,
            "operator.sink_concurrency": a.sink_concurrency,
            "patterns.cache_dir": f"/tmp/oamd-bench-{os.getpid()}", "services.match_max_batch": int(os.environ.get("OAMD_BENCH_MATCH_MAX_BATCH", "64")),
            "services.match_batch_wait_ms": float(os.environ.get("OAMD_BENCH_MATCH_WAIT_MS", "15"))})

    patset = synthetic_library(a.patterns, seed=0)
    pool = None
    t_pool = time.perf_counter()
    if procs > 1:
        # engine processes (spawned) start before this process touches the GPU; each
        # holds the scan DFA and its own copy of the model, and serves max_batch / procs
        from operator_amd.engine.pool import EnginePool

        world_env = int(os.environ.get("WORLD_SIZE", "1"))
        local_env = 0 if share else int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
        dev0 = f"cuda:{local_env}" if torch.cuda.device_count() > 0 else "cpu"
        pool = EnginePool(settings(dev0, max(1, a.max_batch // procs), world_env), patset, devices=[dev0] * procs)

    info = init_from_env(backend="gloo" if share else None)
    rank, world, local = info.rank, info.world, (0 if share else info.local_rank)
    if not child:
        # the job must really span --gpus ranks (one per GPU): a launch that silently
        # measured one GPU, or ranks sharing a device, is an error, not a data point
        pg_world = dist.get_world_size() if dist.is_initialized() else 1
        if pg_world != a.gpus or world != a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} but the process group has {pg_world} ranks")
        if info.backend == "nccl" and not share and torch.cuda.device_count() < world:
            raise SystemExit(f"bench.py: {world} RCCL ranks but only {torch.cuda.device_count()} GPUs")
    if child:   # a child shard: the parent rank's GPU, no process group of its own
        rank, local = int(os.environ["OAMD_BENCH_RANK"]), (0 if share else int(os.environ["OAMD_BENCH_LOCAL"]))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    dev = f"cuda:{local}" if torch.cuda.is_available() else "cpu"

    from operator_amd.controller.operator import Operator
    from operator_amd.engine.explain import ExplainEngine
    from operator_amd.engine.factory import build_llm
    from operator_amd.engine.match import MatchEngine
    from operator_amd.engine.pool import PoolExplainService, PoolMatchService
    from operator_amd.engine.service import LocalExplainService, LocalMatchService
    from operator_amd.kube.fake import FakeKube, failed_pod, running_pod
    from operator_amd.kube.resources import AIPROVIDERS, EVENTS, PODMORTEMS, PODS
    from operator_amd.utils.tracing import mark, trace_range

    s = settings(dev, a.max_batch, int(os.environ.get("OAMD_BENCH_WORLD", world)) if child else world)
    # rest: rank r talks to API server g = r // rpa and is operator shard r - g*rpa of that server's
    # group (run --shard-per-gpu against each server); a group's first rank creates its cluster state
    grp, grp0, grp_n = 0, 0, 1
    apiurl = None
    if rest:
        grp = rank // rpa
        grp0 = grp * rpa
        grp_n = min(rpa, world - grp0)
        s.operator.shard_count, s.operator.shard_index = grp_n, rank - grp0
        if world > 1:
            box = [apiurls]
            dist.broadcast_object_list(box, src=0)
            apiurls = box[0]
        apiurl = apiurls[grp]

    def note(msg: str) -> None:   # stage progress on stderr (the JSON line stays alone on stdout)
        tag = f"rank {rank}" + (f" shard {shard}" if a.shards > 1 else "")
        print(f"[bench {tag}] {msg}", file=sys.stderr, flush=True)

    if os.environ.get("OAMD_BENCH_STACKS_S"):   # debugging a stall: every thread's stack, then exit
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["OAMD_BENCH_STACKS_S"]), exit=True)

    # ---- engines (weights, DFA, graphs) : not timed ----
    note("init: patterns, weights, graphs" + (f" in {procs} engine processes" if pool else ""))
    t_init = time.perf_counter()
    meng = llm = ee = None
    if pool is not None:
        ready = pool.wait_ready(900)
        if ready < procs:
            raise SystemExit(f"only {ready} of {procs} engine processes started: {pool.health()}")
        t_init = t_pool
    else:
        meng = MatchEngine(patset, device=dev, seg_bytes=s.patterns.seg_bytes)
        model, kv, llm, tok = build_llm(s, device=dev)
        llm.warmup([b for b in llm.buckets if b <= a.max_batch])
        ee = ExplainEngine(llm, tok, model_id=a.model, max_prompt_tokens=a.prompt_tokens, ignore_eos=True)
        explainer = LocalExplainService(ee)
    init_s = time.perf_counter() - t_init
    note(f"init done in {init_s:.1f} s")

    def engine_stats() -> dict:
        """Prefill / decode token counters, prefill graph buckets and DFA size, summed
        over the engine processes (or read from the in-process engines)."""
        if pool is None:
            st = llm.stats
            return {"prefill_tokens": st.prefill_tokens, "decode_tokens": st.decode_tokens,
                    "prefill_graph_replays": st.prefill_graph_replays, "use_graphs": bool(llm.use_graphs),
                    "prefill_padded_tokens": st.prefill_padded_tokens, "prefill_eager": st.prefill_eager,
                    "prefix_hits": st.prefix_hits, "prefix_tokens": st.prefix_tokens, "prefix_builds": st.prefix_builds,
                    "decode_launch_s": st.decode_launch_s, "decode_wait_s": st.decode_wait_s,
                    "decode_windows": st.decode_windows, "decode_windows_ahead": st.decode_windows_ahead,
                    "no_pipeline": dict(st.no_pipeline),
                    "prefill_graph_buckets": sorted(getattr(llm, "_prefill_g", {})),
                    "dfa_states": getattr(meng, "dfa_states", None)}
        ws = pool.worker_stats()
        out = {k: sum(w["llm"].get(k, 0) for w in ws) for k in ("prefill_tokens", "decode_tokens", "prefill_graph_replays",
                                                                 "prefill_padded_tokens", "prefill_eager", "prefix_hits",
                                                                 "prefix_tokens", "prefix_builds")}
        out.update(use_graphs=all(w.get("use_graphs") for w in ws),
                   prefill_graph_buckets=sorted({b for w in ws for b in w.get("prefill_graph_buckets", [])}),
                   dfa_states=ws[0].get("dfa_states") if ws else None)
        return out

    fac = LogFactory(n_patterns=a.patterns, seed=100 * rank + shard)
    waves = a.warmup + a.steps
    logs = [fac.batch(a.batch, a.log_kb * 1024, n_failures=3, seed=1000 * rank + 100 * shard + w)[0]
            for w in range(waves)]

    lat: list[float] = []
    t_inject: dict[str, float] = {}
    done_ev = threading.Event()
    counter = {"n": 0, "target": 0, "outcomes": {}}
    lock = threading.Lock()

    if a.mode == "pipeline":
        if rest:
            from operator_amd.controller.failures import in_shard
            from operator_amd.kube.client import KubeClient, KubeConfig

            fk = KubeClient(KubeConfig(apiurl), 120.0)

            def set_log(name: str, text: bytes) -> None:
                st, _, body = fk.pool.request("PUT", f"/api/v1/namespaces/default/pods/{name}/log", text)
                if st >= 300:
                    raise SystemExit(f"log upload failed: {st} {body[:200]!r}")
        else:
            fk = FakeKube()
            set_log = lambda name, text: fk.set_log("default", name, text)  # noqa: E731
        if pool is not None:
            matcher, explainer = PoolMatchService(pool), PoolExplainService(pool)
        else:
            matcher = LocalMatchService(meng, max_batch=64, max_wait_ms=5.0)
        explained = {"n": 0}
        exp_cv = threading.Condition()

        def count_explained() -> None:
            with exp_cv:
                explained["n"] += 1
                exp_cv.notify_all()

        # The hand-off between pipelined waves is the moment a wave's explanations are
        # GENERATED: with the engine in this process, its finish hook (the batch's texts
        # detokenized) counts them, instead of each of the 256 pipeline threads after it
        # has woken up and built its response (~50 ms later at the end of a wave, under
        # the GIL). Pool engines: counted by the explainer wrapper as before.
        generated = {"n": 0, "on": False}
        if llm is not None and a.handoff == "generated":
            inner_hook = llm.finish_hook

            def finish_hook(reqs) -> None:
                if inner_hook is not None:
                    inner_hook(reqs)
                with exp_cv:
                    generated["n"] += len(reqs)
                    if generated["n"] >= generated.get("want", 0):
                        exp_cv.notify_all()

            llm.finish_hook = finish_hook
            generated["on"] = True
        non_ai = {"n": 0}   # failures that never reached the explainer (count toward a hand-off too)

        def handed() -> int:
            return (generated["n"] + non_ai["n"]) if generated["on"] else explained["n"]

        class CountingExplainer:
            """Counts generated explanations: the hand-off point between pipelined waves."""

            def __init__(self, inner):
                self.inner = inner

            def explain(self, result, cfg):
                try:
                    return self.inner.explain(result, cfg)
                finally:
                    count_explained()

            def ready(self):
                return self.inner.ready()

        op = Operator(fk, s, match_service=matcher, explain_service=CountingExplainer(explainer))
        if not rest or rank == grp0:   # cluster state, created once per API server
            fk.create(AIPROVIDERS, {"metadata": {"name": "local-llm", "namespace": "default"},
                                    "spec": {"providerId": "local", "modelId": a.model, "maxTokens": a.max_tokens,
                                             "temperature": 0.3, "cachingEnabled": False,
                                             "timeoutSeconds": 3600}})
            fk.create(PODMORTEMS, {"metadata": {"name": "bench-monitor", "namespace": "default"},
                                   "spec": {"podSelector": {"matchLabels": {"app": "bench"}},
                                            "aiAnalysisEnabled": True, "aiProviderRef": {"name": "local-llm"}}})
        if rest and world > 1:
            dist.barrier()

        def on_done(monitor, pod, outcome):
            name = pod["metadata"]["name"]
            if outcome not in ("ai-complete", "ai-failed"):   # never reached the explainer
                with exp_cv:
                    non_ai["n"] += 1
                count_explained()
            with lock:
                lat.append(time.perf_counter() - t_inject.get(name, time.perf_counter()))
                counter["n"] += 1
                counter["outcomes"][outcome] = counter["outcomes"].get(outcome, 0) + 1
                if counter["n"] >= counter["target"]:
                    done_ev.set()

        op.pipeline.listeners.append(on_done)
        op.start(http=False)
        while not op.monitors.list():
            time.sleep(0.01)

        # The pods (running, with their logs) exist before the benchmark, as in a cluster
        # where a pod runs for a while before it fails: creating them is cluster state,
        # not operator work, and is done here, untimed. A wave is the FAILURE of its
        # pods: each pod's status flips to a terminated, non-zero exit (the MODIFIED
        # watch event the operator reacts to), and its latency is timed from there.
        def shard_name(base: str) -> str:
            """``base`` or the first ``base-xJ`` whose ns/name hash puts it in this rank's
            shard (rest: every rank's pods are the failures its own operator shard owns)."""
            if not rest or grp_n <= 1:
                return base
            j, name = 0, base
            while not in_shard({"metadata": {"namespace": "default", "name": name}}, rank - grp0, grp_n):
                j += 1
                name = f"{base}-x{j}"
            return name

        names_by_wave = [[shard_name(f"app-r{rank}-s{shard}-w{w}-{i}") for i in range(a.batch)] for w in range(waves)]

        def wave_names(w: int) -> list[str]:
            return names_by_wave[w]

        for w in range(waves):
            for name, log in zip(wave_names(w), logs[w]):
                fk.create(PODS, running_pod(name, labels={"app": "bench"}))
                set_log(name, log)
        logs.clear()

        def inject(w: int) -> None:
            with trace_range(f"inject[{w}]"):
                for name in wave_names(w):
                    cur = fk.get(PODS, name, "default")
                    cur["status"] = failed_pod(name, finished_at=f"2025-08-29T10:{w % 60:02d}:00Z")["status"]
                    t_inject[name] = time.perf_counter()
                    fk.replace(PODS, cur)

        def run_wave(w: int) -> None:
            with lock:
                counter["n"], counter["target"] = 0, a.batch
                done_ev.clear()
            inject(w)
            done_ev.wait()
            op.drain(600)

        def run_timed(ws: list[int]) -> None:
            """Pipelined waves (default): wave w+1 is written to the API server as soon as
            every explanation of wave w has been generated, so its scan / prefill overlap
            wave w's result sinks (annotations, status ring, Events) instead of waiting
            behind them, as under a steady stream of failures. Every wave still completes
            (all analyses stored, kube writes drained) inside the timed region."""
            if a.serial_waves:
                for w in ws:
                    run_wave(w)
                return
            with lock:
                counter["n"], counter["target"] = 0, a.batch * len(ws)
                done_ev.clear()
            base = handed()
            for j, w in enumerate(ws):
                inject(w)
                if j + 1 < len(ws):
                    with exp_cv:
                        generated["want"] = base + (j + 1) * a.batch
                        exp_cv.wait_for(lambda: handed() >= base + (j + 1) * a.batch)
                    mark(f"handoff[{w}]")
            done_ev.wait()
            op.drain(600)
    else:
        from operator_amd.api.models import AIProviderConfig
        from operator_amd.controller.storage import pattern_annotation

        cfg = AIProviderConfig(provider_id="local", model_id=a.model, max_tokens=a.max_tokens, temperature=0.3,
                               caching_enabled=False, timeout_seconds=3600)

        def run_wave(w: int) -> None:
            t0 = time.perf_counter()
            res = meng.analyze(logs[w], [(f"app-{w}-{i}", "default") for i in range(a.batch)])
            outs = ee.explain_many([(r, cfg) for r in res])
            for r, o in zip(res, outs):
                _ = pattern_annotation(r) if isinstance(o, Exception) else o.explanation
                lat.append(time.perf_counter() - t0)
            counter["outcomes"]["ai-complete"] = counter["outcomes"].get("ai-complete", 0) + len(outs)

        def run_timed(ws: list[int]) -> None:
            for w in ws:
                run_wave(w)

    # a progress line on stderr every 30 s (stdout stays the ONE JSON line)
    prog_stop = threading.Event()

    def progress():
        t_start = time.perf_counter()
        while not prog_stop.wait(30.0):
            note(f"{time.perf_counter() - t_start:.0f} s, {counter['n']} analyses in the current pass")

    threading.Thread(target=progress, daemon=True).start()
    note(f"{a.warmup} warmup wave(s)")
    for w in range(a.warmup):
        run_wave(w)
    lat.clear()
    counter["outcomes"] = {}
    stats0 = engine_stats()

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if world > 1 and not child:
            dist.barrier()

    if child:   # a child shard: report ready, start on the parent's signal, report the timed pass
        print(f"{SHARD_TAG} READY", flush=True)
        if sys.stdin.readline().strip() != "GO":
            return 1
        mono0 = time.monotonic_ns()
        run_timed(list(range(a.warmup, waves)))
        sync()
        mono1 = time.monotonic_ns()
        prog_stop.set()
        st1 = engine_stats()
        print(f"{SHARD_TAG} RESULT " + json.dumps({
            "t0": mono0, "t1": mono1, "lat": lat, "outcomes": counter["outcomes"],
            "ptoks": st1["prefill_tokens"] - stats0["prefill_tokens"],
            "xtoks": st1.get("prefix_tokens", 0) - stats0.get("prefix_tokens", 0),
            "dtoks": st1["decode_tokens"] - stats0["decode_tokens"],
            "replays": st1["prefill_graph_replays"] - stats0["prefill_graph_replays"]}), flush=True)
        if a.mode == "pipeline":
            op.stop()
        if ee is not None:
            ee.close()
        if pool is not None:
            pool.close()
        return 0

    for k in kids:   # every shard of this rank initialised and warmed up
        shard_read(k, "READY")
    sync()
    note("timed waves")
    mono0 = time.monotonic_ns()  # same clock as rocprofv3 timestamps: lets a trace be cut to the timed region
    for k in kids:
        k.stdin.write("GO\n")
        k.stdin.flush()
    run_timed(list(range(a.warmup, waves)))
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    mono1 = time.monotonic_ns()
    results = [json.loads(shard_read(k, "RESULT")) for k in kids]
    for k in kids:
        k.wait(120)
    # the rank's timed pass: first shard start to last shard end (one host clock)
    t_first = min([mono0] + [r["t0"] for r in results])
    t_last = max([mono1] + [r["t1"] for r in results])
    if world > 1:
        dist.barrier()
    elapsed = (t_last - t_first) / 1e9
    prog_stop.set()
    for r in results:
        lat.extend(r["lat"])
        for o, n in r["outcomes"].items():
            counter["outcomes"][o] = counter["outcomes"].get(o, 0) + n

    # whole-job outcomes (every rank's analyses) and, with one API server, its own record of
    # them: every bench pod must carry exactly one PodmortemAnalysisComplete Event (each
    # failure analysed once, by exactly one operator shard). Untimed: after the timed pass.
    job_outcomes = dict(counter["outcomes"])
    if world > 1:
        allo: list = [None] * world
        dist.all_gather_object(allo, counter["outcomes"])
        job_outcomes = {}
        for d in allo:
            for o, n in d.items():
                job_outcomes[o] = job_outcomes.get(o, 0) + n
    audit = None
    if a.mode == "pipeline" and (rank == grp0 or not rest):
        per_pod: dict[str, int] = {}
        for ev in fk.list(EVENTS, "default"):
            reg = ev.get("regarding") or {}
            if ev.get("reason") == "PodmortemAnalysisComplete" and reg.get("kind") == "Pod" \
                    and reg.get("name", "").startswith("app-r"):
                per_pod[reg["name"]] = per_pod.get(reg["name"], 0) + 1
        counts = list(per_pod.values())
        audit = {"pods_with_complete_event": len(per_pod), "max_complete_events_per_pod": max(counts, default=0),
                 "expected_pods": a.batch * waves * (grp_n if rest else 1)}   # inproc: this process's shard
    if rest and world > 1:   # every API server's own record, merged (group leaders audited theirs)
        alla: list = [None] * world
        dist.all_gather_object(alla, audit)
        parts = [x for x in alla if x is not None]
        audit = {"pods_with_complete_event": sum(x["pods_with_complete_event"] for x in parts),
                 "max_complete_events_per_pod": max(x["max_complete_events_per_pod"] for x in parts),
                 "expected_pods": sum(x["expected_pods"] for x in parts), "apiservers": len(parts)}

    el = torch.tensor([elapsed], dtype=torch.float64, device=dev if info.backend == "nccl" else "cpu")
    p50_local = statistics.median(lat) if lat else float("nan")
    p50 = torch.tensor([p50_local], dtype=torch.float64, device=el.device)
    per_rank_s = [elapsed]
    if world > 1:
        allel = [torch.zeros_like(el) for _ in range(world)]
        dist.all_gather(allel, el)
        per_rank_s = [float(t.item()) for t in allel]
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(p50, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    total = a.batch * a.shards * a.steps * world
    value = total / elapsed
    stats1 = engine_stats()
    ptoks = stats1["prefill_tokens"] - stats0["prefill_tokens"] + sum(r["ptoks"] for r in results)
    # prompt tokens served from the shared prompt-prefix pages (computed once, not per request)
    xtoks = stats1.get("prefix_tokens", 0) - stats0.get("prefix_tokens", 0) + sum(r.get("xtoks", 0) for r in results)
    dtoks = stats1["decode_tokens"] - stats0["decode_tokens"] + sum(r["dtoks"] for r in results)
    replays = stats1["prefill_graph_replays"] - stats0["prefill_graph_replays"] + sum(r["replays"] for r in results)
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "analyses/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic pod logs (LogFactory) + random-init weights",
        "p50_explanation_latency_ms": round(float(p50.item()) * 1e3, 1),
        "config": {"model": a.model, "global_batch": a.batch * a.shards * world,
                   "seq_len": a.prompt_tokens + a.max_tokens,
                   "parallelism": f"dp{world}", "tp": 1, "max_tokens": a.max_tokens,
                   "prompt_tokens_cap": a.prompt_tokens, "log_kib": a.log_kb, "patterns": a.patterns,
                   "mode": a.mode, "hipgraph": stats1["use_graphs"], "engine_procs_per_gpu": procs,
                   "operator_shards_per_gpu": a.shards,
                   "kv_cache_dtype": "fp8_e4m3fn" if a.kv_dtype == "fp8" else "bf16",
                   "kv_page_tokens": a.page_size, "shared_prompt_prefix": not a.no_prefix_sharing,
                   "apiserver": (f"{-(-world // rpa)} REST API server process(es), {rpa} ranks each: rank r = "
                                 f"operator shard r % {rpa} of server r // {rpa} (run --shard-per-gpu)"
                                 if rest else "in-process FakeKube per rank"),
                   "waves": "serial" if (a.serial_waves or a.mode != "pipeline") else "pipelined",
                   "wave_handoff": a.handoff},
        "detail": {"init_s": round(init_s, 1), "prefill_tokens_per_gpu": ptoks, "decode_tokens_per_gpu": dtoks,
                   # workload check: every failure carries three signatures of the scanned library, so
                   # this stays ~885 whatever the rank / shard layout (README "Correction"); it counts
                   # the prompt tokens read from shared prompt-prefix pages too
                   "prompt_tokens_per_analysis": round((ptoks + xtoks) / max(1, a.batch * a.shards * a.steps), 1),
                   "shared_prefix": {"requests": stats1.get("prefix_hits", 0) - stats0.get("prefix_hits", 0),
                                     "prompt_tokens_not_prefilled": xtoks,
                                     "prefixes_computed": stats1.get("prefix_builds", 0) - stats0.get("prefix_builds", 0)},
                   "prefill_graph_replays": replays,
                   "prefill_graph_buckets": stats1["prefill_graph_buckets"],
                   "prefill_padded_tokens": stats1.get("prefill_padded_tokens", 0) - stats0.get("prefill_padded_tokens", 0),
                   "prefill_eager_batches": stats1.get("prefill_eager", 0) - stats0.get("prefill_eager", 0),
                   # host seconds inside decode graph launches (blocked = GPU queue full) / waiting on windows
                   "decode_launch_s": round(stats1.get("decode_launch_s", 0) - stats0.get("decode_launch_s", 0), 2),
                   "decode_wait_s": round(stats1.get("decode_wait_s", 0) - stats0.get("decode_wait_s", 0), 2),
                   "decode_windows": stats1.get("decode_windows", 0) - stats0.get("decode_windows", 0),
                   "decode_windows_ahead": stats1.get("decode_windows_ahead", 0) - stats0.get("decode_windows_ahead", 0),
                   "no_pipeline": stats1.get("no_pipeline", {}),
                   "decode_tok_s_per_gpu": round(dtoks / elapsed, 1), "outcomes": counter["outcomes"],
                   "outcomes_all_ranks": job_outcomes,
                   # the API server's Events (rest: the one server every rank used; warmup waves included)
                   "apiserver_audit": audit,
                   "dfa_states": stats1["dfa_states"], "timed_monotonic_ns": [mono0, mono1],
                   "rccl_world": dist.get_world_size() if dist.is_initialized() else 1,
                   "dist_backend": info.backend,
                   # the flagship is DP (tp = 1): no TP all-reduce to dispatch; tools/bench_tp.py reports the
                   # node-measured one-shot / two-shot / RCCL table (custom_ar.OneShotAllReduce.calibrate)
                   "allreduce_calibration": {"tp": 1, "table": None},
                   "launcher": "bench.py" if os.environ.get("OAMD_BENCH_LAUNCHED") else
                               ("torchrun" if world > 1 else "single"),
                   "per_rank_elapsed_s": [round(x, 3) for x in per_rank_s],
                   "per_rank_analyses_s": [round(a.batch * a.shards * a.steps / x, 3) for x in per_rank_s],
                   "host_max_rss_gb": {"rank": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2),
                                       "child_shards": round(resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss
                                                             / 2**20, 2)}},
    }
    if share:
        out["detail"]["shared_gpu_rehearsal"] = True
    if rank == 0:
        print(json.dumps(out), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(out, f, indent=1)
    if a.mode == "pipeline":
        op.stop()
        if rest:
            fk.close()
    if ee is not None:
        ee.close()
    if pool is not None:
        pool.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    for p_ in apisrvs:
        p_.terminate()
        p_.wait(30)
    return 0


if __name__ == "__main__":
    sys.exit(main())
