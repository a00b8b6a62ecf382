"""Tensor-parallel serving: one LLM engine replica spread over the ranks of a
TP group (BASELINE config 5 "Llama-3-70B, TP=8 over xGMI").

Every rank holds a column/row shard of the model (models/llama.py) and must
run the SAME engine steps on the SAME requests: each step's forward has 2
all-reduces per layer plus the vocab-parallel sampler's all-gather, so a rank
that admitted a different batch would deadlock or corrupt the collectives.

Scheduling in ``LLMEngine`` is deterministic given the order of submissions
and cancellations relative to steps, so only those need to be replicated:

* the **leader** (TP rank 0) owns request intake. ``submit``/``cancel`` from
  any thread only queue; at the top of each ``step`` the leader broadcasts the
  queued submissions (prompt + sampling params) and cancellations over a small
  gloo control group, applies them to its own engine, and steps;
* each **follower** blocks in ``follow()``: receive the step's control message,
  apply it identically (same request ids by construction), step; a ``None``
  message ends the loop.

Tokens need no broadcast: the sampler already agrees across ranks (global
max over vocab shards), so every rank appends the same tokens and retires the
same requests. The leader steps only when it has work, so idle followers just
wait in the broadcast. Device-side collectives (RCCL, or the one-shot IPC
all-reduce of parallel/custom_ar.py for decode-size messages) run inside the
captured decode graphs exactly as at TP=1.
"""
from __future__ import annotations

import threading

import numpy as np
import torch.distributed as dist

from .llm import GenRequest, LLMEngine


def encode_submit(r: GenRequest) -> tuple:
    """A submission as a control-message entry: the prompt as packed int32 bytes (one
    buffer to pickle instead of ~1k Python ints: 256 prompts cost ~0.3 ms, not ~6 ms)."""
    return ("s", np.asarray(r.prompt, dtype=np.int32).tobytes(), r.max_tokens, r.temperature, r.seed, r.ignore_eos)


def decode_submit(m: tuple) -> GenRequest:
    return GenRequest(np.frombuffer(m[1], dtype=np.int32).tolist(), max_tokens=m[2], temperature=m[3], seed=m[4],
                      ignore_eos=m[5])


class _FatalTPError(RuntimeError):
    fatal = True


def control_group(tp_group):
    """A gloo group over the TP ranks for host-side control messages."""
    ranks = getattr(tp_group, "ranks", None)
    return dist.new_group(ranks=ranks, backend="gloo")


class TPLLMEngine(LLMEngine):
    def __init__(self, *args, tp_group=None, ctrl_group=None, ctrl_transport: str = "shm", **kw):
        """``ctrl_transport``: "shm" (default: the per-step control message through a
        shared-memory slot, parallel/shm_ring.py -- ~8 us per step at world 8 against
        ~1 ms for a gloo broadcast_object_list, tools/bench_tp_ctrl.py) or "gloo".
        Constructing a TP engine is collective over ``ctrl_group``."""
        super().__init__(*args, **kw)
        self.tp_group = tp_group
        self.ctrl = ctrl_group
        self.ring = None
        if ctrl_transport not in ("shm", "gloo"):
            raise ValueError(f"ctrl_transport {ctrl_transport!r}")
        if ctrl_transport == "shm" and tp_group is not None and tp_group.world > 1:
            from operator_amd.parallel.shm_ring import ControlRing

            self.ring = ControlRing.create_for_group(ctrl_group, name_hint="tp")
        self.leader = tp_group is None or tp_group.rank == 0
        self._src = tp_group.ranks[0] if tp_group is not None else 0
        self._pending: list[GenRequest] = []
        self._cancels: list[GenRequest] = []
        self._by_rid: dict[int, GenRequest] = {}
        self._qlock = threading.Lock()
        self.closed = False
        car = getattr(tp_group, "oneshot", None)
        if car is not None:   # a timed-out one-shot all-reduce fails the replica (NaN output, never partial sums)
            self.health_checks.append(car.check)

    # ------------------------------------------------------------------ leader API
    def submit(self, req: GenRequest) -> GenRequest:
        if not self.leader:
            raise RuntimeError("requests are submitted to the TP leader (rank 0) only")
        if not req.prompt:
            raise ValueError("empty prompt")
        if len(req.prompt) >= self.max_context:
            raise ValueError(f"prompt of {len(req.prompt)} tokens exceeds max_context {self.max_context}")
        with self._qlock:
            self._pending.append(req)
        return req

    def cancel(self, req: GenRequest) -> None:
        with self._qlock:
            if req in self._pending:   # never broadcast: drop locally
                self._pending.remove(req)
                req.done, req.error = True, "cancelled"
                req.event.set()
                return
            self._cancels.append(req)

    def has_work(self) -> bool:
        return bool(self._pending or self._cancels) or super().has_work()

    def queued_prompt_tokens(self) -> int:
        with self._qlock:
            n = sum(len(r.prompt) for r in self._pending)
        return n + super().queued_prompt_tokens()

    def step(self) -> list[GenRequest]:
        if not self.leader:
            raise RuntimeError("TP followers step from follow()")
        with self._qlock:
            new, canc = self._pending, self._cancels
            self._pending, self._cancels = [], []
        msg = [encode_submit(r) for r in new] + [("c", r.rid) for r in canc]
        self._bcast(msg)
        self._apply(msg, new)
        try:
            return self._step_and_forget()
        except BaseException as e:
            # A step that failed on this rank only (OOM, a kernel error) leaves the peers
            # inside the same step's collectives, or one step ahead of a leader that would
            # abort and prefill a fresh batch: RCCL has no device-side timeout, so a
            # local abort_all could hang the replica. Every TP step error is fatal: the
            # replica stops and the pool respawns it.
            if self.tp_group is not None and self.tp_group.world > 1:
                try:
                    e.fatal = True
                except AttributeError:
                    raise _FatalTPError(str(e)) from e
            raise

    def close(self) -> None:
        """Release the followers (collective over the control group)."""
        if self.leader and not self.closed and self.tp_group is not None and self.tp_group.world > 1:
            self._bcast(None)
        self.closed = True
        if self.ring is not None and self.leader:
            self.ring.close()

    # ------------------------------------------------------------------ follower loop
    def follow(self) -> None:
        if self.leader:
            raise RuntimeError("the TP leader does not follow")
        while True:
            msg = self._bcast(None)
            if msg is None:
                self.closed = True
                if self.ring is not None:
                    self.ring.close()
                return
            self._apply(msg, None)
            self._step_and_forget()

    # ------------------------------------------------------------------ shared
    def _bcast(self, msg):
        if self.tp_group is None or self.tp_group.world == 1:
            return msg
        if self.ring is not None:
            return self.ring.publish(msg) if self.leader else self.ring.receive()
        box = [msg]
        dist.broadcast_object_list(box, src=self._src, group=self.ctrl)
        return box[0]

    def _apply(self, msg, reqs: list[GenRequest] | None) -> None:
        it = iter(reqs or [])
        for m in msg:
            if m[0] == "s":
                r = next(it) if self.leader else decode_submit(m)
                LLMEngine.submit(self, r)
                self._by_rid[r.rid] = r
            else:
                r = self._by_rid.get(m[1])
                if r is not None:
                    LLMEngine.cancel(self, r)
                    r.cancelled = True
                    if r.done:   # was still waiting: never reaped
                        self._by_rid.pop(r.rid, None)

    def _step_and_forget(self) -> list[GenRequest]:
        fin = LLMEngine.step(self)
        for r in fin:
            self._by_rid.pop(r.rid, None)
        return fin
