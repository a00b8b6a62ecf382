"""Host control messages of a single-node TP replica over shared memory.

``TPLLMEngine`` (engine/tp.py) replicates each engine step's submissions and
cancellations from the leader to every follower before the step runs: at a
2-4 ms decode step that message is on the critical path of every step. A gloo
``broadcast_object_list`` costs two collectives (size, then payload) plus a
pickle per rank; ``tools/bench_tp_ctrl.py`` measures both transports at world 8.

``ControlRing`` is one shared-memory slot that the leader writes and the
followers read, all on one host (a TP group never spans nodes here: TP=8 is
one MI355X node over xGMI):

* header: ``seq`` (messages published), ``length``, the leader's pid, and one
  64-byte line per follower holding the last ``seq`` it consumed;
* ``publish`` waits until every follower acknowledged the previous message
  (so the slot is free), writes the pickled payload, then its length, then
  bumps ``seq`` (x86 stores are seen in program order by other processes);
* ``receive`` spins on ``seq`` (tight for ~50 us, then yielding, then short
  sleeps so an idle follower does not burn a core), reads the payload and acks.

A message larger than the slot goes through the gloo group instead (the slot
then carries a marker). A follower whose leader process has exited raises
instead of waiting forever (the pool respawns the replica).
"""
from __future__ import annotations

import os
import pickle
import struct
import time
import uuid
from multiprocessing import resource_tracker, shared_memory

import torch.distributed as dist

_HDR_LINE = 64
_BIG = b"\x00__oamd_ring_big__"


class ControlRing:
    def __init__(self, shm: shared_memory.SharedMemory, rank: int, world: int, owner: bool, group=None,
                 src: int = 0):
        self.shm, self.rank, self.world, self.owner = shm, rank, world, owner
        self.group, self.src = group, src
        self.buf = shm.buf
        self.data_off = _HDR_LINE * (1 + world)
        self.cap = shm.size - self.data_off
        self.seq = 0   # messages this side has published / consumed

    # layout helpers -------------------------------------------------------------------------
    def _get(self, off: int) -> int:
        return struct.unpack_from("<Q", self.buf, off)[0]

    def _put(self, off: int, v: int) -> None:
        struct.pack_into("<Q", self.buf, off, v)

    @classmethod
    def create_for_group(cls, group, capacity: int = 8 << 20, name_hint: str = "ctrl") -> "ControlRing":
        """Collective over ``group`` (all ranks on this host): its first rank creates the
        segment and broadcasts the name over the group; the others attach."""
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
        me = dist.get_rank()
        grank = ranks.index(me)
        world = len(ranks)
        box = [None]
        shm = None
        if grank == 0:
            shm = shared_memory.SharedMemory(create=True, size=_HDR_LINE * (1 + world) + capacity,
                                             name=f"oamd_{name_hint}_{os.getpid()}_{uuid.uuid4().hex[:8]}")
            shm.buf[:_HDR_LINE * (1 + world)] = bytes(_HDR_LINE * (1 + world))
            struct.pack_into("<Q", shm.buf, 16, os.getpid())
            box = [shm.name]
        dist.broadcast_object_list(box, src=ranks[0], group=group)
        if grank != 0:
            shm = shared_memory.SharedMemory(name=box[0])
            # attached, not owned: keep Python's resource tracker from unlinking the
            # leader's segment when this process exits
            try:
                resource_tracker.unregister(shm._name, "shared_memory")   # noqa: SLF001
            except Exception:
                pass
        return cls(shm, grank, world, grank == 0, group=group, src=ranks[0])

    # leader ---------------------------------------------------------------------------------
    def publish(self, msg):
        """Leader: hand ``msg`` to every follower; returns ``msg``."""
        payload = pickle.dumps(msg, protocol=pickle.HIGHEST_PROTOCOL)
        big = len(payload) > self.cap
        self._wait(lambda: all(self._get(_HDR_LINE * (1 + f)) >= self.seq for f in range(1, self.world)))
        body = _BIG if big else payload
        self.buf[self.data_off:self.data_off + len(body)] = body
        self._put(8, len(body))
        self.seq += 1
        self._put(0, self.seq)
        if big:   # followers read the marker, then join this broadcast
            dist.broadcast_object_list([msg], src=self.src, group=self.group)
        return msg

    # follower -------------------------------------------------------------------------------
    def receive(self):
        """Follower: the next message the leader published."""
        want = self.seq + 1
        self._wait(lambda: self._get(0) >= want, check_leader=True)
        n = self._get(8)
        body = bytes(self.buf[self.data_off:self.data_off + n])
        self.seq = want
        self._put(_HDR_LINE * (1 + self.rank), self.seq)
        if body == _BIG:
            box = [None]
            dist.broadcast_object_list(box, src=self.src, group=self.group)
            return box[0]
        return pickle.loads(body)

    def _wait(self, ready, check_leader: bool = False) -> None:
        t0 = time.perf_counter()
        spins = 0
        next_check = t0 + 1.0
        while not ready():
            spins += 1
            if spins < 2000:
                continue
            now = time.perf_counter()
            if now - t0 < 0.002:
                time.sleep(0)
            else:
                time.sleep(5e-5 if now - t0 < 0.05 else 5e-4)
            if check_leader and now > next_check:
                next_check = now + 1.0
                pid = self._get(16)
                try:
                    os.kill(pid, 0)
                except ProcessLookupError:
                    raise RuntimeError(f"TP control ring: leader process {pid} exited") from None
                except PermissionError:
                    pass

    def close(self) -> None:
        try:
            self.buf = None
            self.shm.close()
            if self.owner:
                self.shm.unlink()
        except (FileNotFoundError, BufferError):
            pass
