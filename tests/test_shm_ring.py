"""parallel/shm_ring.py: the TP replica's per-step control messages through one shared
memory slot, at gloo world 4 (processes of one host): every follower receives every
message in order, including one larger than the slot (sent through gloo behind a
marker) and the None that ends a follower loop; a follower whose leader is gone fails
instead of waiting forever."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from operator_amd.parallel.shm_ring import ControlRing

    ring = ControlRing.create_for_group(dist.group.WORLD, capacity=4096, name_hint="t")
    msgs = [[], [("s", b"\x01\x02", 5, 0.3, 7, True)], list(range(5000)), {"k": "v" * 10}, None]
    got = []
    for m in msgs:
        got.append(ring.publish(m) if rank == 0 else ring.receive())
    dist.barrier()
    ring.close()
    q.put((rank, got == msgs))
    dist.destroy_process_group()


def test_ring_delivers_every_message_in_order():
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    assert res == {r: True for r in range(world)}


def test_follower_fails_when_leader_is_gone():
    """A segment whose recorded leader pid does not exist: receive raises within ~1 s."""
    import struct
    from multiprocessing import shared_memory

    from operator_amd.parallel.shm_ring import ControlRing

    shm = shared_memory.SharedMemory(create=True, size=64 * 3 + 1024)
    try:
        shm.buf[:64 * 3] = bytes(64 * 3)
        struct.pack_into("<Q", shm.buf, 16, 2 ** 22 + 12345)   # no such pid
        ring = ControlRing(shm, rank=1, world=2, owner=False)
        with pytest.raises(RuntimeError, match="leader process"):
            ring.receive()
    finally:
        shm.close()
        shm.unlink()
