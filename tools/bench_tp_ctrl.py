"""TP control-plane cost: the per-engine-step control message of TPLLMEngine (engine/tp.py)
at gloo world W on one host -- an empty step message (the decode steady state) and a
submission of 256 prompts (a prefill admission) -- for the gloo broadcast_object_list
path and the shared-memory ring (parallel/shm_ring.py). One JSON line per (transport,
message) on rank 0.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_tp_ctrl.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.distributed as dist  # noqa: E402


def main() -> int:
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from operator_amd.parallel.shm_ring import ControlRing

    ring = ControlRing.create_for_group(dist.group.WORLD, name_hint="ctrlbench")
    from operator_amd.engine.llm import GenRequest
    from operator_amd.engine.tp import encode_submit

    msgs = {"empty": [],
            "submit256": [encode_submit(GenRequest(list(range(900)), max_tokens=500, temperature=0.3, seed=i,
                                                   ignore_eos=True)) for i in range(256)]}
    iters = {"empty": 2000, "submit256": 50}
    for transport in ("gloo", "shm"):
        for kind, msg in msgs.items():
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters[kind]):
                if transport == "gloo":
                    box = [msg if rank == 0 else None]
                    dist.broadcast_object_list(box, src=0)
                    got = box[0]
                else:
                    got = ring.publish(msg) if rank == 0 else ring.receive()
                assert len(got) == len(msg)
            dt = (time.perf_counter() - t0) / iters[kind] * 1e6
            t = [dt]
            allt = [None] * world
            dist.all_gather_object(allt, t)
            if rank == 0:
                print(json.dumps({"transport": transport, "message": kind, "world": world,
                                  "us_per_step_max_rank": round(max(x[0] for x in allt), 1),
                                  "us_per_step_leader": round(dt, 1)}), flush=True)
    ring.close()
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
