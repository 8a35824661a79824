"""Cost of the per-optimiser-step gradient all-reduce (BaseModel._dp_sync) through RCCL on the
devices of this box: one in-place all_reduce(SUM) of the fluid (533 KB) and el3D (1.32 MB)
gradient arenas, timed with HIP events over R back-to-back calls.  With one GPU this is the
world-1 cost (launch + RCCL's local path), the floor under the 8-rank ring on xGMI.

    python -m torch.distributed.run --nproc-per-node K tools/allreduce_cost.py
"""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
    dist.init_process_group("nccl", rank=rank, world_size=world)
    out = {"world_size": world}
    for name, floats in (("fluid_arena_533KB", 533 * 1024 // 4), ("el3d_arena_1.32MB", 1320 * 1024 // 4)):
        t = torch.ones(floats, device="cuda")
        for _ in range(20):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 200
        e0.record()
        for _ in range(reps):
            dist.all_reduce(t)
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
    if rank == 0:
        print(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
