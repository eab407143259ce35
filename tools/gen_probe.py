"""How long the fan-in generator takes with several ranks on one GPU (the full-size gloo rehearsal):
concurrent on every rank, then rank by rank behind barriers.  torchrun --nproc-per-node N tools/gen_probe.py T [serial,concurrent]"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd.workload import gen_fanin  # noqa: E402

total = int(sys.argv[1])
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
torch.cuda.set_device(0)
for mode in (sys.argv[2] if len(sys.argv) > 2 else "serial,concurrent").split(","):
    dist.barrier()
    t0 = time.time()
    for r in range(world):
        if mode == "concurrent" or r == rank:
            ts = time.time()
            wl = gen_fanin(total=total, R=1024, K=1 << 28, n_local=1 << 27, s=0.8, device="cuda", rank=rank,
                           world=world, route=True, census=True)
            torch.cuda.synchronize()
            print(f"[probe] {mode} rank {rank}: {time.time() - ts:.1f}s", file=sys.stderr, flush=True)
            del wl
            torch.cuda.empty_cache()
        if mode == "serial":
            dist.barrier()
        else:
            break
    dist.barrier()
    if rank == 0:
        print(f"[probe] {mode}: all ranks {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
dist.destroy_process_group()
