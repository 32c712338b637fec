"""Microbenchmark: the one-shot IPC all-reduce (csrc/kernels/allreduce.hip) with two ranks sharing
ONE MI355X (the only topology a one-GPU box offers): the peers' "remote" buffers are then local HBM,
so this measures the kernel's fixed protocol cost (uncached staging copy, system-scope flag round
trip, rank-order reduction) — not xGMI bandwidth. Calls are captured in a hipGraph and replayed
back to back. Prints one JSON line per message size from rank 0.

    python bench/micro_allreduce.py
"""

import json
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SIZES_KIB = [16, 64, 256, 512, 1024, 4096]


def _worker(rank, world, port):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.parallel.custom_allreduce import CustomAllReduce

    car = CustomAllReduce(rank, world, max_bytes=8 << 20)
    iters = 50
    for kib in SIZES_KIB:
        n = kib * 1024 // 2
        x = torch.randn(n, device="cuda").to(torch.bfloat16)
        y = torch.empty_like(x)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                car.all_reduce(x, y)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                car.all_reduce(x, y)
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        t = torch.tensor([us])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            print(json.dumps({"bench": "custom_allreduce", "ranks": world, "topology": "2 procs on 1 GPU",
                              "kib": kib, "us": round(float(t), 2),
                              "algbw_gbs": round(kib * 1024 / float(t) / 1e3, 1)}), flush=True)
    assert not car.error()
    dist.barrier()
    car.close()
    dist.destroy_process_group()


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, 2, port)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    sys.exit(max(p.exitcode or 0 for p in ps))


if __name__ == "__main__":
    main()
