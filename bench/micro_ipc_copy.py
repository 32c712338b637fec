"""Cross-process KV shipping copy: shader-store kernel vs hipMemcpyAsync (copy engines) into an
IPC-mapped landing zone, two processes sharing the GPU.

Process 1 owns a 1 GiB landing zone (src.parallel.kv_transfer.IPCLandingZone); process 0 maps it
(IPCSender) and, for packet sizes of 16-256 MiB, times (a) the copy alone, (b) a bf16 GEMM loop
alone and (c) the GEMM loop while copies run on the sender's transfer stream — whichever copy
steals fewer CUs slows the concurrent compute less. One JSON line per (method, size)."""

import json
import os
import sys
import time

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def owner(q_handle, q_done):
    from src.parallel.kv_transfer import IPCLandingZone

    torch.cuda.set_device(0)
    z = IPCLandingZone("cuda:0", 1 << 30)
    q_handle.put((z.handle, z.capacity))
    q_done.get()
    z.close()


def gemm_loop(a, b, n):
    for _ in range(n):
        torch.mm(a, b)


def main():
    ctx = mp.get_context("spawn")
    qh, qd = ctx.Queue(), ctx.Queue()
    p = ctx.Process(target=owner, args=(qh, qd))
    p.start()
    handle, cap = qh.get(timeout=120)
    from src.parallel.kv_transfer import IPCSender

    torch.cuda.set_device(0)
    snd = IPCSender(handle, cap, "cuda:0")
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    gemm_loop(a, b, 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gemm_loop(a, b, 20)
    torch.cuda.synchronize()
    g_alone = (time.perf_counter() - t0) / 20
    for method in ("shader", "dma"):
        snd.dma = method == "dma"
        for mb in (16, 64, 256):
            kv = torch.randn(mb << 19, device="cuda").to(torch.bfloat16)  # mb MiB
            for _ in range(2):
                snd.write(0, kv).synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                ev = snd.write(0, kv)
            ev.synchronize()
            c_alone = (time.perf_counter() - t0) / 5
            # concurrent: copies on the transfer stream while the GEMM loop runs on the default stream
            torch.cuda.synchronize()
            n_copies = max(1, int(20 * g_alone / c_alone))
            t0 = time.perf_counter()
            for _ in range(n_copies):
                snd.write(0, kv)
            gemm_loop(a, b, 20)
            torch.cuda.current_stream().synchronize()
            g_with = (time.perf_counter() - t0) / 20
            torch.cuda.synchronize()
            print(json.dumps({"bench": "ipc_copy", "method": method, "mib": mb, "copy_ms": round(c_alone * 1e3, 3),
                              "copy_gbps": round((mb << 20) / c_alone / 1e9, 1),
                              "gemm_ms_alone": round(g_alone * 1e3, 3), "gemm_ms_with_copies": round(g_with * 1e3, 3),
                              "concurrent_copies": n_copies}), flush=True)
    snd.close()
    qd.put(1)
    p.join(60)


if __name__ == "__main__":
    main()
