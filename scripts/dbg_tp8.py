"""Debug: the TP engine with N ranks sharing one GPU (gloo step protocol, IPC exchange), configurable decode window;
prints the leader's time per generate and the group's error word. Not a test (round-6 bisect of the 8-rank case)."""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker(rank, world, port, window, q):
    from src.config import EngineConfig
    from src.parallel.tp import TPContext
    from src.parallel.tp_runner import build_tp_engine
    from src.preproc import SamplingParams

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPContext(rank=rank, world_size=world)
    cfg = EngineConfig(max_num_seqs=4, max_num_batched_tokens=256, num_kv_blocks=128, max_latency_ms=0.0,
                       use_cuda_graph=True, graph_batch_sizes=[1, 2, 4], decode_window=window)
    obj = build_tp_engine("llama-mini", tp, "cuda:0", cfg=cfg, max_model_len=512, capture=True, full_init=True, seed=3)
    if rank == 0:
        obj.eos_token_id = None
        plan = obj.model.decode_plan(4)
        print("plan", {k: plan[k] for k in ("o", "down", "tp_fused", "o_half", "down_half")}, flush=True)
        for it in range(2):
            t0 = time.perf_counter()
            outs = obj.generate([[5, 9, 33, 12, 7] * 9, [100, 200, 300], list(range(3, 140))],
                                SamplingParams(max_tokens=8))
            torch.cuda.synchronize()
            print("generate", it, round(time.perf_counter() - t0, 3), "s", "err", tp.car.error(),
                  "windows", obj.runner.windows_synced, flush=True)
        t0 = time.perf_counter()
        obj.generate([[5, 9, 33, 12, 7] * 9, [100, 200, 300], list(range(3, 140))],
                     SamplingParams(max_tokens=12, temperature=0.9, top_k=40, top_p=0.9, seed=11))
        torch.cuda.synchronize()
        print("sampled", round(time.perf_counter() - t0, 3), "s", "err", tp.car.error(), flush=True)
        obj.runner.stop_followers()
        torch.cuda.synchronize()
        q.put((0, outs))
    else:
        obj.follower_loop()
        print("follower", rank, "stopped", flush=True)
        torch.cuda.synchronize()
        q.put((rank, obj.d_tokens.cpu()))
    dist.destroy_process_group()


if __name__ == "__main__":
    world, window = int(sys.argv[1]), int(sys.argv[2])
    if len(sys.argv) > 3 and sys.argv[3] == "parentcuda":  # the pytest parent holds a context (earlier tests)
        keep = torch.zeros(1 << 20, device="cuda")
        torch.cuda.synchronize()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, window, q)) for r in range(world)]
    for p in ps:
        p.start()
    for _ in range(world):
        r, v = q.get(timeout=120)
        print("got", r, flush=True)
    for p in ps:
        p.join(30)
        print("joined", p.exitcode, flush=True)
