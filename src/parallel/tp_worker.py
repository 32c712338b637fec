"""
Tensor-parallel worker group: ``torchrun --nproc-per-node T -m src.parallel.tp_worker ...``.

Rank 0 serves the worker RPC API (same wire format as ``src/worker.py``) on
top of a TP engine; ranks 1..T-1 mirror its steps (``follower_loop``). The
group appears to the coordinator as ONE worker / one shard — a TP group fails
as a unit (BASELINE config 4: Llama-3-70B, TP=8 over RCCL/xGMI).
"""

from __future__ import annotations

import asyncio
import os
import sys

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from src.config import ModelConfig  # noqa: E402
from src.parallel.tp import init_tp  # noqa: E402
from src.parallel.tp_runner import build_tp_engine  # noqa: E402
from src.utils import setup_logging  # noqa: E402
from src.worker import Worker, build_arg_parser  # noqa: E402


async def serve(args, engine) -> None:
    from src.engine.backend import LLMBackend, engine_config_from  # noqa: F401

    cfg = ModelConfig(model_name=args.model, model_path=args.model_path, max_batch_size=args.max_batch_size,
                      arch=args.arch, preset=args.preset, tp_size=args.tp_size, role=args.role,
                      max_model_len=args.max_model_len, max_latency_ms=args.max_latency_ms)
    worker = Worker(args.worker_id or f"tp-worker-{os.getpid()}", host=args.host, port=args.port,
                    coordinator=args.coordinator, metadata={"tp_size": args.tp_size, "role": args.role})
    worker.models[args.model] = LLMBackend(cfg, engine=engine)
    port = await worker.start()
    if args.port_file:
        with open(args.port_file + ".tmp", "w") as f:
            f.write(str(port))
        os.replace(args.port_file + ".tmp", args.port_file)
    print(f"TP worker (tp={args.tp_size}) listening on {port}", flush=True)
    await worker.wait_closed()


def main(argv=None) -> None:
    setup_logging()
    args = build_arg_parser().parse_args(argv)
    if args.arch == "mock":
        args.arch = "llama"
    tp = init_tp(args.tp_size, timeout_s=300)  # idle leaders send heartbeats (tp_runner.HEARTBEAT_S)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = f"cuda:{local}" if torch.cuda.is_available() else "cpu"
    from src.engine.backend import engine_config_from

    mcfg = ModelConfig(model_name=args.model, model_path=args.model_path, max_batch_size=args.max_batch_size,
                       arch=args.arch, preset=args.preset, max_model_len=args.max_model_len,
                       max_latency_ms=args.max_latency_ms, use_cuda_graph=not args.no_graph)
    obj = build_tp_engine(args.preset or "llama3-70b", tp, device, cfg=engine_config_from(mcfg),
                          max_model_len=args.max_model_len, capture=not args.no_graph,
                          moe_parallel=args.moe_parallel, sequence_parallel=args.sequence_parallel)
    if tp.rank == 0:
        try:
            asyncio.run(serve(args, obj))
        finally:
            obj.runner.stop_followers()
    else:
        obj.follower_loop()


if __name__ == "__main__":
    main()
