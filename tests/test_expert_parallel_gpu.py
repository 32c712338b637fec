"""All-to-all expert parallelism on the HIP MoE kernels: two ranks share the MI355X (gloo group,
the all-to-all staged through the host), bf16 experts run by ops.moe_apply (align / gather /
grouped GEMM / combine kernels); each rank's output must match the fp32 single-process MoE over
all experts within bf16 tolerance, in both exchange forms."""

import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

E, H, I, K = 8, 256, 512, 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _weights():
    g = torch.Generator().manual_seed(7)
    router = torch.randn(E, H, generator=g)
    w13 = torch.randn(E, 2 * I, H, generator=g) / H ** 0.5
    w2 = torch.randn(E, H, I, generator=g) / I ** 0.5
    return router, w13, w2


def _tokens(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(24 + 5 * rank, H, generator=g)


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.parallel.expert_parallel import ep_moe_forward

        router, w13, w2 = _weights()
        el = E // world
        dev, bf = "cuda", torch.bfloat16
        w13_l = w13[rank * el:(rank + 1) * el].to(dev, bf).contiguous()
        w2_l = w2[rank * el:(rank + 1) * el].to(dev, bf).contiguous()
        x = _tokens(rank).to(dev, bf)
        r = router.to(dev, bf)
        exact = ep_moe_forward(x, r, w13_l, w2_l, K, capacity=None)
        padded = ep_moe_forward(x, r, w13_l, w2_l, K, capacity=(24 + 5 * (world - 1)) * K)
        torch.cuda.synchronize()
        q.put((rank, exact.float().cpu().numpy(), padded.float().cpu().numpy()))  # by value (see the CPU test)
    finally:
        dist.destroy_process_group()


def test_ep_all_to_all_on_gpu_kernels():
    import torch.multiprocessing as mp

    from src.ops import reference as ref

    world = 2
    router, w13, w2 = _weights()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (a, b)) for r, a, b in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    bf = torch.bfloat16
    for r in range(world):
        x = _tokens(r).to(bf).float()
        w13b, w2b = w13.to(bf).float(), w2.to(bf).float()
        # the same bf16 gating GEMM as the ranks ran (identical routing, no near-tie flips)
        gating = torch.nn.functional.linear(_tokens(r).to("cuda", bf), router.to("cuda", bf)).float().cpu()
        want = ref.moe_forward(x, w13b, w2b, gating, K)
        for out in got[r]:
            torch.testing.assert_close(torch.from_numpy(out), want, rtol=5e-2, atol=5e-2)
