"""Expert parallelism with all-to-all dispatch (src/parallel/expert_parallel.py) on CPU (gloo,
2 and 4 ranks): every rank routes its OWN tokens (different counts per rank), ships each
assignment to the rank owning the expert, and must get back exactly what the single-process MoE
with all experts computes — in both exchange forms (static capacity, graph-capturable; exact
counts, eager) — and the capacity form must drop (weight 0) exactly the assignments past C."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

E, H, I, K = 8, 64, 96, 2


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
    return torch.randn(5 + 3 * rank, H, generator=g)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.parallel.expert_parallel import ep_moe_forward

        router, w13, w2 = _weights()
        el = E // world
        w13_l, w2_l = w13[rank * el:(rank + 1) * el], w2[rank * el:(rank + 1) * el]
        x = _tokens(rank)
        exact = ep_moe_forward(x, router, w13_l, w2_l, K, capacity=None)
        tmax = 5 + 3 * (world - 1)
        padded = ep_moe_forward(x, router, w13_l, w2_l, K, capacity=tmax * K)
        tight = ep_moe_forward(x, router, w13_l, w2_l, K, capacity=2)
        # numpy arrays pickle by value: a tensor would travel as a shared-memory fd that vanishes
        # when this process exits before the parent has read it
        q.put((rank, exact.numpy(), padded.numpy(), tight.numpy()))
    except Exception as e:  # surface the failure in the parent instead of a queue timeout
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_ep_all_to_all_matches_single_process(world):
    from src.ops import reference as ref

    router, w13, w2 = _weights()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (a, b, c)) for r, a, b, c in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(60)
    for r in range(world):
        assert not isinstance(got[r][0], str), got[r][0]
    assert all(p.exitcode == 0 for p in procs)
    for r in range(world):
        x = _tokens(r)
        want = ref.moe_forward(x, w13, w2, x @ router.t(), K)
        exact, padded, tight = (torch.from_numpy(a) for a in got[r])
        torch.testing.assert_close(exact, want, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(padded, want, rtol=1e-5, atol=1e-5)
        # capacity 2 per destination: assignments past the first two (in token order) are dropped
        w, ids = ref.topk_softmax(x @ router.t(), K)
        el = E // world
        dest = (ids.long() // el).reshape(-1)
        seen = [0] * world
        keep = torch.zeros(dest.numel(), dtype=torch.bool)
        for j, d in enumerate(dest.tolist()):
            keep[j] = seen[d] < 2
            seen[d] += 1
        wk = torch.where(keep.view(ids.shape), w, torch.zeros_like(w))
        want_t = ref.moe_experts(x, w13, w2, wk, ids)
        torch.testing.assert_close(tight, want_t, rtol=1e-5, atol=1e-5)
