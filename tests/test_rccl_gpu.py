"""The RCCL branches of TPContext on a real GPU: a ONE-rank "nccl" (= RCCL on ROCm) process group with
the collectives forced on, so that every RCCL call the TP=8 path makes (all_reduce above the one-shot
size, reduce_scatter_rows, all_gather_rows, all_gather_last, broadcast) runs with the engine's shapes and
dtypes. A one-GPU box cannot show xGMI traffic; this pins the calls themselves."""

import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rccl_worker(port, q):
    try:
        import torch.distributed as dist

        from src.parallel.tp import TPContext

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        assert dist.get_backend() == "nccl"
        tp = TPContext(rank=0, world_size=1, force_collectives=True)
        assert tp.enabled and tp.car is None
        res = {}
        g = torch.Generator(device="cuda").manual_seed(1)
        # prefill-sized all-reduce (70B TP=8: [T, 8192] bf16) -> dist.all_reduce
        x = torch.randn(2048, 8192, device="cuda", generator=g).to(torch.bfloat16)
        y = tp.all_reduce(x.clone())
        res["all_reduce"] = bool(torch.equal(y, x)) and y.dtype == torch.bfloat16
        # sequence parallel halves -> reduce_scatter_tensor / all_gather_into_tensor
        rs = tp.reduce_scatter_rows(x)
        res["reduce_scatter_rows"] = tuple(rs.shape) == (2048, 8192) and bool(torch.equal(rs, x))
        ag = tp.all_gather_rows(x[:100])
        res["all_gather_rows"] = tuple(ag.shape) == (100, 8192) and bool(torch.equal(ag, x[:100]))
        # vocab-parallel logits (prefill size: above the one-shot gather) -> all_gather_into_tensor + permute
        lg = torch.randn(64, 16032, device="cuda", generator=g).to(torch.bfloat16)
        al = tp.all_gather_last(lg)
        res["all_gather_last"] = tuple(al.shape) == (64, 16032) and bool(torch.equal(al, lg))
        # step-protocol payload broadcast (int64 over RCCL)
        pk = torch.arange(777, dtype=torch.int64, device="cuda")
        res["broadcast"] = bool(torch.equal(tp.broadcast(pk.clone()), pk))
        # the same calls captured in a hipGraph (RCCL collectives are graph-capturable)
        s = torch.cuda.Stream()
        xin = torch.ones(32, 8192, device="cuda", dtype=torch.bfloat16)
        with torch.cuda.stream(s):
            tp.all_reduce(xin)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            tp.all_reduce(xin)
        xin.fill_(3.0)
        gr.replay()
        torch.cuda.synchronize()
        res["graph_all_reduce"] = bool((xin.float() == 3.0).all())
        dist.destroy_process_group()
        q.put(res)
    except Exception as e:  # surface it in the parent
        q.put(repr(e))
        raise


def test_rccl_branches_one_rank():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(60)
    assert isinstance(res, dict), res
    assert all(res.values()), res
    assert p.exitcode == 0
