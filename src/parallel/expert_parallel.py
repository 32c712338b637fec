"""
Expert parallelism with all-to-all token dispatch (data-parallel attention + expert-parallel MoE).

Two EP layouts exist in this engine:

* **EP over replicated tokens** (``CausalLM(moe_parallel="ep")`` under tensor parallelism): the
  attention is TP-sharded, so every rank already holds every token; each rank computes its own
  experts' share and the MoE's TP all-reduce is the combine (``ops.expert_parallel_local``).
* **EP over distinct tokens** (this module): each rank runs its own batch (a data-parallel
  replica's attention) and owns ``E / W`` whole experts. A MoE layer then

    1. routes locally (router replicated), top-k over all E experts;
    2. packs every (token, slot) assignment into the send buffer of the rank that owns its
       expert — ``[W, C, H]`` rows plus ``[W, C]`` local expert ids (-1 = empty row);
    3. ``all_to_all`` (RCCL over xGMI: one direct link per peer on an MI355X node, the same
       point-to-point pattern RCCL's all-to-all uses) delivers each rank the rows for its experts;
    4. runs its experts on the received rows (``ops.moe_apply``, grouped HIP GEMMs);
    5. a second ``all_to_all`` returns the expert outputs to the senders, which combine them with
       the routing weights.

  Two shapes of the exchange:

  * ``capacity=C`` (static, hipGraph-capturable, no host sync): C rows per destination; a
    destination overflowing C drops its surplus assignments (weight 0) — capacity-factor
    semantics. ``C = T * k`` never drops.
  * ``capacity=None`` (exact, eager): the per-destination counts are exchanged first
    (``all_to_all_single`` of W integers + one host read) and only the real rows travel — the
    prefill form, where a [W, T*k, H] padded buffer would be gigabytes.

The packing/unpacking is plain tensor index arithmetic (sort by destination, rank within the
destination by a cumulative sum), so the GPU path launches no Python loop per token.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from src import ops


def _a2a(out: torch.Tensor, inp: torch.Tensor, group, out_splits=None, in_splits=None) -> None:
    """all_to_all_single; GPU tensors on a gloo group are staged through the host (tests)."""
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def ep_moe_forward(x: torch.Tensor, router: torch.Tensor, w13_local: torch.Tensor, w2_local: torch.Tensor,
                   top_k: int, group=None, capacity: Optional[int] = None, renorm: bool = True) -> torch.Tensor:
    """MoE layer for this rank's tokens ``x [T, H]`` with experts sharded over ``group``:
    rank r owns experts ``[r * E_l, (r + 1) * E_l)`` (``w13_local [E_l, 2I, H]``,
    ``w2_local [E_l, H, I]``); ``router [E, H]`` is replicated. Returns ``[T, H]``."""
    W = dist.get_world_size(group)
    r = dist.get_rank(group)
    T, H = x.shape
    El = w13_local.shape[0]
    E = router.shape[0]
    if E != El * W:
        raise ValueError(f"{E} experts do not split into {W} x {El}")
    dev = x.device
    gating = torch.nn.functional.linear(x, router)
    w, ids = ops.topk_softmax(gating, top_k, renorm)      # [T, k] fp32, int32
    ids = ids.long()
    n = T * top_k
    dest = (ids // El).reshape(-1)                        # owner rank of each assignment
    loc = (ids % El).reshape(-1)                          # expert id on the owner
    tok = torch.arange(T, device=dev).repeat_interleave(top_k)
    order = torch.argsort(dest, stable=True)              # assignments grouped by destination
    d_sorted = dest[order]
    counts = torch.bincount(dest, minlength=W)            # [W]
    starts = torch.cumsum(counts, 0) - counts
    rank_in_dest = torch.arange(n, device=dev) - starts[d_sorted]  # slot within its destination

    if capacity is not None:
        C = int(capacity)
        keep = rank_in_dest < C
        slot = d_sorted * C + rank_in_dest.clamp(max=C - 1)
        send = torch.zeros(W * C, H, dtype=x.dtype, device=dev)
        send_id = torch.full((W * C,), -1, dtype=torch.int32, device=dev)
        src_rows = tok[order]
        send.index_copy_(0, slot[keep], x[src_rows[keep]])
        send_id.index_copy_(0, slot[keep], loc[order][keep].to(torch.int32))
        recv = torch.empty_like(send)
        recv_id = torch.empty_like(send_id)
        _a2a(recv, send, group)
        _a2a(recv_id, send_id, group)
        y = _run_local_experts(recv, recv_id, w13_local, w2_local, El)
        back = torch.empty_like(y)
        _a2a(back, y, group)
        # assignment (sorted position j) -> its returned row; dropped ones contribute 0
        contrib = torch.zeros(n, H, dtype=torch.float32, device=dev)
        contrib[order[keep]] = back[slot[keep]].float()
    else:
        in_splits = counts.tolist()
        cnt_out = torch.empty_like(counts)
        _a2a(cnt_out, counts, group)
        out_splits = cnt_out.tolist()
        send = x[tok[order]].contiguous()
        send_id = loc[order].to(torch.int32).contiguous()
        recv = torch.empty(sum(out_splits), H, dtype=x.dtype, device=dev)
        recv_id = torch.empty(sum(out_splits), dtype=torch.int32, device=dev)
        _a2a(recv, send, group, out_splits, in_splits)
        _a2a(recv_id, send_id, group, out_splits, in_splits)
        y = _run_local_experts(recv, recv_id, w13_local, w2_local, El)
        back = torch.empty(n, H, dtype=x.dtype, device=dev)
        _a2a(back, y, group, in_splits, out_splits)
        contrib = torch.zeros(n, H, dtype=torch.float32, device=dev)
        contrib[order] = back.float()
    # weighted combine in the routing's (token, slot) order
    out = (contrib.view(T, top_k, H) * w.view(T, top_k, 1)).sum(1)
    del r
    return out.to(x.dtype)


def _run_local_experts(rows: torch.Tensor, ids: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor,
                       El: int) -> torch.Tensor:
    """Each received row through its local expert (``ids`` -1 = empty row -> zeros)."""
    if rows.shape[0] == 0:
        return rows.clone()
    valid = ids >= 0
    ids1 = torch.where(valid, ids, torch.full_like(ids, El)).view(-1, 1)
    wts = valid.to(torch.float32).view(-1, 1)
    return ops.moe_apply(rows, w13, w2, wts, ids1, El + 1)
