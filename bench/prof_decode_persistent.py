"""Timeline of the persistent decode-step kernel (needs a DIE_KERNEL_DIAG=1 build): per phase of each layer,
when the workgroups entered their task, had its data, finished the compute and finished the epilogue
(100 MHz clock, microseconds from the earliest stamp). Llama-3-8B shapes at batch 32, random init.

DIE_C_DIAG=1 python bench/prof_decode_persistent.py [layers]

(ready_wait = task entry -> its first chunk's data in LDS: the dependency wait, the late activation loads
and the first chunk; compute = the chunk stream; epi = the epilogue and publish.)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DIE_PERSISTENT", "1")

from src import ops  # noqa: E402
from src.models.llama import AttnMetadata, CausalLM  # noqa: E402
from src.models.presets import get_preset  # noqa: E402

PH = ("qkv", "att", "o", "gu", "dn")


def main():
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda:0")
    M, bs, max_ctx = 32, 16, 1024
    m = CausalLM(get_preset("llama3-8b", num_layers=layers), dev, seed=0, max_position=max_ctx + 16)
    nbps = max_ctx // bs
    nblocks = M * nbps + 8
    pool = (torch.randn(layers, 2, nblocks, m.hkv, bs, 128, device=dev) * 0.5).to(torch.bfloat16)
    bt = torch.randperm(nblocks - 8)[: M * nbps].view(M, nbps).to(torch.int32).to(dev)
    ctx = torch.tensor([512 + 4 * i for i in range(M)], dtype=torch.int32, device=dev)
    pos = (ctx - 1).long()
    slots = bt[torch.arange(M, device=dev), pos // bs].long() * bs + pos % bs
    ids = torch.randint(0, 128256, (M,), device=dev)
    sc = m.alloc_decode_scratch(M)
    assert m.prepare_persistent(pool, sc)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    pbuf = torch.zeros(ncu * layers * 5 * 4, dtype=torch.int64, device=dev)
    prof = pbuf.view(ncu, layers * 5, 4)
    sc["persistent"]["prof"] = pbuf
    maxp = ops.decode_partials(max_ctx)
    meta = AttnMetadata(False, slots, bt, ctx, max_ctx=max_ctx, scratch=sc,
                        part_o=torch.empty(M * m.hq * maxp * 128, dtype=torch.float32, device=dev),
                        part_ml=torch.empty(M * m.hq * maxp * 2, dtype=torch.float32, device=dev),
                        attn_cnt=torch.zeros(M * m.hkv, dtype=torch.int32, device=dev))
    with torch.inference_mode():
        for _ in range(3):
            pbuf.zero_()
            m.forward(ids, pos, meta, pool)
        torch.cuda.synchronize()
    summarize(prof.cpu(), layers, int(sc["persistent"]["err"].item()))


def summarize(p, layers, err):
    valid = p[..., 0] > 0
    t0 = p[..., 0][valid].min().item()
    us = (p.double() - t0) / 100.0  # 100 MHz -> us
    print(json.dumps({"err": err, "stamped_tasks": int(valid.sum()),
                      "total_us": round(us[..., 3][valid].max().item(), 1),
                      "us_per_layer": round(us[..., 3][valid].max().item() / layers, 1)}), flush=True)
    for q in range(layers * 5):
        v = valid[:, q]
        if not v.any():
            continue
        s = us[v, q]
        row = {"layer": q // 5, "phase": PH[q % 5], "tasks": int(v.sum())}
        for i, name in enumerate(("enter", "ready", "computed", "done")):
            row[name] = [round(s[:, i].min().item(), 1), round(s[:, i].median().item(), 1),
                         round(s[:, i].max().item(), 1)]
        row["ready_wait_med"] = round((s[:, 1] - s[:, 0]).median().item(), 1)
        row["compute_med"] = round((s[:, 2] - s[:, 1]).median().item(), 1)
        row["epi_med"] = round((s[:, 3] - s[:, 2]).median().item(), 1)
        row["last_done_minus_med"] = round(row["done"][2] - row["done"][1], 1)
        row["span"] = round(row["done"][2] - row["enter"][0], 1)
        if q // 5 == 1 or layers == 1:
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
