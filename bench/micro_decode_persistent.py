"""Decode-step layers of Llama-3-8B at batch 32 (contexts ~512-640 keys, random init): the persistent
decode-step kernel (csrc/kernels/decode_persistent.hip, all 32 layers in one launch) against the multi-launch
fused path (5 launches per layer) — with the production tiles and with the persistent kernel's own tiles.
Each variant is captured in a hipGraph; the timed region is graph replays (layers + final norm, no LM head).

python bench/micro_decode_persistent.py [layers] [reps] [rows]
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


def main():
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    bs, max_ctx = 16, 1024
    m = CausalLM(get_preset("llama3-8b", num_layers=layers), dev, seed=0, max_position=max_ctx + 16)
    nbps = max_ctx // bs
    nblocks = M * nbps + 8
    pool = (torch.randn(layers, 2, nblocks, m.hkv, bs, 128, device=dev) * 0.5).to(torch.bfloat16)
    bt = torch.randperm(nblocks - 8)[: M * nbps].view(M, nbps).to(torch.int32).to(dev)
    ctx = torch.tensor([512 + 4 * i for i in range(M)], dtype=torch.int32, device=dev)
    pos = (ctx - 1).long()
    slots = bt[torch.arange(M, device=dev), pos // bs].long() * bs + pos % bs
    ids = torch.randint(0, 128256, (M,), device=dev)
    maxp = ops.decode_partials(max_ctx)
    kw = dict(part_o=torch.empty(M * m.hq * maxp * 128, dtype=torch.float32, device=dev),
              part_ml=torch.empty(M * m.hq * maxp * 2, dtype=torch.float32, device=dev),
              attn_cnt=torch.zeros(M * m.hkv, dtype=torch.int32, device=dev))
    sc = m.alloc_decode_scratch(M)
    assert m.prepare_persistent(pool, sc), "no persistent instantiation"
    cfg = sc["persistent"]["cfg"]
    ptile = {"qkv": (cfg["wrq"], 128, cfg["skq"]), "o": (cfg["wro"], 128, cfg["sko"]),
             "down": (cfg["wrd"], 128, cfg["skd"]), "gate_up": (cfg["wrg"], 128)}
    multi = {k: v for k, v in sc.items() if k != "persistent"}
    multi_pt = dict(multi, plans={b: ptile for b in sc["plans"]})
    variants = {"multi_launch": multi, "multi_launch_persistent_tiles": multi_pt, "persistent": sc}
    res = {}
    for name, scratch in variants.items():
        meta = AttnMetadata(False, slots, bt, ctx, max_ctx=max_ctx, scratch=scratch, **kw)
        with torch.inference_mode():
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    m.forward(ids, pos, meta, pool)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                m.forward(ids, pos, meta, pool)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(reps):
                g.replay()
            t1.record()
            torch.cuda.synchronize()
            ms = t0.elapsed_time(t1) / reps
        wbytes = sum(getattr(lw, n).numel() * 2 for lw in m.layers for n in ("qkv", "o", "gate_up", "down"))
        kvbytes = int(ctx.sum()) * m.hkv * 128 * 2 * 2 * layers
        res[name] = ms
        print(json.dumps({"variant": name, "layers": layers, "rows": M, "ms_per_step": round(ms, 4),
                          "us_per_layer": round(1e3 * ms / layers, 2),
                          "TBps": round((wbytes + kvbytes) / ms / 1e9, 2)}), flush=True)
    err = int(sc["persistent"]["err"].item())
    print(json.dumps({"persistent_err_word": err,
                      "speedup_vs_multi_launch": round(res["multi_launch"] / res["persistent"], 4)}), flush=True)


if __name__ == "__main__":
    main()
