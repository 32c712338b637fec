"""Repeat the persistent decode step on fixed inputs (eager launches, then hipGraph replays) and report which
runs differ from the first: max |diff| of the output and of the KV pool. Diagnoses races in
csrc/kernels/decode_persistent.hip. python bench/check_dp_determinism.py [preset] [layers] [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DIE_PERSISTENT", "1")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

from test_decode_persistent_gpu import _setup  # noqa: E402
from src.models.llama import AttnMetadata  # noqa: E402


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "llama-mini"
    layers = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    m, pool, bt, ctx, pos, slots, ids, meta_kw, max_ctx = _setup(preset, layers, 32, [100] * 32, seed=5)
    sc = m.alloc_decode_scratch(32)
    assert m.prepare_persistent(pool, sc)
    meta = AttnMetadata(False, slots, bt, ctx, max_ctx=max_ctx, scratch=sc, **meta_kw)
    outs, pools, stages = [], [], []
    cfg, ws = sc["persistent"]["cfg"], sc["persistent"]["ws"]
    H, nq = m.arch.hidden_size, (m.hq + 2 * m.hkv) * 128
    sizes = {"slab_q": cfg["skq"] * 32 * nq * 4, "attn": 32 * m.hq * 128 * 2,
             "slab_od": max(cfg["sko"], cfg["skd"]) * 32 * H * 4, "act": 32 * m.inter * 2,
             "ssp_o": (H // cfg["wro"]) * 128 * 4, "ssp_d": (H // cfg["wrd"]) * 128 * 4}
    offs = {"slab_q": "slabq_off", "attn": "attn_off", "slab_od": "slabod_off", "act": "act_off",
            "ssp_o": "sspo_off", "ssp_d": "sspd_off"}
    names = [(n, offs[n], sizes[n]) for n in sizes]

    def snap():
        return {n: ws[cfg[o]:cfg[o] + sz].clone() for n, o, sz in names}
    with torch.inference_mode():
        for _ in range(reps):
            outs.append(m.forward(ids, pos, meta, pool).clone())
            torch.cuda.synchronize()
            pools.append(pool.clone())
            stages.append(snap())
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m.forward(ids, pos, meta, pool)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph):
            out = m.forward(ids, pos, meta, pool)
        zero = os.environ.get("DP_ZERO_SYNC") == "1"
        for _ in range(reps):
            if zero:  # experiment: counters zeroed outside the graph before each replay
                ws[cfg["sync_off"]:].zero_()
                torch.cuda.synchronize()
            graph.replay()
            torch.cuda.synchronize()
            outs.append(out.clone())
            pools.append(pool.clone())
            stages.append(snap())
    ref, pref = outs[0].float(), pools[0].float()
    res = []
    for i, (o, p) in enumerate(zip(outs, pools)):
        d = {"run": i, "graph": i >= reps, "out": float((o.float() - ref).abs().max()),
             "pool": float((p.float() - pref).abs().max())}
        d["stages_differ"] = [n for n, _, _ in names if not torch.equal(stages[i][n], stages[0][n])]
        if d["pool"] > 0:
            diff = (p.float() - pref).abs().amax(dim=(-1,))  # [L, 2, blocks, hkv, 16]
            idx = diff.nonzero()[:8].tolist()
            d["pool_rows"] = idx
        res.append(d)
    print(json.dumps({"err": sc["persistent"]["err_info"].tolist(), "preset": preset, "layers": layers}))
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
