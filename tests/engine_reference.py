"""No-cache reference generation: every token recomputed from the full
sequence with a fresh KV pool (independent of paging, prefix caching,
chunking, batching and hipGraphs)."""

import torch

from src.models.llama import AttnMetadata


@torch.inference_mode()
def greedy_reference(model, prompt, max_tokens, block_size=16):
    dev = model.device
    ids = list(prompt)
    out = []
    n_total = len(prompt) + max_tokens
    nb = (n_total + block_size - 1) // block_size
    pool = torch.zeros(model.arch.num_layers, 2, nb, model.hkv, block_size, model.head_dim,
                       dtype=model.dtype, device=dev)
    for _ in range(max_tokens):
        t = len(ids)
        x = torch.tensor(ids, dtype=torch.long, device=dev)
        pos = torch.arange(t, dtype=torch.long, device=dev)
        meta = AttnMetadata(is_prefill=True, slot_mapping=pos.clone(),
                            block_tables=torch.arange(nb, dtype=torch.int32, device=dev)[None],
                            ctx_lens=torch.tensor([t], dtype=torch.int32, device=dev),
                            cu_q=torch.tensor([0, t], dtype=torch.int32, device=dev), max_q_len=t)
        h = model.forward(x, pos, meta, pool)
        logits = model.compute_logits(h[-1:])
        tok = int(torch.argmax(logits[0].float()))
        ids.append(tok)
        out.append(tok)
    return out
