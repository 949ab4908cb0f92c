"""Generation sharding across GPUs (weak scaling, no data-path collective).

Generations are independent: rank ``rank`` of ``world`` owns the contiguous
generation range [rank*G, (rank+1)*G) of one logical batch, with the same source / repair id
bases that a single-GPU run over the whole batch would use, so every coefficient -- and hence
every repair byte and decode outcome -- is identical to the 1-GPU result.  The only
inter-rank traffic is a barrier and a max-reduce of the step time, over gloo on host tensors
(bench.py's default on the GPUs too, so no RCCL communicator is created; NTC_BENCH_BACKEND=nccl
selects RCCL for that reduction).
"""
from __future__ import annotations

import numpy as np


def generation_shard(rank: int, world: int, G: int, k: int, r: int,
                     sid_origin: int = 0, rid_origin: int = 0):
    """Per-generation id bases (uint32, wrapping like the reference's uint32 ids) for a rank."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    g = np.arange(rank * G, (rank + 1) * G, dtype=np.uint64)
    sid = ((sid_origin + g * k) & 0xFFFFFFFF).astype(np.uint32)
    rid = ((rid_origin + g * r) & 0xFFFFFFFF).astype(np.uint32)
    return sid, rid


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of a scalar over the process group (the bench's step-time reduction)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    if dist.get_backend() == "gloo":
        device = None                    # gloo reduces host tensors
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
