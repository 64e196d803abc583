"""Utterance data-parallelism across the GPUs of one node.

Utterances are independent, so the hot path shards with no collective in it: each rank aligns its own utterances
end to end.  The only exchange is the final gather of the compact per-utterance boundary arrays
(ph_idx_seq, ph_time_int, n, frame_confidence) to rank 0 — one padded ``all_gather_into_tensor`` per array over
RCCL (backend "nccl" on ROCm, xGMI links); with ``gloo`` the same code runs on CPU tensors (tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def env_rank_world():
    import os
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def shard_lpt(costs, world: int):
    """Longest-processing-time assignment of utterance indices to ranks (estimated cost per utterance)."""
    order = sorted(range(len(costs)), key=lambda i: -costs[i])
    loads = [0.0] * world
    shards = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: loads[k])
        shards[r].append(i)
        loads[r] += costs[i]
    return [sorted(s) for s in shards]


def utterance_cost(n_samples: int, n_states: int, sr: int = 44100, hop: int = 512) -> float:
    """alpha*L^2 + beta*L + gamma*T*S in arbitrary units (Hubert frames L at 50 fps)."""
    L = n_samples / sr * 50.0
    T = n_samples / hop
    return 1e-3 * L * L + 1.0 * L + 1e-4 * T * n_states


def gather_boundaries(dev_out: dict, dst_world: int | None = None):
    """All-gather the per-utterance boundary arrays of every rank (same local batch shape on every rank).

    Returns a dict of [world * B, ...] tensors (ph_idx_seq, ph_time_int, n, frame_confidence).
    """
    world = dist.get_world_size() if dist.is_initialized() else 1
    keys = ("ph_idx_seq", "ph_time_int", "n", "frame_confidence")
    if world == 1:
        return {k: dev_out[k] for k in keys}
    out = {}
    host_side = dist.get_backend() == "gloo"   # gloo moves host tensors; RCCL moves device tensors over xGMI
    for k in keys:
        t = dev_out[k].contiguous()
        if host_side:
            t = t.cpu()
        buf = torch.empty((world * t.shape[0], *t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(buf, t)
        out[k] = buf
    return out
