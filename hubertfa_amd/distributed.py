"""Utterance data-parallelism across the GPUs of one node.

Utterances are independent, so the hot path shards with no collective in it: each rank aligns its own utterances
end to end.  The only data exchange is the final gather of the compact per-utterance boundary arrays
(ph_idx_seq, ph_time_int, frame_confidence, edge_diff, ...) to rank 0: an all_gather of every rank's table shape,
then one padded ``all_gather_into_tensor`` per array over RCCL (backend "nccl" on ROCm, xGMI links).  With
``gloo`` the same code moves host tensors (CPU tests, rehearsals).

The CLI (infer.py) adds a control plane over a gloo group (host memory, works even when a rank's GPU is lost):
every rank reports whether its shard completed; the shards of failed ranks are re-sharded (LPT) over the healthy
ranks and run again before the gather ("a GPU failure on one rank -> re-queue its shard").
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

BOUNDARY_KEYS = ("ph_idx_seq", "ph_time_int", "n", "frame_confidence")


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
    """alpha*L^2 + beta*L + gamma*T*S in arbitrary units (Hubert frames L at 50 fps); ``n_samples`` at ``sr``
    (the WAV header's own count and rate: hubertfa_amd.wav_io.wav_info)."""
    L = n_samples / sr * 50.0
    T = n_samples / sr * 44100 / hop
    return 1e-3 * L * L + 1.0 * L + 1e-4 * T * n_states


def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _comm_device(group=None) -> torch.device:
    """gloo moves host tensors; RCCL (nccl) moves device tensors over xGMI."""
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def gather_boundaries(dev_out: dict, keys=BOUNDARY_KEYS, uniform: bool = False, group=None, shortcut: bool = True):
    """All-gather per-utterance arrays of every rank; the local shapes may differ between ranks.

    ``dev_out[k]`` is [B] or [B, Tmax, ...] (one B per rank, one Tmax per rank over the 2-D keys).  Step 1
    all-gathers each rank's (B, Tmax); step 2 pads every array to the maximum and runs one
    ``all_gather_into_tensor`` per key.  ``uniform=True`` skips step 1 (every rank is known to hold the same
    shapes, e.g. the benchmark's equal batches: no host synchronisation then).

    Returns ``{k: [tensor of rank r, unpadded to its own (B_r, Tmax_r)] for r in ranks}``.  ``shortcut=False``
    runs the collectives even in a one-rank group (exercises the RCCL path on a one-GPU box)."""
    world = _world(group)
    if world == 1 and (shortcut or not dist.is_initialized()):
        return {k: [dev_out[k]] for k in keys}
    cdev = _comm_device(group)
    first2d = next((k for k in keys if dev_out[k].dim() >= 2), None)
    B = dev_out[keys[0]].shape[0]
    Tm = dev_out[first2d].shape[1] if first2d is not None else 0
    if uniform:
        shapes = [(B, Tm)] * world
    else:
        mine = torch.tensor([B, Tm], dtype=torch.int64, device=cdev)
        allsh = torch.empty((world * 2,), dtype=torch.int64, device=cdev)
        dist.all_gather_into_tensor(allsh, mine, group=group)
        shapes = [tuple(int(v) for v in row) for row in allsh.view(world, 2).cpu().tolist()]
    Bm = max(s[0] for s in shapes)
    Tmm = max(s[1] for s in shapes)
    out = {}
    for k in keys:
        t = dev_out[k].to(cdev)
        two_d = t.dim() >= 2
        pad_shape = (Bm, Tmm, *t.shape[2:]) if two_d else (Bm, *t.shape[1:])
        if tuple(t.shape) != pad_shape:
            p = torch.zeros(pad_shape, dtype=t.dtype, device=cdev)
            if two_d:
                p[:t.shape[0], :t.shape[1]] = t
            else:
                p[:t.shape[0]] = t
            t = p
        buf = torch.empty((world * Bm, *pad_shape[1:]), dtype=t.dtype, device=cdev)
        if Bm > 0:
            dist.all_gather_into_tensor(buf, t.contiguous(), group=group)
        out[k] = [buf[r * Bm:r * Bm + shapes[r][0], :shapes[r][1]] if two_d else buf[r * Bm:r * Bm + shapes[r][0]]
                  for r in range(world)]
    return out


# ---- the CLI's per-utterance boundary table ----------------------------------------------------------------
TABLE_KEYS = ("key", "n44", "T", "n", "ph_idx_seq", "ph_time_int", "frame_confidence", "edge_diff")


def pack_records(records: dict) -> dict:
    """{dataset index: raw record} -> padded host tensors (one row per utterance) for gather_boundaries.  A raw
    record holds exactly what the host assembly consumes: n44, T, ph_idx_seq/ph_time_int [n] and
    frame_confidence/edge_diff [T] (f32, as they leave the GPU)."""
    keys = sorted(records)
    U = len(keys)
    Tm = max([records[k]["T"] for k in keys], default=0)
    tab = {
        "key": torch.tensor(keys, dtype=torch.int64),
        "n44": torch.tensor([records[k]["n44"] for k in keys], dtype=torch.int64),
        "T": torch.tensor([records[k]["T"] for k in keys], dtype=torch.int32),
        "n": torch.tensor([len(records[k]["ph_idx_seq"]) for k in keys], dtype=torch.int32),
        "ph_idx_seq": torch.zeros((U, Tm), dtype=torch.int32),
        "ph_time_int": torch.zeros((U, Tm), dtype=torch.int32),
        "frame_confidence": torch.zeros((U, Tm), dtype=torch.float32),
        "edge_diff": torch.zeros((U, Tm), dtype=torch.float32),
    }
    for i, k in enumerate(keys):
        r = records[k]
        n, T = len(r["ph_idx_seq"]), r["T"]
        tab["ph_idx_seq"][i, :n] = torch.from_numpy(np.asarray(r["ph_idx_seq"], np.int32))
        tab["ph_time_int"][i, :n] = torch.from_numpy(np.asarray(r["ph_time_int"], np.int32))
        tab["frame_confidence"][i, :T] = torch.from_numpy(np.asarray(r["frame_confidence"], np.float32))
        tab["edge_diff"][i, :T] = torch.from_numpy(np.asarray(r["edge_diff"], np.float32))
    return tab


def unpack_records(gathered: dict) -> dict:
    """gather_boundaries output of packed tables -> {dataset index: raw record} over all ranks."""
    out = {}
    for r in range(len(gathered["key"])):
        g = {k: gathered[k][r].cpu().numpy() for k in TABLE_KEYS}
        for i in range(len(g["key"])):
            n, T = int(g["n"][i]), int(g["T"][i])
            out[int(g["key"][i])] = dict(n44=int(g["n44"][i]), T=T, ph_idx_seq=g["ph_idx_seq"][i, :n].astype(np.int64),
                                         ph_time_int=g["ph_time_int"][i, :n].astype(np.int64),
                                         frame_confidence=g["frame_confidence"][i, :T].copy(),
                                         edge_diff=g["edge_diff"][i, :T].copy())
    return out


def gather_records(records: dict, group=None) -> dict:
    """All ranks' raw records (every rank receives them; rank 0 exports)."""
    tab = pack_records(records)
    if _world(group) > 1 and _comm_device(group).type == "cuda":
        tab = {k: v.cuda() for k, v in tab.items()}
    return unpack_records(gather_boundaries(tab, TABLE_KEYS, group=group))
