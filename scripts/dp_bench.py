"""Viterbi forward/backtrack microbenchmark (GPU box): config 2 (B=32, T=861, S=91) and config 5 (B=1,
T=25839, S=1801) lattices, default and forced states-per-lane variants."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402


def run(B, T, S, force_k, reps=3):
    dev = torch.device("cuda")
    P = -(-S // 8) * 8
    g = torch.Generator(device="cpu").manual_seed(0)
    pl = (-torch.rand((B, T, P), generator=g) * 5).to(dev)
    E = (-torch.rand((B, T), generator=g)).to(dev)
    nE = (-torch.rand((B, T), generator=g)).to(dev)
    ids = torch.randint(1, 60, (B, P), generator=g, dtype=torch.int32).to(dev)
    ids[:, ::3] = 0
    Tt = torch.full((B,), T, dtype=torch.int32, device=dev)
    St = torch.full((B,), S, dtype=torch.int32, device=dev)
    dp = torch.full((B, T, P), float("-inf"), device=dev)
    dp[:, 0, 0] = 0
    bt = torch.empty((B, T, P), dtype=torch.int8, device=dev)
    curr = torch.full((B, P), float("-inf"), dtype=torch.float64, device=dev)
    _lib.lib().hfa_viterbi_tuning(force_k)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ops.viterbi_forward(pl, nE, E, curr, dp, bt, ids, Tt, St)
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        ops.viterbi_forward(pl, nE, E, curr, dp, bt, ids, Tt, St)
    ev[1].record()
    for _ in range(reps):
        ops.viterbi_backtrack(dp, bt, ids, Tt, St)
    ev[2].record()
    torch.cuda.synchronize()
    _lib.lib().hfa_viterbi_tuning(0)
    f = ev[0].elapsed_time(ev[1]) / reps
    b = ev[1].elapsed_time(ev[2]) / reps
    print(f"B={B:3d} T={T:6d} S={S:5d} K={force_k or 'auto'}: forward {f:8.3f} ms ({1e3 * f / T:6.3f} us/step), "
          f"backtrack {b:7.3f} ms", flush=True)


if __name__ == "__main__":
    for k in (0, 2, 4):
        run(32, 861, 91, k)
    for k in (0, 2, 4, 8):
        run(1, 25839, 1801, k)
