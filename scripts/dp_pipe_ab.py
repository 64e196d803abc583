"""Multi-wave Viterbi forward A/B (GPU box; needs viterbi.hip of commit 6e78506, where hfa_viterbi_tuning(100 + k)
selects the ring): the per-step barrier exchange vs the point-to-point boundary ring.  Checks the two give
bit-identical dp / bt / curr, then times both, interleaved (profiles/r04/dp_ring_ab.txt).
    python scripts/dp_pipe_ab.py [--reps 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import ops, _lib  # noqa: E402


def lattice(B, T, S, seed=0):
    dev = torch.device("cuda")
    P = -(-S // 8) * 8
    g = torch.Generator(device="cpu").manual_seed(seed)
    pl = (-torch.rand((B, T, P), generator=g) * 5).to(dev)
    E = (-torch.rand((B, T), generator=g)).to(dev)
    nE = (-torch.rand((B, T), generator=g)).to(dev)
    ids = torch.randint(1, 60, (B, P), generator=g, dtype=torch.int32).to(dev)
    ids[:, ::3] = 0
    Tt = torch.full((B,), T, dtype=torch.int32, device=dev)
    St = torch.full((B,), S, dtype=torch.int32, device=dev)
    return pl, E, nE, ids, Tt, St, P


def forward(lat, mode, reps):
    pl, E, nE, ids, Tt, St, P = lat
    B, T = pl.shape[0], pl.shape[1]
    dev = pl.device
    dp = torch.full((B, T, P), float("-inf"), device=dev)
    dp[:, 0, 0] = 0
    bt = torch.zeros((B, T, P), dtype=torch.int8, device=dev)
    curr0 = torch.full((B, P), float("-inf"), dtype=torch.float64, device=dev)
    curr0[:, 0] = 0
    _lib.lib().hfa_viterbi_tuning(mode)
    try:
        curr = curr0.clone()
        ops.viterbi_forward(pl, nE, E, curr, dp, bt, ids, Tt, St)
        out = (dp.clone(), bt.clone(), curr.clone())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            curr.copy_(curr0)
            ops.viterbi_forward(pl, nE, E, curr, dp, bt, ids, Tt, St)
        e1.record()
        torch.cuda.synchronize()
    finally:
        _lib.lib().hfa_viterbi_tuning(0)
    return out, e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    cases = [(4, 3000, 300), (4, 3000, 700), (2, 6000, 1100), (1, 25839, 1801), (2, 4000, 3000),
             (1, 6000, 4000), (1, 4000, 6000), (1, 3000, 8000)]
    for B, T, S in cases:
        lat = lattice(B, T, S)
        for k in (0, 2, 8):
            if k == 2 and S > 2048:
                continue
            (a, ta), (b, tb) = forward(lat, k, args.reps), forward(lat, 100 + k, args.reps)
            same = all(torch.equal(x, y) for x, y in zip(a, b))
            _, ta2 = forward(lat, k, args.reps)
            _, tb2 = forward(lat, 100 + k, args.reps)
            tA, tB = min(ta, ta2), min(tb, tb2)
            print(f"B={B} T={T:5d} S={S:5d} K={k or 'auto'}: barrier {tA:8.3f} ms ({1e3 * tA / T:.3f} us/step), "
                  f"ring {tB:8.3f} ms ({1e3 * tB / T:.3f} us/step), x{tA / tB:.3f}, bit-identical {same}", flush=True)
            if not same:
                print("MISMATCH", flush=True)
                sys.exit(1)


if __name__ == "__main__":
    main()
