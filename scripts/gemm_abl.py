"""Split-GEMM microbenchmark for library A/Bs (HFA_LIB selects the build): us per launch and f32-equivalent TF/s on
config 2's dominant shapes with the automatic tile, median of 5 x --reps launches (run on the GPU box)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hubertfa_amd import _lib, ops  # noqa: E402

# name, M, N, K, Zb, conv (k, stride, Tin, Cin) or None, epilogue, planes out, residual planes
SHAPES = [("conv1", 15999, 512, 1536, 32, (3, 2, 31999, 512), 1, True, False),
          ("ffn1", 15968, 3072, 768, 1, None, 1, True, False),
          ("qkv", 15968, 2304, 768, 1, None, 0, True, False),
          ("ffn2", 15968, 768, 3072, 1, None, 0, False, True),
          ("outproj", 15968, 768, 768, 1, None, 0, False, True)]
# --convs: the extractor's k = 3 convs at config 2 (B = 32), and conv1 / conv2 at other batch sizes
CONVS = [("conv1", 15999, 512, 1536, 32, (3, 2, 31999, 512), 1, True, False),
         ("conv2", 7999, 512, 1536, 32, (3, 2, 15999, 512), 1, True, False),
         ("conv3", 3999, 512, 1536, 32, (3, 2, 7999, 512), 1, True, False),
         ("conv4", 1999, 512, 1536, 32, (3, 2, 3999, 512), 1, True, False),
         ("conv1b16", 15999, 512, 1536, 16, (3, 2, 31999, 512), 1, True, False),
         ("conv2b64", 7999, 512, 1536, 64, (3, 2, 15999, 512), 1, True, False)]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--data", default="randn", choices=["randn", "zeros", "hionly", "wrows", "arows", "gelu", "gelu_off", "gelu_s4"],
                    help="operand data: randn, all zeros, f16-exact values (zero low planes), every W row equal (wrows) or every "
                         "A row equal (arows)")
    ap.add_argument("--convs", action="store_true", help="the extractor conv shapes instead")
    ap.add_argument("--chain", action="store_true",
                    help="with --convs: conv1..conv4 back to back (each reading the previous output), each timed "
                         "with events, after the isolated loops")
    ap.add_argument("--cfg", type=int, default=0, help="split tile (hfa_gemm_split_tuning); outputs are checked "
                    "bit for bit against the automatic tile's")
    ap.add_argument("--tag", default=os.path.basename(os.path.dirname(os.environ.get("HFA_LIB", "cur/x"))))
    args = ap.parse_args()
    d = torch.device("cuda")

    def rnd(*shape):
        x = torch.randn(*shape, device=d)
        if args.data == "zeros":
            return torch.zeros_like(x)
        return x

    def act(x):                                # the A operand: GELU outputs like the extractor's conv inputs
        if args.data == "gelu":
            return torch.nn.functional.gelu(x)
        if args.data == "gelu_s4":
            return torch.nn.functional.gelu(4.0 * x)
        if args.data == "gelu_off":            # shifted positive (sign bit constant, exponents concentrated)
            return torch.nn.functional.gelu(x) + 0.25
        return x

    def rows_equal(x, which):                  # hionly rounding; every row (last dim) a copy of row 0 for `which`
        if args.data == "hionly":
            return x.half().float()
        if args.data != which:
            return x
        x2 = x.reshape(-1, x.shape[-1])
        return x2[:1].expand_as(x2).contiguous().reshape(x.shape)

    for name, M, N, K, Zb, conv, epi, outs, res in (CONVS if args.convs else SHAPES):
        W = ops.split(rows_equal(rnd(N, K) * K ** -0.5, "wrows"))
        b = torch.randn(N, device=d)
        if conv:
            k, s, Tin, Cin = conv
            A = ops.split(act(rows_equal(rnd(Zb, Tin, Cin), "arows")))
            C = torch.empty(2, Zb, M, N, dtype=torch.float16, device=d)

            def go():
                ops.conv_gemm_split(A, W, Cs=C, M=M, N=N, K=K, Zb=Zb, sAb=Tin * Cin, ldx=Cin, stride=s, Cg=Cin,
                                    Tin=Tin, bias=b, sCb=M * N, ldc=N, epilogue=epi)
                return C
        else:
            A = ops.split(act(rows_equal(rnd(M, K), "arows")))
            R = ops.split(torch.randn(M, N, device=d)) if res else None

            def go():
                return ops.linear_split(A, W, b, residual=R, epilogue=epi, out_split=outs)
        tag = args.tag
        if args.cfg:
            ref = go().clone()
            _lib.lib().hfa_gemm_split_tuning(args.cfg)
            same = torch.equal(go(), ref)
            tag = f"{args.tag}/cfg{args.cfg}{'' if same else '/MISMATCH'}"
        us = timeit(go, args.reps // (4 if conv else 1) or 1)
        if args.cfg:
            _lib.lib().hfa_gemm_split_tuning(0)
        print(f"{tag + '/' + args.data:18s} {name:8s} {us:8.1f} us {2.0 * M * N * K * Zb / us / 1e6:7.1f} TF/s", flush=True)
    if args.convs and args.chain:
        chain_convs(d)


def chain_convs(d):
    """conv1 -> conv2 -> conv3 -> conv4 as in the extractor (each conv's planes are the next one's input), 10
    chains after 3 warm-up chains, every conv timed with its own events: the per-conv time in sequence against the
    isolated loops above."""
    B, T = 32, 31999
    x = ops.split(torch.nn.functional.gelu(torch.randn(B, T, 512, device=d)))
    plan, Tin = [], T
    for i in range(4):
        M = (Tin - 3) // 2 + 1
        W = ops.split(torch.randn(512, 1536, device=d) * 1536 ** -0.5)
        C = torch.empty(2, B, M, 512, dtype=torch.float16, device=d)
        plan.append((M, Tin, W, C))
        Tin = M
    b = torch.randn(512, device=d)

    def run(evs):
        A = x
        for i, (M, Tin_, W, C) in enumerate(plan):
            evs[i][0].record()
            ops.conv_gemm_split(A, W, Cs=C, M=M, N=512, K=1536, Zb=B, sAb=Tin_ * 512, ldx=512, stride=2, Cg=512,
                                Tin=Tin_, bias=b, sCb=M * 512, ldc=512, epilogue=1)
            evs[i][1].record()
            A = C
    ts = [[] for _ in plan]
    for rep in range(13):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in plan]
        run(evs)
        torch.cuda.synchronize()
        if rep >= 3:
            for i in range(len(plan)):
                ts[i].append(evs[i][0].elapsed_time(evs[i][1]) * 1e3)
    for i, (M, Tin_, W, C) in enumerate(plan):
        us = sorted(ts[i])[len(ts[i]) // 2]
        print(f"chain              conv{i + 1}    {us:8.1f} us {2.0 * M * 512 * 1536 * B / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
