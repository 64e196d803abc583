"""CPU experiment: what does evaluating every GEMM/conv of the encoder + UNet as a split low-precision MFMA
product do to the per-frame log-probs and the boundaries?  (Decides the GEMM arithmetic; not a test.)

Modes (operand a = a1 + a2 [+ a3], every partial product exact in f32, f32 accumulation — what the MFMA does):
  bf16x3: a1 = bf16(a), a2 = bf16(a - a1);                  a1b1 + a1b2 + a2b1
  bf16x6: three bf16 pieces (exact split of f32);           + a1b3 + a2b2 + a3b1
  fp16x3: a1 = fp16(a), a2 = fp16((a - a1) * 2^11);         a1b1 + 2^-11 (a1b2 + a2b1)
Reference: the same oracle in f64 (the f32 oracle's own error is printed beside).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import yaml  # noqa: E402

import bench  # noqa: E402
from hubertfa_amd import synth  # noqa: E402
from hubertfa_amd.task import synth_checkpoint  # noqa: E402
from oracle import decode as odec, hubert_cpu, resample as ores  # noqa: E402


def pieces(t, mode):
    if mode == "fp16x3":
        a1 = t.half().float()
        return [a1, ((t - a1) * 2048.0).half().float()]
    a1 = t.bfloat16().float()
    r = t - a1
    a2 = r.bfloat16().float()
    if mode == "bf16x3":
        return [a1, a2]
    return [a1, a2, (r - a2).bfloat16().float()]


def split_op(op, mode):
    def f(x, w, b=None, **kw):
        if x.dtype == torch.float64:
            return op(x, w, b, **kw)
        xs, ws = pieces(x, mode), pieces(w, mode)
        if mode == "fp16x3":
            out = op(xs[0], ws[0], None, **kw) + (op(xs[0], ws[1], None, **kw) + op(xs[1], ws[0], None, **kw)) / 2048.0
        else:
            terms = [(0, 0), (0, 1), (1, 0)] + ([(0, 2), (1, 1), (2, 0)] if mode == "bf16x6" else [])
            out = sum(op(xs[i], ws[j], None, **kw) for i, j in reversed(terms))
        return out if b is None else out + (b.view(-1, *([1] * (out.dim() - 2))) if op is not F.linear else b)
    return f


class FNS:
    def __init__(self, mode):
        self.mode = mode

    def __getattr__(self, k):
        v = getattr(F, k)
        if self.mode and k in ("linear", "conv1d", "conv_transpose1d"):
            return split_op(v, self.mode)
        return v


def run(mode, dtype, wav, ph_seqs, word_seqs, p2ws, vocab, sd, usd, ua, arch):
    hubert_cpu.F = FNS(mode)
    orig_float = torch.Tensor.float
    if dtype == torch.float64:   # the oracle casts with .float(): run it in f64 by redirecting the cast
        torch.Tensor.float = lambda t, *a, **k: t.double()
    sd_ = {k: v.to(dtype) if torch.is_tensor(v) and v.is_floating_point() else v for k, v in sd.items()}
    usd_ = {k: v.astype(np.float64 if dtype == torch.float64 else np.float32) if v.dtype.kind == "f" else v
            for k, v in usd.items()}
    outs = []
    for b in range(len(ph_seqs)):
        x44 = ores.resample(torch.from_numpy(wav[b:b + 1]), 16000, 44100, 6)
        x16 = ores.resample(x44, 44100, 16000, 128).to(dtype)
        units = hubert_cpu.hubert_forward(arch, sd_, x16)
        n44 = x44.shape[-1]
        nf = n44 // 512 + 1
        idx = torch.clamp(torch.round(((512 / 44100) / (320 / 16000)) * torch.arange(nf)).long(),
                          max=units.shape[1] - 1)
        logits = hubert_cpu.unet_head_forward(ua, usd_, units[:, idx])
        torch.Tensor.float = orig_float
        logits = logits.float()
        ph, ph_iv, w, w_iv, conf, ex = odec.decode(vocab, logits[:, :, 2:], logits[:, :, 0], n44 / 44100,
                                                   ph_seqs[b], word_seqs[b], p2ws[b])
        ids = np.array([vocab["vocab"][p] for p in ph_seqs[b]])
        if dtype == torch.float64:
            torch.Tensor.float = lambda t, *a, **k: t.double()
        outs.append((ex["ph_prob_log"][:, ids], ex["tint"], float(units.abs().max())))
    hubert_cpu.F = F
    torch.Tensor.float = orig_float
    return outs


def main():
    torch.set_num_threads(8)
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    vocab = yaml.safe_load(ckpt["hyper_parameters"]["vocab_text"])
    B = int(os.environ.get("SIM_B", 3))
    wav, ph_seqs, word_seqs, p2ws = bench.make_inputs(B, 10.0, 30, 777)
    arch = synth.arch_cnhubert_base()
    sd = synth.synth_hubert_state_dict(arch, seed=0)
    ua = synth.UNetArch(vocab_size=vocab["vocab_size"])
    usd = {k: v.numpy() for k, v in ckpt["state_dict"].items()}
    args = (wav, ph_seqs, word_seqs, p2ws, vocab, sd, usd, ua, arch)
    ref64 = run(None, torch.float64, *args)
    ref32 = run(None, torch.float32, *args)
    for name, outs in [("f32", ref32)] + [(m, run(m, torch.float32, *args)) for m in ("bf16x3", "bf16x6", "fp16x3")]:
        e64 = max(float(np.abs(o[0] - r[0]).max()) for o, r in zip(outs, ref64))
        e32 = max(float(np.abs(o[0] - r[0]).max()) for o, r in zip(outs, ref32))
        same = all(np.array_equal(o[1], r[1]) for o, r in zip(outs, ref32))
        print(f"{name:7s} max|dlogp| vs f64 {e64:.2e}  vs f32 oracle {e32:.2e}  boundaries==f32 oracle: {same}",
              flush=True)


if __name__ == "__main__":
    main()
