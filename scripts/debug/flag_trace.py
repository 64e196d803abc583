"""Debug: which split producer raises the range flag on a variable-length batch (GPU box)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hubertfa_amd import synth, ops  # noqa: E402
from hubertfa_amd.hubert import HubertEncoder  # noqa: E402

d = torch.device("cuda")
arch = synth.arch_cnhubert_base()
sd = synth.synth_hubert_state_dict(arch, seed=0)
enc = HubertEncoder(arch, sd, d)
flag = ops.split_flag(d)
orig_call = ops._lib.call


def traced(name, *a):
    r = orig_call(name, *a)
    torch.cuda.synchronize()
    if int(flag.item()):
        print("FLAG raised by", name, flush=True)
        flag.zero_()
    return r


ops._lib.call = traced
SECS = (2.0, 2.0, 3.5, 2.7, 1.3)
wavs = [synth.synth_audio(int(s * 16000), seed=i) for i, s in enumerate(SECS)]
N = max(len(w) for w in wavs)
batch = np.zeros((len(wavs), N), np.float32)
for i, w in enumerate(wavs):
    batch[i, :len(w)] = w
print("batched")
enc(torch.from_numpy(batch).to(d), lengths=[len(w) for w in wavs])
print("single")
for w in wavs:
    enc(torch.from_numpy(w)[None].to(d))
print("done")
