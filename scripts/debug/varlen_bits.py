"""Debug: per-row bit equality of a variable-length batch vs one-utterance runs through the split encoder,
layer by layer (GPU box).  python scripts/debug/varlen_bits.py"""
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
SECS = (2.0, 2.0, 3.5, 2.7, 1.3)
wavs = [synth.synth_audio(int(s * 16000), seed=i) for i, s in enumerate(SECS)]
N = max(len(w) for w in wavs)
batch = np.zeros((len(wavs), N), np.float32)
for i, w in enumerate(wavs):
    batch[i, :len(w)] = w
for nl in (0, 1, 2, 12):
    ub = enc(torch.from_numpy(batch).to(d), n_layers=nl, lengths=[len(w) for w in wavs])
    for i, w in enumerate(wavs):
        u1 = enc(torch.from_numpy(w)[None].to(d), n_layers=nl)
        L = u1.shape[1]
        same = torch.equal(ub[i, :L], u1[0])
        print(f"layers={nl} row {i}: L={L} equal={same} maxdiff={float((ub[i, :L] - u1[0]).abs().max()):.3e}",
              flush=True)
print("flag", int(ops.split_flag(d).item()))
