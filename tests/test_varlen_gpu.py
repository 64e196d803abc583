"""Variable-length batches: every row of a zero-padded batch with per-row lengths aligns exactly as the same
utterance alone (the reference runs one utterance at a time, so "alone" is the reference's own geometry).

Covers the three encoder layouts (cnhubert GroupNorm-conv post-LN, cnhubert-large LN-conv pre-LN, hubertsoft with
its 40-sample wave padding), the resamplers' tails, conv0's per-row GroupNorm statistics, the positional conv's
padding, per-row attention lengths, the per-row frame gather and the UNet's per-level masks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

LENGTHS = [48000, 75211, 80000, 35330]          # 16 kHz samples: 3.0, 4.7, 5.0, 2.2 s


@pytest.mark.parametrize("encoder", ["cnhubert", "hubertsoft", "cnhubert-large"])
def test_variable_length_batch_equals_alone(encoder):
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(encoder=encoder, model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    task.on_predict_start()
    B = len(LENGTHS)
    wav, ph, ws, pw = bench.make_inputs(B, max(LENGTHS) / 16000, 8, 4242)
    for b, n in enumerate(LENGTHS):
        wav[b, n:] = 0.0
    batched = task.align_batch(torch.from_numpy(wav).to(dev), ph, ws, pw, wav_sr=16000, host=False,
                               lengths=LENGTHS)
    res_b = task.decoder.assemble(batched, ph, ws, pw)
    pl_b = batched["lattice"]["prob_log"].cpu().numpy()
    for b, n in enumerate(LENGTHS):
        alone = task.align_batch(torch.from_numpy(wav[b:b + 1, :n].copy()).to(dev), ph[b:b + 1], ws[b:b + 1],
                                 pw[b:b + 1], wav_sr=16000, host=False)
        res_a = task.decoder.assemble(alone, ph[b:b + 1], ws[b:b + 1], pw[b:b + 1])[0]
        pl_a = alone["lattice"]["prob_log"].cpu().numpy()[0]
        T, S = res_a["T"], len(ph[b])
        assert res_b[b]["T"] == T
        assert np.array_equal(pl_b[b, :T, :S], pl_a[:T, :S]), \
            f"{encoder} row {b}: lattice differs (max {np.abs(pl_b[b, :T, :S] - pl_a[:T, :S]).max():.2e})"
        assert np.array_equal(res_b[b]["ph_idx_seq"], res_a["ph_idx_seq"])
        assert np.array_equal(res_b[b]["ph_time_int"], res_a["ph_time_int"])
        assert np.array_equal(res_b[b]["frame_confidence"], res_a["frame_confidence"])
        assert list(res_b[b]["word_seq"]) == list(res_a["word_seq"])
