"""The reference-API surface of the drop-in, called the way the reference calls it, against the CPU
oracle:

* ``ForcedAlignmentTask.predict_step((wav_path, ph_seq, word_seq, ph_idx_to_word_idx), idx)`` — the reference's
  per-utterance driver (networks/task/forced_alignment.py:154-186): WAV file -> 7-tuple.
* ``UnitsEncoder.encode(audio[B, N], sample_rate, hop_size) -> [B, C, T]`` (tools/encoder.py:36-60).
* ``ForcedAlignmentTask.forward(x[B, T, C]) -> (ph_frame_logits, ph_edge_logits, ctc_logits)``
  (forced_alignment.py:284-292).
* The split-f16 range guard on forward()/encode(): an out-of-range activation gives the f32 result, never a
  non-finite one, and leaves no raised flag behind to trigger a redo of the next batch.
"""
import numpy as np
import pytest

from oracle_path import LOGPROB_TOL, OraclePath

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _task(encoder="cnhubert"):
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    ckpt = synth_checkpoint(encoder=encoder, model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device="cuda")
    task.on_predict_start()
    return task, ckpt


def test_predict_step_on_wav_file_vs_oracle(tmp_path):
    import bench
    from hubertfa_amd.wav_io import read_wav, write_wav
    task, ckpt = _task()
    wav, ph, ws, pw = bench.make_inputs(1, 6.5, 20, 2024)
    path = tmp_path / "utt.wav"
    write_wav(path, wav[0], 16000)
    out = task.predict_step((path, ph[0], ws[0], pw[0]), 0)
    assert len(out) == 7
    wav_path, wav_length, conf, ph_pred, ph_iv, w_pred, w_iv = out
    assert wav_path == path
    x, sr = read_wav(path)                                    # the quantised samples the reference reads
    assert sr == 16000
    n44 = -(-441 * x.shape[1] // 160)
    assert abs(wav_length - n44 / 44100) < 1e-12
    ref_ph, ref_ph_iv, ref_w, ref_w_iv, ref_conf, ex = OraclePath(ckpt).align(x[0], ph[0], ws[0], pw[0])
    assert list(ph_pred) == list(ref_ph) and list(w_pred) == list(ref_w)
    np.testing.assert_allclose(ph_iv, ref_ph_iv, atol=1e-5)
    np.testing.assert_allclose(w_iv, ref_w_iv, atol=1e-5)
    np.testing.assert_allclose(conf, ref_conf, rtol=1e-4)
    # boundary frames: predict_step's decoder attributes are not kept (batched path), so compare via intervals'
    # integer part reconstructed by the decoder on the same lattice: re-run the batched path for the raw arrays
    dev_out = task.align_batch(task.upload(x[:1]), ph, ws, pw, wav_sr=16000, host=False)
    r = task.decoder.assemble(dev_out, ph, ws, pw)[0]
    assert np.array_equal(r["ph_time_int"], ex["tint"]) and np.array_equal(r["ph_idx_seq"], ex["idx"])


def test_units_encoder_encode_shape_and_values():
    import bench
    task, ckpt = _task()
    enc = task.unitsEncoder
    wav, *_ = bench.make_inputs(2, 3.0, 4, 31)
    x44 = task.upsampler(16000)(torch.from_numpy(wav).cuda())          # load_wav's 16k -> 44.1k
    units = enc.encode(x44, 44100, 512)
    n_frames = x44.shape[-1] // 512 + 1
    assert units.shape == (2, 768, n_frames)                             # [B, C, T] like the reference
    orc = OraclePath(ckpt)
    for b in range(2):
        n44, u = orc.units(wav[b])
        idx = torch.clamp(torch.round(((512 / 44100) / (320 / 16000)) * torch.arange(n_frames)).long(),
                          max=u.shape[1] - 1)
        ref = u[0, idx].T.numpy()
        err = float(np.abs(units[b].cpu().numpy() - ref).max())
        assert err < 2e-3, f"encode row {b}: max error {err:.2e}"


def test_forward_logits_vs_oracle():
    from oracle import hubert_cpu
    from hubertfa_amd import synth
    task, ckpt = _task()
    T = 431                                                               # config 1's frame count (5 s)
    x = synth.rng(77).standard_normal((2, T, 768)).astype(np.float32)
    frame, edge, ctc = task.forward(torch.from_numpy(x))
    assert frame.shape == (2, T, 63) and edge.shape == (2, T) and ctc.shape == (2, T, 63)
    orc = OraclePath(ckpt)
    Tp = task.head.padded_len(T)
    xp = np.zeros((2, Tp, 768), np.float32)
    xp[:, :T] = x
    ref = hubert_cpu.unet_head_forward(orc.ua, orc.usd, torch.from_numpy(xp))[:, :T].numpy()
    assert float(np.abs(frame.cpu().numpy() - ref[:, :, 2:]).max()) < 2e-4
    assert float(np.abs(edge.cpu().numpy() - ref[:, :, 0]).max()) < 2e-4
    ref_ctc = np.concatenate([ref[:, :, 1:2], ref[:, :, 3:]], -1)
    assert float(np.abs(ctc.cpu().numpy() - ref_ctc).max()) < 2e-4


def test_forward_range_guard():
    """An out-of-range head activation: forward() returns the f32-GEMM logits (finite), clears the flag."""
    from hubertfa_amd import synth
    task, _ = _task()
    x = torch.from_numpy(synth.rng(5).standard_normal((1, 128, 768)).astype(np.float32))
    blk = task.head.encoders[0][0]
    blk.gn[1][3] = 1.0e5                    # GroupNorm beta of one hidden channel: its conv2 input ~1e5
    got = task.forward(x)
    assert task.head.precision == "split" and int(task.head.flag.item()) == 0
    task.head.precision = "f32"
    ref = task.forward(x)
    task.head.precision = "split"
    for a, b in zip(got, ref):
        assert torch.isfinite(a).all() and torch.equal(a, b)


def test_encode_range_guard_and_no_stale_flag():
    """An out-of-range encoder activation: encode() returns the f32 units and leaves the flag clear, so the next
    batch through the pipelined path is not re-run."""
    import bench
    from hubertfa_amd import ops
    task, _ = _task()
    enc = task.unitsEncoder
    wav, ph, ws, pw = bench.make_inputs(1, 2.0, 6, 8)
    x = torch.from_numpy(wav).cuda()
    beta = enc.model.conv_ln[0][1]
    saved = float(beta[5])
    beta[5] = 1.0e5
    got = enc.encode(x, 16000, 320)
    assert enc.model.precision == "split" and int(ops.split_flag(x.device).item()) == 0
    enc.model.precision = "f32"
    ref = enc.encode(x, 16000, 320)
    enc.model.precision = "split"
    assert torch.isfinite(got).all() and torch.equal(got, ref)
    beta[5] = saved
    calls = []
    redo = task._align_f32
    task._align_f32 = lambda *a: calls.append(1) or redo(*a)
    task.decoder.assemble(task.submit(x, ph, ws, pw, wav_sr=16000), ph, ws, pw)
    assert calls == []


def test_logprob_tolerance_is_the_north_star():
    assert LOGPROB_TOL == 1e-4
