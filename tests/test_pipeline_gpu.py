"""End-to-end parity of the GPU infer path (wave -> boundaries) against the CPU oracle at config-2 geometry.

Bars (north star): per-frame log-probs within 1e-4 (fp32); phoneme boundary indices bit-exact with the CPU
reference path.  Boundary exactness is asserted per utterance; the lattice difference that could break it is
bounded by the log-prob check.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _inputs(B, seconds, words, seed0):
    import bench
    return bench.make_inputs(B, seconds, words, seed0)


@pytest.mark.parametrize("precision", ["split", "f32"])
def test_full_path_logprobs_and_boundaries_vs_oracle(precision):
    """Both arithmetic paths meet the bars: the default split-f16 contractions and the f32-MFMA path the range
    guard falls back to."""
    import yaml
    from hubertfa_amd import synth
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    from oracle import decode as odec, hubert_cpu, resample as ores
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    vocab = yaml.safe_load(ckpt["hyper_parameters"]["vocab_text"])
    B = 3
    wav, ph_seqs, word_seqs, p2ws = _inputs(B, 10.0, 30, 777)
    task.on_predict_start()
    task.unitsEncoder.model.precision = task.head.precision = precision
    dev_out = task.align_batch(torch.from_numpy(wav).to(dev), ph_seqs, word_seqs, p2ws, wav_sr=16000, host=False)
    res = task.decoder.assemble(dev_out, ph_seqs, word_seqs, p2ws)
    gpu_pl = dev_out["lattice"]["prob_log"].cpu().numpy()
    arch = synth.arch_cnhubert_base()
    sd = synth.synth_hubert_state_dict(arch, seed=0)
    ua = synth.UNetArch(vocab_size=vocab["vocab_size"])
    usd = {k: v.numpy() for k, v in ckpt["state_dict"].items()}
    worst = 0.0
    for b in range(B):
        x44 = ores.resample(torch.from_numpy(wav[b:b + 1]), 16000, 44100, 6)
        units = hubert_cpu.hubert_forward(arch, sd, ores.resample(x44, 44100, 16000, 128))
        n44 = x44.shape[-1]
        nf = n44 // 512 + 1
        idx = torch.clamp(torch.round(((512 / 44100) / (320 / 16000)) * torch.arange(nf)).long(),
                          max=units.shape[1] - 1)
        logits = hubert_cpu.unet_head_forward(ua, usd, units[:, idx])
        ph, ph_iv, w, w_iv, conf, ex = odec.decode(vocab, logits[:, :, 2:], logits[:, :, 0], n44 / 44100,
                                                   ph_seqs[b], word_seqs[b], p2ws[b])
        T = res[b]["T"]
        assert T == 861
        ids = np.array([vocab["vocab"][p] for p in ph_seqs[b]])
        err = np.abs(gpu_pl[b, :T, :len(ids)] - ex["ph_prob_log"][:, ids]).max()
        worst = max(worst, float(err))
        assert err < 1e-4, f"utt {b}: per-frame log-prob error {err:.2e} > 1e-4"
        assert np.array_equal(res[b]["ph_idx_seq"], ex["idx"]), f"utt {b}: phone path differs"
        assert np.array_equal(res[b]["ph_time_int"], ex["tint"]), f"utt {b}: boundary frames differ"
        assert list(res[b]["ph_seq"]) == list(ph) and list(res[b]["word_seq"]) == list(w)
        np.testing.assert_allclose(res[b]["ph_intervals"], ph_iv, atol=1e-5)
        np.testing.assert_allclose(res[b]["confidence"], conf, rtol=1e-4)
    print(f"[{precision}] max per-frame log-prob error over {B} x 10 s: {worst:.2e}")


def test_smoke_entry():
    from hubertfa_amd.smoke import run_smoke
    r = run_smoke()
    assert r["boundary_exact"] == r["utterances"]


def test_pipelined_long_lattice_dp_held_for_next_encoder():
    """task.submit holds a long lattice's forward DP (defer_dp_frames) and runs it in step ranges beside the next
    batch's attention launches: three 120 s utterances pipelined (the first two held and run under the next
    encoder, the last one flushed by assemble) give the boundaries, confidences and edge terms of align_batch on
    each alone, bit for bit.  Also a held handle assembled before any further submit, and windowed long-form
    (chunk_seconds), which never holds."""
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    task.on_predict_start()
    task.defer_dp_frames = 8192          # (the shipped 16 384 needs ~190 s utterances; the mechanism is the same)
    batches = [_inputs(1, 120.0, 240, 900 + i) for i in range(3)]
    alone = []
    for wav, ph, ws, pw in batches:
        alone.append(task.align_batch(torch.from_numpy(wav).to(dev), ph, ws, pw, wav_sr=16000)[0])
    T = alone[0]["T"]
    assert T >= task.defer_dp_frames and task.dp_ranges(T + 1, 512) > 1
    handles = []
    for wav, ph, ws, pw in batches:
        handles.append(task.submit(torch.from_numpy(wav).to(dev), ph, ws, pw, wav_sr=16000))
        assert "resolve" in handles[-1]                     # held: its DP runs under the next submit / assemble
    got = [task.decoder.assemble(h, *b[1:])[0] for h, b in zip(handles, batches)]
    h = task.submit(torch.from_numpy(batches[0][0]).to(dev), *batches[0][1:], wav_sr=16000)
    got.append(task.decoder.assemble(h, *batches[0][1:])[0])
    for i, (g, a) in enumerate(zip(got, alone + alone[:1])):
        for k in ("ph_idx_seq", "ph_time_int", "frame_confidence", "edge_diff"):
            assert np.array_equal(np.asarray(g[k]), np.asarray(a[k])), f"batch {i}: {k}"
        assert list(g["ph_seq"]) == list(a["ph_seq"])
        assert np.array_equal(np.asarray(g["ph_intervals"]), np.asarray(a["ph_intervals"])), f"batch {i}"
    hc = task.submit(torch.from_numpy(batches[1][0]).to(dev), *batches[1][1:], wav_sr=16000, chunk_seconds=20.0)
    assert "resolve" not in hc
    task.decoder.assemble(hc, *batches[1][1:])


def test_pipelined_submit_matches_align_batch():
    """Four config-2-geometry batches through task.submit (the encoder of batch i+1 beside batch i's head + DP on the
    side stream) give align_batch's boundaries, confidences and edge terms bit for bit, batch by batch."""
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    task.on_predict_start()
    batches = [_inputs(8, 10.0, 30, 300 + 10 * i) for i in range(4)]
    alone = [task.align_batch(torch.from_numpy(w).to(dev), ph, ws, pw, wav_sr=16000) for w, ph, ws, pw in batches]
    handles = [task.submit(torch.from_numpy(w).to(dev), ph, ws, pw, wav_sr=16000) for w, ph, ws, pw in batches]
    for i, (h, b, a) in enumerate(zip(handles, batches, alone)):
        got = task.decoder.assemble(h, *b[1:])
        for u, (g, r) in enumerate(zip(got, a)):
            for k in ("ph_idx_seq", "ph_time_int", "frame_confidence", "edge_diff"):
                assert np.array_equal(np.asarray(g[k]), np.asarray(r[k])), f"batch {i} utt {u}: {k}"


def test_chain_resampler_path_matches_two_stages():
    """The product path's one-pass resampling chain (task.encode_batch -> resample.ChainResampler) against the two
    stages it replaces (task.chain_resample = False), end to end at config-2 geometry with a ragged batch: the
    lattices within the north-star bar of each other (1e-4: the two resamplings differ by f32 rounding, ~2e-5 after
    twelve layers) and every boundary and phone path identical."""
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    task.on_predict_start()
    B = 4
    wav, ph_seqs, word_seqs, p2ws = _inputs(B, 10.0, 30, 4242)
    lens = [wav.shape[1], wav.shape[1] - 16000 * 3 - 7, wav.shape[1] - 12345, wav.shape[1] - 1]
    x = torch.from_numpy(wav).to(dev)
    for b, n in enumerate(lens):
        x[b, n:] = 0
    got = {}
    for chain in (True, False):
        task.chain_resample = chain
        dev_out = task.align_batch(x, ph_seqs, word_seqs, p2ws, wav_sr=16000, lengths=lens, host=False)
        got[chain] = (dev_out["lattice"]["prob_log"].cpu().numpy(), task.decoder.assemble(dev_out, ph_seqs, word_seqs,
                                                                                           p2ws))
    task.chain_resample = True
    (pl_c, res_c), (pl_t, res_t) = got[True], got[False]
    for b in range(B):
        T, S = res_c[b]["T"], len(ph_seqs[b])
        assert T == res_t[b]["T"]
        assert np.abs(pl_c[b, :T, :S] - pl_t[b, :T, :S]).max() < 1e-4, b
        assert np.array_equal(res_c[b]["ph_idx_seq"], res_t[b]["ph_idx_seq"]), b
        assert np.array_equal(res_c[b]["ph_time_int"], res_t[b]["ph_time_int"]), b
