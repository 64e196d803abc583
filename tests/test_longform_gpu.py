"""Config 5 (long-form, unchunked): 1 x 300 s through the whole GPU path.

The reference encodes each wav whole (O(L^2) attention); this is the unchunked parity anchor
for future chunked streaming.  Checked: geometry (L = 14 999 Hubert frames, T = 25 839 DP frames,
S = 1 801 states), a complete monotone path covering every phone, and DP/backtrack bit-exactness against the C
oracle on the GPU-produced lattice (size-independent property: same lattice -> same path); then the per-frame
log-probs of the whole 300 s utterance (attention over 15 k keys: 59 key tiles of online softmax per query) against
the pinned CPU oracle at the north-star 1e-4, with the oracle's own boundaries bit-exact; and the chunked path
(20 s windows) at the same length by its properties.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
torch = pytest.importorskip("torch")


def test_300s_unchunked_path():
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    from oracle import decode as od
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    wav, ph_seqs, word_seqs, p2ws = bench.make_inputs(1, 300.0, 600, 4242)
    task.on_predict_start()
    dev_out = task.align_batch(torch.from_numpy(wav).to(dev), ph_seqs, word_seqs, p2ws, wav_sr=16000, host=False)
    res = task.decoder.assemble(dev_out, ph_seqs, word_seqs, p2ws)[0]
    S = len(ph_seqs[0])
    assert S == 1801 and res["T"] == 25839
    assert len(res["word_seq"]) == 600 and list(res["word_seq"]) == word_seqs[0]
    iv = res["ph_intervals"]
    assert np.all(np.diff(iv[:, 0]) >= 0) and iv[-1, 1] <= 300.0 + 1e-6
    # same lattice through the pinned CPU oracle -> identical path
    lat = dev_out["lattice"]
    T = res["T"]
    ids = np.array([task.vocab["vocab"][p] for p in ph_seqs[0]])
    pl = lat["prob_log"][0, :T, :S].cpu().numpy()
    E = lat["edge_log"][0, :T].cpu().numpy()
    nE = lat["not_edge_log"][0, :T].cpu().numpy()
    curr = np.full(S, -np.inf)
    dp = np.full((T, S), -np.inf, np.float32)
    bt = np.full((T, S), -1, np.int32)
    dp[0, 0] = pl[0, 0]
    curr[0] = pl[0, 0]
    if ids[0] == 0:
        dp[0, 1] = pl[0, 1]
        curr[1] = pl[0, 1]
    d, b, c = od.forward_pass(T, S, pl, nE, E, curr, dp, bt, ids, 2)
    i_ref, t_ref, _ = od.backtrack(d, b, ids)
    assert np.array_equal(res["ph_idx_seq"], i_ref) and np.array_equal(res["ph_time_int"], t_ref)


@pytest.mark.timeout(900)
def test_300s_unchunked_logprobs_vs_oracle():
    """The whole 300 s utterance through the CPU oracle chain (tests/oracle_path.py: resamplers -> Hubert base
    12L unchunked -> grid gather -> UNet + head -> decode with the C Viterbi; ~1 min on 16 host threads, ~21 GB
    of attention scores): per-frame log-probs within 1e-4, phone path and boundary frames bit-exact."""
    import bench
    from oracle_path import OraclePath
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    wav, ph_seqs, word_seqs, p2ws = bench.make_inputs(1, 300.0, 600, 4242)
    task.on_predict_start()
    dev_out = task.align_batch(torch.from_numpy(wav).to(dev), ph_seqs, word_seqs, p2ws, wav_sr=16000, host=False)
    res = task.decoder.assemble(dev_out, ph_seqs, word_seqs, p2ws)[0]
    lattice = dev_out["lattice"]["prob_log"][0].cpu().numpy()
    assert res["T"] == 25839 and len(ph_seqs[0]) == 1801
    err = OraclePath(ckpt).check(res, lattice, wav[0], ph_seqs[0], word_seqs[0], p2ws[0], tag="300 s")
    print(f"300 s unchunked: per-frame log-prob error vs the oracle {err:.2e}")


def test_300s_chunked_properties():
    """The chunked long-form path at full length (20 s windows, 100-frame overlap, one variable-length batch):
    the same DP grid as the unchunked run (T = 25 839), finite lattice, strictly increasing boundaries starting at
    frame 0, every word of the transcript emitted in order, intervals inside the utterance."""
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    dev = torch.device("cuda")
    ckpt = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ckpt["hyper_parameters"], state_dict=ckpt["state_dict"], device=dev)
    wav, ph_seqs, word_seqs, p2ws = bench.make_inputs(1, 300.0, 600, 4242)
    task.on_predict_start()
    dev_out = task.align_batch(torch.from_numpy(wav).to(dev), ph_seqs, word_seqs, p2ws, wav_sr=16000, host=False,
                               chunk_seconds=20.0)
    T = dev_out["T"][0]
    pl = dev_out["lattice"]["prob_log"][0, :T, :len(ph_seqs[0])]
    assert bool(torch.isfinite(pl).all())
    res = task.decoder.assemble(dev_out, ph_seqs, word_seqs, p2ws)[0]
    assert res["T"] == T == 25839
    tint = res["ph_time_int"]
    assert tint[0] == 0 and np.all(np.diff(tint) > 0) and tint[-1] < T
    assert np.all(np.diff(res["ph_idx_seq"]) > 0)
    assert list(res["word_seq"]) == word_seqs[0]
    iv = res["ph_intervals"]
    assert np.all(iv[:, 1] > iv[:, 0]) and iv[0, 0] >= 0 and iv[-1, 1] <= 300.0 + 1e-6
    assert np.all(np.diff(iv[:, 0]) > 0)
    # quantified against the anchor, the unchunked run (bench.chunk_agreement; the same numbers go into the
    # config-5c bench line): printed, and bounded loosely -- random weights, so only gross breakage is asserted
    agr = bench.chunk_agreement(task, torch.from_numpy(wav).to(dev), ph_seqs, word_seqs, p2ws, 20.0)["utterances"][0]
    print(f"chunked vs unchunked at 300 s: {agr}")
    assert agr["phones_in_both"] > 0 and agr["within_5"] is not None and np.isfinite(agr["max_logprob_diff"])
