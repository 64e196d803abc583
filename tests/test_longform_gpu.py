"""Config 5 (long-form, unchunked): 1 x 300 s through the whole GPU path.

The reference encodes each wav whole (O(L^2) attention); this is the unchunked parity anchor
for future chunked streaming.  Checked: geometry (L = 14 999 Hubert frames, T = 25 839 DP frames,
S = 1 801 states), a complete monotone path covering every phone, and DP/backtrack bit-exactness against the C
oracle on the GPU-produced lattice (size-independent property: same lattice -> same path).
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
