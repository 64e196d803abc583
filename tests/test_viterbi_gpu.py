"""GPU parity of the alignment decoder kernels against the reference goldens and the C oracle.

Bit-exact bar: dp, backtrack codes, curr_ph_max_prob_log, ph_idx_seq, ph_time_int (integer/index work).
Tolerances: frame_confidence rtol 2e-6 (expf vs numpy's float32 exp); per-frame log-probs atol 1e-5
(north star allows 1e-4).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _cases():
    z = np.load(os.path.join(GOLDEN, "dp_cases.npz"))
    return z, int(z["n"])


def _lattice(z, c):
    from oracle import decode as od
    p = f"c{c}_"
    ids = z[p + "ids"].astype(np.int64)
    return ids, od.lattice_inputs(ids, z[p + "ph_prob_log"], z[p + "edge_prob"])


def test_forward_batched_bit_exact():
    from hubertfa_amd import ops
    z, n = _cases()
    lats = [_lattice(z, c) for c in range(n)]
    B = n
    Tmax = max(l[1][4].shape[0] for l in lats)
    Smax = max(l[1][4].shape[1] for l in lats)
    pl = np.zeros((B, Tmax, Smax), np.float32)
    E = np.zeros((B, Tmax), np.float32)
    nE = np.zeros((B, Tmax), np.float32)
    cu = np.full((B, Smax), -np.inf)
    dp = np.full((B, Tmax, Smax), -np.inf, np.float32)
    ids = np.zeros((B, Smax), np.int32)
    Ts, Ss = [], []
    for b, (i, (p, e, ne, c0, d0, _, _)) in enumerate(lats):
        T, S = d0.shape
        Ts.append(T); Ss.append(S)
        pl[b, :T, :S] = p; E[b, :T] = e; nE[b, :T] = ne; cu[b, :S] = c0; dp[b, :T, :S] = d0; ids[b, :S] = i
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(a).to(dev)
    dp_t, cu_t = t(dp), t(cu)
    bt_t = torch.full((B, Tmax, Smax), -1, dtype=torch.int8, device=dev)
    T_t = torch.tensor(Ts, dtype=torch.int32, device=dev)
    S_t = torch.tensor(Ss, dtype=torch.int32, device=dev)
    ids_t = t(ids)
    ops.viterbi_forward(t(pl), t(nE), t(E), cu_t, dp_t, bt_t, ids_t, T_t, S_t)
    dp_h, bt_h, cu_h = dp_t.cpu().numpy(), bt_t.cpu().numpy(), cu_t.cpu().numpy()
    for b in range(B):
        p = f"c{b}_"
        T, S = Ts[b], Ss[b]
        assert np.array_equal(dp_h[b, :T, :S].view(np.int32), z[p + "dp"].view(np.int32)), f"dp case {b}"
        assert np.array_equal(bt_h[b, 1:T, :S], z[p + "bt"][1:]), f"bt case {b}"
        assert np.array_equal(cu_h[b, :S].view(np.int64), z[p + "curr"].view(np.int64)), f"curr case {b}"
    # backtrack on the same device buffers
    idx, tint, nn, fc = ops.viterbi_backtrack(dp_t, bt_t, ids_t, T_t, S_t)
    idx, tint, nn, fc = idx.cpu().numpy(), tint.cpu().numpy(), nn.cpu().numpy(), fc.cpu().numpy()
    for b in range(B):
        p = f"c{b}_"
        k = nn[b]
        assert np.array_equal(idx[b, :k], z[p + "ph_idx_seq"]), f"ph_idx_seq case {b}"
        assert np.array_equal(tint[b, :k], z[p + "ph_time_int"]), f"ph_time_int case {b}"
        np.testing.assert_allclose(fc[b, :Ts[b]], z[p + "frame_confidence"], rtol=2e-6, atol=0, equal_nan=True)


def test_forward_step_ranges_bit_exact():
    """hfa_viterbi_forward_steps: the DP cut into consecutive time-step ranges (the pipeline runs a long lattice in
    pieces beside the next batch's attention kernels) gives the one-call bits.  The 45 reference lattices batched
    (ragged T: cuts fall past some utterances' ends, one range is a single step), and a multi-wave lattice
    (S = 1801, 8 waves) in 12 ranges against the pinned C oracle."""
    from hubertfa_amd import ops
    from oracle import decode as od
    z, n = _cases()
    lats = [_lattice(z, c) for c in range(n)]
    B = n
    Tmax = max(l[1][4].shape[0] for l in lats)
    Smax = max(l[1][4].shape[1] for l in lats)
    pl = np.zeros((B, Tmax, Smax), np.float32)
    E = np.zeros((B, Tmax), np.float32)
    nE = np.zeros((B, Tmax), np.float32)
    cu = np.full((B, Smax), -np.inf)
    dp = np.full((B, Tmax, Smax), -np.inf, np.float32)
    ids = np.zeros((B, Smax), np.int32)
    Ts, Ss = [], []
    for b, (i, (p, e, ne, c0, d0, _, _)) in enumerate(lats):
        T, S = d0.shape
        Ts.append(T); Ss.append(S)
        pl[b, :T, :S] = p; E[b, :T] = e; nE[b, :T] = ne; cu[b, :S] = c0; dp[b, :T, :S] = d0; ids[b, :S] = i
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dp_t, cu_t = t(dp), t(cu)
    bt_t = torch.full((B, Tmax, Smax), -1, dtype=torch.int8, device=dev)
    T_t = torch.tensor(Ts, dtype=torch.int32, device=dev)
    S_t = torch.tensor(Ss, dtype=torch.int32, device=dev)
    cuts = sorted({1, 37, 200, 201, min(Ts) + 3, Tmax // 2, Tmax})
    for a, c in zip(cuts[:-1], cuts[1:]):
        ops.viterbi_forward(t(pl), t(nE), t(E), cu_t, dp_t, bt_t, t(ids), T_t, S_t, steps=(a, c))
    dp_h, bt_h, cu_h = dp_t.cpu().numpy(), bt_t.cpu().numpy(), cu_t.cpu().numpy()
    for b in range(B):
        p = f"c{b}_"
        T, S = Ts[b], Ss[b]
        assert np.array_equal(dp_h[b, :T, :S].view(np.int32), z[p + "dp"].view(np.int32)), f"dp case {b}"
        assert np.array_equal(bt_h[b, 1:T, :S], z[p + "bt"][1:]), f"bt case {b}"
        assert np.array_equal(cu_h[b, :S].view(np.int64), z[p + "curr"].view(np.int64)), f"curr case {b}"

    T, S, V = 3000, 1801, 63
    r = np.random.default_rng(5)
    ids1 = r.integers(1, V, S).astype(np.int64)
    ids1[::3] = 0
    ids1[0] = ids1[-1] = 0
    lp = torch.log_softmax(torch.from_numpy((3 * r.standard_normal((T, V))).astype(np.float32)), -1).numpy()
    pl1, E1, nE1, cu1, dp1, bt1, pad = od.lattice_inputs(ids1, lp, np.clip(r.uniform(-0.2, 1.2, T), 0, 1))
    d_ref, b_ref, c_ref = od.forward_pass(T, S, pl1, nE1, E1, cu1.copy(), dp1.copy(), bt1.copy(), ids1, pad)
    P = -(-S // 8) * 8

    def padded(a, fill):
        out = np.full(a.shape[:-1] + (P,), fill, dtype=a.dtype)
        out[..., :S] = a
        return out
    t1 = lambda a: t(a)[None]
    dp_t, cu_t = t1(padded(dp1, -np.inf)), t1(padded(cu1, -np.inf))
    bt_t = torch.full((1, T, P), -1, dtype=torch.int8, device=dev)
    Tt, St = (torch.tensor([v], dtype=torch.int32, device=dev) for v in (T, S))
    edges = np.linspace(1, T, 13).astype(int)
    for a, c in zip(edges[:-1], edges[1:]):
        ops.viterbi_forward(t1(padded(pl1, 0.0)), t1(nE1), t1(E1), cu_t, dp_t, bt_t, t1(padded(ids1.astype(np.int32), 0)),
                            Tt, St, steps=(a, c))
    assert np.array_equal(dp_t[0, :, :S].cpu().numpy().view(np.int32), d_ref.view(np.int32))
    assert np.array_equal(bt_t[0, 1:, :S].cpu().numpy().astype(np.int32), b_ref[1:])
    assert np.array_equal(cu_t[0, :S].cpu().numpy().view(np.int64), c_ref.view(np.int64))


@pytest.mark.parametrize("T,S", [(300, 200), (900, 1801)])
def test_forward_f64_curr_bit_exact(T, S):
    """The DP runs curr in f32 when every incoming value is an f32 one (the lattice prologue's, and everything the DP
    itself writes); a caller's curr with f64-only values (forward_pass takes any float64 array) takes the f64 form:
    both bit-exact with the pinned C oracle, on a one-wave and a multi-wave lattice."""
    from hubertfa_amd import ops
    from oracle import decode as od
    r = np.random.default_rng(T + S)
    V = 63
    ids = r.integers(1, V, S).astype(np.int64)
    ids[::3] = 0
    ids[0] = ids[-1] = 0
    lp = torch.log_softmax(torch.from_numpy((3 * r.standard_normal((T, V))).astype(np.float32)), -1).numpy()
    pl, E, nE, cu, dp, bt, pad = od.lattice_inputs(ids, lp, np.clip(r.uniform(-0.2, 1.2, T), 0, 1))
    P = -(-S // 8) * 8

    def padded(a, fill):
        out = np.full(a.shape[:-1] + (P,), fill, dtype=a.dtype)
        out[..., :S] = a
        return out
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))[None].to(dev)
    for label, c0 in (("f32 values", cu), ("f64 values", -5.0 * r.random(S) - 1e-9 * r.random(S))):
        assert (label == "f32 values") == bool(np.all(c0.astype(np.float32).astype(np.float64) == c0))
        d_ref, b_ref, c_ref = od.forward_pass(T, S, pl, nE, E, c0.copy(), dp.copy(), bt.copy(), ids, pad)
        dp_t, cu_t = t(padded(dp, -np.inf)), t(padded(c0, -np.inf))
        bt_t = torch.full((1, T, P), -1, dtype=torch.int8, device=dev)
        Tt, St = (torch.tensor([v], dtype=torch.int32, device=dev) for v in (T, S))
        ops.viterbi_forward(t(padded(pl, 0.0)), t(nE), t(E), cu_t, dp_t, bt_t, t(padded(ids.astype(np.int32), 0)),
                            Tt, St)
        assert np.array_equal(dp_t[0, :, :S].cpu().numpy().view(np.int32), d_ref.view(np.int32)), label
        assert np.array_equal(bt_t[0, 1:, :S].cpu().numpy().astype(np.int32), b_ref[1:]), label
        assert np.array_equal(cu_t[0, :S].cpu().numpy().view(np.int64), c_ref.view(np.int64)), label


@pytest.mark.parametrize("T,S,force_k,pitch8", [(700, 300, 0, False), (1200, 513, 0, False), (3000, 1801, 0, False),
                                                (2500, 4100, 0, False), (4200, 8000, 0, False),
                                                (3000, 1801, 0, True), (1200, 513, 2, True), (3000, 1801, 2, True),
                                                (3000, 1801, 4, True), (3000, 1801, 8, True), (2500, 4100, 4, False),
                                                (700, 300, 2, False), (70000, 61, 0, True), (65537, 300, 0, False),
                                                (65536, 31, 0, True), (64000, 31, 0, True), (2000, 9000, 0, True),
                                                (1500, 20000, 0, False), (1200, 32767, 0, True), (9000, 8500, 2, False),
                                                (861, 91, 1, True), (861, 91, 5, True), (1000, 77, 1, False)])
def test_forward_many_states_vs_oracle(T, S, force_k, pitch8):
    """Single- and multi-wave DP variants (S up to 8192; 2/4/8 states per lane, the short emission rings 1/5; scalar
    and vector state pitch), the
    segmented form past 8192 states (up to the backtrack's 32767), all bit-exact with the pinned C oracle, and the
    windowed backtrack with it (T > 64000: the path kept in global memory instead of LDS; the reference takes any T
    and S)."""
    from hubertfa_amd import ops, _lib
    from oracle import decode as od
    r = np.random.default_rng(T * 7 + S)
    V = 63
    ids = r.integers(1, V, S).astype(np.int64)
    ids[::3] = 0
    ids[0] = ids[-1] = 0
    logits = (3 * r.standard_normal((T, V))).astype(np.float32)
    ph_prob_log = torch.log_softmax(torch.from_numpy(logits), -1).numpy()
    edge = np.clip(r.uniform(-0.2, 1.2, T), 0, 1)
    pl, E, nE, cu, dp, bt, pad = od.lattice_inputs(ids, ph_prob_log, edge)
    d_ref, b_ref, c_ref = od.forward_pass(T, S, pl, nE, E, cu.copy(), dp.copy(), bt.copy(), ids, pad)
    P = -(-S // 8) * 8 if pitch8 else S                 # state pitch (the decoder pads it to 8)

    def padded(a, fill):
        out = np.full(a.shape[:-1] + (P,), fill, dtype=a.dtype)
        out[..., :S] = a
        return out
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))[None].to(dev)
    dp_t, cu_t = t(padded(dp, -np.inf)), t(padded(cu, -np.inf))
    bt_t = torch.full((1, T, P), -1, dtype=torch.int8, device=dev)
    ids_t = t(padded(ids.astype(np.int32), 0))
    Tt = torch.tensor([T], dtype=torch.int32, device=dev)
    St = torch.tensor([S], dtype=torch.int32, device=dev)
    _lib.lib().hfa_viterbi_tuning(force_k)
    try:
        ops.viterbi_forward(t(padded(pl, 0.0)), t(nE), t(E), cu_t, dp_t, bt_t, ids_t, Tt, St)
    finally:
        _lib.lib().hfa_viterbi_tuning(0)
    assert np.array_equal(dp_t[0, :, :S].cpu().numpy().view(np.int32), d_ref.view(np.int32))
    assert np.array_equal(bt_t[0, 1:, :S].cpu().numpy().astype(np.int32), b_ref[1:])
    assert np.array_equal(cu_t[0, :S].cpu().numpy().view(np.int64), c_ref.view(np.int64))
    idx, tint, n, fc = ops.viterbi_backtrack(dp_t, bt_t, ids_t, Tt, St)
    i_ref, t_ref, f_ref = od.backtrack(d_ref, b_ref, ids)
    k = int(n[0])
    assert np.array_equal(idx[0, :k].cpu().numpy(), i_ref) and np.array_equal(tint[0, :k].cpu().numpy(), t_ref)
    np.testing.assert_allclose(fc[0].cpu().numpy(), f_ref, rtol=2e-6, atol=0, equal_nan=True)


def test_reference_api_forward_pass_and_decode():
    from hubertfa_amd.alignment_decoder import AlignmentDecoder
    z, n = _cases()
    dec = AlignmentDecoder({"vocab": {}, "vocab_size": 63}, {"hop_length": 512, "sample_rate": 44100})
    for c in (0, 7, 28, 33, 35, 36, 38, 40, 42):
        ids, (p, e, ne, c0, d0, b0, pad) = _lattice(z, c)
        T, S = d0.shape
        d, b, cu = AlignmentDecoder.forward_pass(T, S, p, ne, e, c0, d0, b0, ids, pad)
        pre = f"c{c}_"
        assert np.array_equal(d.view(np.int32), z[pre + "dp"].view(np.int32))
        assert np.array_equal(b, z[pre + "bt"].astype(np.int32))
        idx, tint, fc = dec._decode(ids, z[pre + "ph_prob_log"], z[pre + "edge_prob"])
        assert np.array_equal(idx, z[pre + "ph_idx_seq"]) and np.array_equal(tint, z[pre + "ph_time_int"])


def test_prologue_logprobs_within_tolerance():
    from hubertfa_amd import ops
    meta = json.load(open(os.path.join(GOLDEN, "decode_cases.json")))
    zz = np.load(os.path.join(GOLDEN, "decode_cases.npz"))
    vocab = meta["vocab"]
    for ci, case in enumerate(meta["cases"]):
        logits = zz[f"c{ci}_logits"]
        lt = torch.from_numpy(logits)
        ids = np.array([vocab["vocab"][p] for p in case["ph_seq"]], np.int32)
        mask = np.zeros(vocab["vocab_size"]); mask[ids] = 1; mask[0] = 1
        x = lt[:, :, 2:].float() - (torch.from_numpy(mask)[None, None].logical_not() * 1e9).float()
        ref_lp = torch.log_softmax(x, -1)[0].numpy()
        ref_sm = torch.softmax(x, -1)[0].numpy()
        dev = torch.device("cuda")
        lg = lt.to(dev)
        T = logits.shape[1]
        out = ops.lattice_prologue(lg[:, :, 2:], lg[:, :, 0], torch.from_numpy(ids)[None].to(dev),
                                   torch.tensor([T], dtype=torch.int32, device=dev),
                                   torch.tensor([len(ids)], dtype=torch.int32, device=dev), want_frame_probs=True)
        lp = out["ph_prob_log"][0].cpu().numpy()
        allowed = np.zeros(vocab["vocab_size"], bool); allowed[ids] = True; allowed[0] = True
        np.testing.assert_allclose(lp[:, allowed], ref_lp[:, allowed], atol=1e-5, rtol=0)
        np.testing.assert_allclose(out["ph_frame_pred"][0].cpu().numpy(), ref_sm, atol=1e-6, rtol=0)
        np.testing.assert_allclose(out["prob_log"][0].cpu().numpy(), ref_lp[:, ids], atol=1e-5, rtol=0)
        e = ((torch.sigmoid(lt[:, :, 0]) - 0.1) / 0.8).clamp(0, 1)[0].numpy()
        ep = (e + np.concatenate(([0], e[:-1]))).clip(0, 1)
        np.testing.assert_allclose(out["edge_prob"][0].cpu().numpy(), ep, atol=1e-6, rtol=0)
        np.testing.assert_allclose(out["edge_log"][0].cpu().numpy(), np.log(ep + 1e-6).astype(np.float32),
                                   atol=2e-4, rtol=1e-5)


def test_decode_end_to_end_matches_reference():
    from hubertfa_amd.alignment_decoder import AlignmentDecoder
    meta = json.load(open(os.path.join(GOLDEN, "decode_cases.json")))
    zz = np.load(os.path.join(GOLDEN, "decode_cases.npz"))
    dec = AlignmentDecoder(meta["vocab"], {"hop_length": 512, "sample_rate": 44100})
    for ci, case in enumerate(meta["cases"]):
        lt = torch.from_numpy(zz[f"c{ci}_logits"]).cuda()
        ph, ph_iv, w, w_iv, conf = dec.decode(lt[:, :, 2:], lt[:, :, 0], torch.cat([lt[:, :, [1]], lt[:, :, 3:]], -1),
                                              case["wav_length"], case["ph_seq"], case["word_seq"],
                                              case["ph_idx_to_word_idx"])
        assert list(ph) == case["ph_seq_pred"], ci
        assert list(w) == case["word_seq_pred"], ci
        assert np.array_equal(dec.ph_idx_seq, zz[f"c{ci}_ph_idx_seq"]), ci
        assert np.array_equal(dec.ph_time_int_pred, zz[f"c{ci}_ph_time_int"]), ci
        np.testing.assert_allclose(ph_iv, zz[f"c{ci}_ph_intervals"], atol=1e-6)
        np.testing.assert_allclose(w_iv, zz[f"c{ci}_word_intervals"], atol=1e-6)
        np.testing.assert_allclose(conf, case["total_confidence"], rtol=1e-4)


@pytest.mark.parametrize("first_sp", [True, False])
def test_dp_initialisation_in_prologue(first_sp):
    """_decode's initialisation (alignment_decoder.py:244-254) written by the lattice prologue (init_dp) and by
    hfa_viterbi_init: dp[0, 0] = curr[0] = L[0, 0]; with an id-0 first phone and S > 1 also dp[0, 1] = curr[1] =
    L[0, 1]; every other state of row 0 (padding pitch included) and of curr -inf; a row with T = 0 all -inf; S = 1
    keeps only state 0.  Bit-exact, in a batch with unequal T and S."""
    from hubertfa_amd import ops
    dev = torch.device("cuda")
    rng = np.random.default_rng(5)
    V = 20
    Ts, Ss = [7, 0, 5, 9], [5, 3, 1, 2]
    B, Tmax, Smax = len(Ts), max(Ts), 8
    ids = rng.integers(1, V, (B, Smax)).astype(np.int32)
    if first_sp:
        ids[:, 0] = 0
    logits = torch.from_numpy(rng.normal(0, 3, (B, Tmax, V + 2)).astype(np.float32)).to(dev)
    T_t = torch.tensor(Ts, dtype=torch.int32, device=dev)
    S_t = torch.tensor(Ss, dtype=torch.int32, device=dev)
    ids_t = torch.from_numpy(ids).to(dev)
    out = ops.lattice_prologue(logits[:, :, 2:], logits[:, :, 0], ids_t, T_t, S_t, init_dp=True)
    dp2, _, cu2 = ops.viterbi_init(out["prob_log"], ids_t, T_t, S_t)
    pl = out["prob_log"].cpu().numpy()
    for b in range(B):
        exp = np.full(Smax, -np.inf)
        if Ts[b] > 0:
            exp[0] = pl[b, 0, 0]
            if first_sp and Ss[b] > 1:
                exp[1] = pl[b, 0, 1]
        for dp, cu in ((out["dp"], out["curr"]), (dp2, cu2)):
            assert np.array_equal(dp[b, 0].cpu().numpy(), exp.astype(np.float32)), b
            assert np.array_equal(cu[b].cpu().numpy(), exp.astype(np.float32).astype(np.float64)), b
