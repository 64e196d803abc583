"""Generate the golden parity fixtures by importing the reference in THIS container (never on the GPU box).

Run:  python tests/golden/gen_golden.py        (needs /root/reference; skips itself otherwise)

The reference is pure Python.  ``numba`` is absent here, so ``numba.jit`` is stubbed as the
identity: numba's scalar typing equals numpy's for this code (f32+f32->f32, f32+f64->f64) and numba performs no
FMA contraction without fastmath, so the pure-Python execution is the reference's arithmetic.

Everything written is DATA (inputs + expected outputs) under tests/golden/.  No reference source is copied.
Weights come from ``hubertfa_amd.synth`` (numpy PCG64) so the GPU box can regenerate them bit-identically.

Reference call sites exercised:
  * tools/alignment_decoder.py:170-230  AlignmentDecoder.forward_pass   -> dp_cases.npz (dp, bt, curr)
  * tools/alignment_decoder.py:232-294  AlignmentDecoder._decode        -> dp_cases.npz (path, confidence)
  * tools/alignment_decoder.py:26-143   AlignmentDecoder.decode         -> decode_cases.npz
  * tools/alignment_decoder.py:152-168 + tools/plot.py  AlignmentDecoder.plot -> plot.json / plot.npz
  * networks/g2p/*.py                   G2P plugins                     -> g2p.json
  * networks/g2p/dictionary_g2p.py over dictionary/*.txt (the CLI's default -d)  -> g2p_dicts.json
  * networks/g2p/*.py + alignment_decoder.py:35 on edge inputs (error types)   -> g2p_edges.json
  * tools/post_processing.py:68-105     post_processing                 -> postproc.json
  * tools/encoder.py:56-59              grid gather index (torch expr)  -> gather_index.npz
  * networks/hubert/model.py            HubertSoft.units                -> hubert_soft.npz
  * transformers HubertModel            cnhubert base / large(reduced)  -> hubert_hf_base.npz / hubert_hf_large.npz
  * networks/layer/backbone/unet.py + head (forced_alignment.py:53-55,284-292) -> unet_head.npz
"""
from __future__ import annotations

import json
import os
import sys
import types
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (ckpt_files)

from hubertfa_amd import synth  # noqa: E402


def _import_reference():
    stub = types.ModuleType("numba")
    stub.jit = lambda f=None, **kw: f if f is not None else (lambda g: g)
    sys.modules.setdefault("numba", stub)
    sys.path.insert(0, REF)


def _phone_seq_ids(r, n_inner: int, V: int, mode: str) -> np.ndarray:
    """A G2P-shaped ph_seq_id: SP(0) framed, phones 1..V-1, SP between words (dictionary_g2p.py:37-39)."""
    if mode == "g2p":
        ids = [0]
        while len(ids) < n_inner - 1:
            for _ in range(int(r.integers(1, 3))):
                ids.append(int(r.integers(1, V)))
            ids.append(0)
        ids = (ids + [0] * n_inner)[:n_inner]
        if n_inner >= 2:
            ids[-1] = 0
        return np.array(ids, dtype=np.int64)
    if mode == "no_sp_start":   # ph_seq_id[0] != 0
        ids = r.integers(1, V, n_inner)
        return ids.astype(np.int64)
    if mode == "double_zero":   # AP/SP both map to id 0 -> consecutive id-0 states
        ids = list(r.integers(0, V, n_inner))
        for i in range(0, n_inner - 1, 5):
            ids[i] = 0
            ids[i + 1] = 0
        return np.array(ids, dtype=np.int64)
    if mode == "random":
        return r.integers(0, V, n_inner).astype(np.int64)
    raise ValueError(mode)


def gen_dp_cases():
    from tools.alignment_decoder import AlignmentDecoder
    import torch

    V = 63
    dec = AlignmentDecoder({"vocab": {}, "vocab_size": V}, {"hop_length": 512, "sample_rate": 44100})
    r = synth.rng(1234)
    specs = []
    for T in (1, 2, 5, 64, 430, 861):
        for S in (1, 2, 3, 31, 91, 256):
            if T * S > 861 * 91 * 1.2 and not (T == 861 and S == 256):
                continue
            specs.append((T, S, "g2p", "normal"))
    specs += [(200, 31, "no_sp_start", "normal"), (300, 46, "double_zero", "normal"),
              (300, 46, "random", "normal"), (120, 31, "g2p", "const"), (64, 31, "g2p", "const_edge"),
              (20, 31, "g2p", "normal"), (30, 91, "g2p", "normal"),  # T < S: infeasible, -inf path
              (861, 91, "g2p", "normal"), (861, 91, "double_zero", "normal"), (430, 46, "g2p", "normal")]
    out = {"n": len(specs)}
    for ci, (T, S, mode, lat) in enumerate(specs):
        ids = _phone_seq_ids(r, S, V, mode)
        if lat == "const":
            logits = np.zeros((T, V), np.float32)
        else:
            logits = (3.0 * r.standard_normal((T, V))).astype(np.float32)
        ph_prob_log = torch.log_softmax(torch.from_numpy(logits), -1).numpy().astype(np.float32)
        if lat == "const_edge":
            edge_prob = np.full(T, 0.5, np.float32)
        else:
            e = r.uniform(-0.2, 1.2, T).astype(np.float32)
            edge_prob = np.clip(e, 0, 1).astype(np.float32)
        # forward_pass inputs exactly as _decode builds them (alignment_decoder.py:239-257)
        prob_log = ph_prob_log[:, ids]
        E = np.log(edge_prob + 1e-6).astype("float32")
        nE = np.log(1 - edge_prob + 1e-6).astype("float32")
        curr = np.full(S, -np.inf)
        dp = np.full((T, S), -np.inf, dtype="float32")
        bt = np.full_like(dp, -1, dtype="int32")
        dp[0, 0] = prob_log[0, 0]
        curr[0] = prob_log[0, 0]
        if ids[0] == 0 and prob_log.shape[-1] > 1:
            dp[0, 1] = prob_log[0, 1]
            curr[1] = prob_log[0, 1]
        pad = 2 if S >= 2 else 1
        dp, bt, curr = AlignmentDecoder.forward_pass(T, S, prob_log, nE, E, curr, dp, bt, ids, pad)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            idx, tint, fconf = dec._decode(ids, ph_prob_log, edge_prob)
        p = f"c{ci}_"
        out[p + "ids"] = ids.astype(np.int32)
        out[p + "ph_prob_log"] = ph_prob_log
        out[p + "edge_prob"] = edge_prob
        out[p + "dp"] = dp
        out[p + "bt"] = bt.astype(np.int8)
        out[p + "curr"] = curr
        out[p + "ph_idx_seq"] = idx.astype(np.int32)
        out[p + "ph_time_int"] = tint.astype(np.int32)
        out[p + "frame_confidence"] = fconf.astype(np.float32)
        print(f"dp case {ci}: T={T} S={S} {mode}/{lat} n_ph={len(idx)}")
    np.savez_compressed(os.path.join(HERE, "dp_cases.npz"), **out)


def gen_decode_cases():
    from tools.alignment_decoder import AlignmentDecoder
    import torch

    vocab = synth.synth_vocab()
    dic = synth.synth_dictionary()
    V = vocab["vocab_size"]
    dec = AlignmentDecoder(vocab, {"hop_length": 512, "sample_rate": 44100})
    r = synth.rng(99)
    cases = []
    arrays = {}
    for ci, (n_words, secs, wl_mode) in enumerate(
            [(15, 5.0, "exact"), (30, 10.0, "exact"), (4, 1.3, "exact"), (8, 2.0, "none"), (12, 3.1, "short")]):
        lab = synth.synth_lab(n_words, dic, seed=100 + ci)
        ph_seq, word_seq, p2w = ["SP"], [], [-1]
        for w in lab.split(" "):
            word_seq.append(w)
            for ph in dic[w]:
                ph_seq.append(ph)
                p2w.append(len(word_seq) - 1)
            ph_seq.append("SP")
            p2w.append(-1)
        if ci == 2:  # an AP (id 0) inside the sequence
            ph_seq.insert(3, "AP")
            p2w.insert(3, -1)
        n44 = int(round(secs * 44100))
        n_frames = n44 // 512 + 1
        logits = (3.0 * r.standard_normal((1, n_frames, V + 2))).astype(np.float32)
        lt = torch.from_numpy(logits)
        frame, edge, ctc = lt[:, :, 2:], lt[:, :, 0], torch.cat([lt[:, :, [1]], lt[:, :, 3:]], dim=-1)
        wav_length = n44 / 44100 if wl_mode == "exact" else (None if wl_mode == "none" else n44 / 44100 - 0.05)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            res = dec.decode(frame, edge, ctc, wav_length, ph_seq, word_seq, p2w)
        ph_pred, ph_int, w_pred, w_int, conf = res
        arrays[f"c{ci}_logits"] = logits
        arrays[f"c{ci}_ph_intervals"] = np.asarray(ph_int, np.float64)
        arrays[f"c{ci}_word_intervals"] = np.asarray(w_int, np.float64)
        arrays[f"c{ci}_ph_idx_seq"] = dec.ph_idx_seq.astype(np.int32)
        arrays[f"c{ci}_ph_time_int"] = dec.ph_time_int_pred.astype(np.int32)
        arrays[f"c{ci}_frame_confidence"] = dec.frame_confidence.astype(np.float32)
        arrays[f"c{ci}_edge_prob"] = dec.edge_prob.astype(np.float32)
        cases.append({"ph_seq": ph_seq, "word_seq": word_seq, "ph_idx_to_word_idx": p2w,
                      "wav_length": wav_length, "ph_seq_pred": [str(x) for x in ph_pred],
                      "word_seq_pred": [str(x) for x in w_pred], "total_confidence": float(conf)})
        print(f"decode case {ci}: S={len(ph_seq)} T={n_frames} conf={conf:.4f}")
    np.savez_compressed(os.path.join(HERE, "decode_cases.npz"), **arrays)
    with open(os.path.join(HERE, "decode_cases.json"), "w") as f:
        json.dump({"vocab": vocab, "cases": cases}, f, indent=1)


def _figure_data(fig) -> dict:
    """What a validation figure shows, as data: the top axes' vertical lines, phone labels and confidence curve, the
    bottom axes' image and curves, the figure size and the subplot layout."""
    ax1, ax2 = fig.axes
    vl = [float(ln.get_xdata()[0]) for ln in ax1.lines if len(ln.get_xdata()) == 2 and ln.get_xdata()[0] ==
          ln.get_xdata()[1]]
    curves1 = [np.asarray(ln.get_ydata(), np.float64) for ln in ax1.lines if len(ln.get_xdata()) != 2]
    return {"vlines": vl,
            "texts": [[t.get_text(), float(t.get_position()[0]), float(t.get_position()[1]), str(t.get_color())]
                      for t in ax1.texts],
            "conf_curve": curves1[0].tolist() if curves1 else [],
            "image_shape": list(ax2.images[0].get_array().shape),
            "bottom_curves": [np.asarray(ln.get_ydata(), np.float64).tolist() for ln in ax2.lines],
            "size": [float(v) for v in fig.get_size_inches()],
            "subplotpars": [fig.subplotpars.left, fig.subplotpars.right, fig.subplotpars.top,
                            fig.subplotpars.bottom, fig.subplotpars.hspace]}


def gen_plot():
    """AlignmentDecoder.plot (tools/alignment_decoder.py:152-168) -> tools/plot.py plot_for_valid on the decode
    cases, with a seeded synthetic mel spectrogram: the plot's inputs (as the decoder derives them) and the figure's
    data (plot.json / plot.npz)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    import torch
    from tools.alignment_decoder import AlignmentDecoder
    d = json.load(open(os.path.join(HERE, "decode_cases.json")))
    z = np.load(os.path.join(HERE, "decode_cases.npz"))
    dec = AlignmentDecoder(d["vocab"], {"hop_length": 512, "sample_rate": 44100})
    captured = {}
    import tools.alignment_decoder as tad
    real = tad.plot_for_valid

    def capture(*args):
        captured["args"] = args
        return real(*args)
    tad.plot_for_valid = capture
    arrays, out = {}, []
    try:
        for ci, c in enumerate(d["cases"]):
            lt = torch.from_numpy(z[f"c{ci}_logits"])
            frame, edge = lt[:, :, 2:], lt[:, :, 0]
            ctc = torch.cat([lt[:, :, [1]], lt[:, :, 3:]], dim=-1)
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                dec.decode(frame, edge, ctc, c["wav_length"], c["ph_seq"], c["word_seq"], c["ph_idx_to_word_idx"])
            T = dec.ph_frame_pred.shape[0]
            mel = synth.rng(500 + ci).standard_normal((1, 64, T)).astype(np.float32)
            fig = dec.plot(torch.from_numpy(mel))
            a = captured["args"]
            arrays[f"c{ci}_mel"] = mel
            arrays[f"c{ci}_ph_intervals_int"] = np.asarray(a[2], np.int32)
            arrays[f"c{ci}_frame_confidence"] = np.asarray(a[3])         # each in the dtype the reference passes
            arrays[f"c{ci}_ph_frame_prob"] = np.asarray(a[4])
            arrays[f"c{ci}_ph_idx_frame"] = np.asarray(a[5])
            arrays[f"c{ci}_edge_prob"] = np.asarray(a[6])
            out.append({"ph_seq": [str(x) for x in a[1]], "figure": _figure_data(fig)})
            plt.close(fig)
    finally:
        tad.plot_for_valid = real
    np.savez_compressed(os.path.join(HERE, "plot.npz"), **arrays)
    with open(os.path.join(HERE, "plot.json"), "w") as f:
        json.dump({"cases": out}, f)
    print(f"plot: {len(out)} cases")


def gen_g2p():
    from networks.g2p import DictionaryG2P, NoneG2P, PhonemeG2P

    dic = synth.synth_dictionary(n_words=40)
    dpath = os.path.join(HERE, "synth_dict.txt")
    with open(dpath, "w") as f:
        for w, phs in dic.items():
            f.write(f"{w}\t{' '.join(phs)}\n")
    g_dict = DictionaryG2P(dictionary=dpath)
    g_none, g_ph = NoneG2P(), PhonemeG2P()
    texts = ["w000 w001 w002", "w003  w004", "w005 oov_word w006", "w007", "w010 w011 w012 w013 w014 w015"]
    ph_texts = ["a b c", "SP a SP SP b", "a b SP", "x"]
    res = {"dictionary": "synth_dict.txt", "dict": [], "none": [], "phoneme": []}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for t in texts:
            try:
                ph, w, m = g_dict(t)
                res["dict"].append({"text": t, "ph_seq": ph, "word_seq": w, "map": [int(x) for x in m]})
            except Exception as e:  # noqa: BLE001
                res["dict"].append({"text": t, "error": type(e).__name__})
        for t in ph_texts:
            for name, g in (("none", g_none), ("phoneme", g_ph)):
                try:
                    ph, w, m = g(t)
                    res[name].append({"text": t, "ph_seq": list(ph), "word_seq": list(w),
                                      "map": [int(x) for x in m]})
                except Exception as e:  # noqa: BLE001
                    res[name].append({"text": t, "error": type(e).__name__})
    with open(os.path.join(HERE, "g2p.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("g2p done")


def gen_g2p_edges():
    """Edge inputs through the reference's G2P plugins and the decoder's phone lookup: empty and blank texts, SP-only
    texts, repeated / leading / trailing spaces, dictionaries with no known word; the exception type when one is
    raised (base_g2p.py:37-40 AssertionError, alignment_decoder.py:35 KeyError), else the outputs."""
    import torch
    from networks.g2p import DictionaryG2P, NoneG2P, PhonemeG2P
    from tools.alignment_decoder import AlignmentDecoder

    g_dict = DictionaryG2P(dictionary=os.path.join(HERE, "synth_dict.txt"))
    texts = ["", " ", "SP", "SP SP", "a", " a", "a ", "a  b", "SP a SP", "AP a", "a\tb", "oov_only", "w000  ",
             "  w000 w001", "w000 oov w001 oov"]
    res = {"dictionary": "synth_dict.txt", "cases": []}

    def run(g, t):
        try:
            ph, w, m = g(t)
            return {"ph_seq": list(ph), "word_seq": list(w), "map": [int(x) for x in m]}
        except Exception as e:  # noqa: BLE001
            return {"error": type(e).__name__}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for t in texts:
            res["cases"].append({"text": t, "dict": run(g_dict, t), "none": run(NoneG2P(), t),
                                 "phoneme": run(PhonemeG2P(), t)})
    vocab = {"vocab": {"SP": 0, "AP": 0, "a": 1, "b": 2}, "vocab_size": 3}
    dec = AlignmentDecoder(vocab, {"sample_rate": 44100, "hop_length": 512})
    lg = torch.zeros(1, 8, 3)
    oov = []
    for ph_seq in (["SP", "a", "SP"], ["SP", "zz", "SP"], ["SP", "", "SP"]):
        try:
            dec.decode(lg, torch.zeros(1, 8), lg, None, ph_seq)
            oov.append({"ph_seq": ph_seq, "error": None})
        except Exception as e:  # noqa: BLE001
            oov.append({"ph_seq": ph_seq, "error": type(e).__name__})
    res["decode_lookup"] = {"vocab": vocab, "cases": oov}
    with open(os.path.join(HERE, "g2p_edges.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("g2p edges done")


def gen_g2p_dicts():
    """The reference's own shipped dictionaries (infer.py:37-41 default -d dictionary/opencpop-extension.txt, and the
    jyutping / japanese ones) through its DictionaryG2P: lyrics-like texts with OOV words, repeated spaces and
    every entry shape the files hold.  Stored: the texts, the expected outputs, and the dictionary entries the texts
    touch (so the test also runs where /root/reference is absent)."""
    from networks.g2p import DictionaryG2P
    rng = np.random.default_rng(7)
    res = {}
    for name in ("opencpop-extension", "jyutping_dict", "japanese_dict_full"):
        dpath = os.path.join(REF, "dictionary", name + ".txt")
        g = DictionaryG2P(dictionary=dpath)
        words = sorted(g.dictionary)
        texts = []
        for n in (1, 3, 8, 20, 40):
            texts.append(" ".join(words[int(i)] for i in rng.integers(0, len(words), n)))
        texts.append(" ".join([words[0], "not_a_word", words[-1], "  ", words[len(words) // 2]]))
        multi = [w for w in words if len(g.dictionary[w]) > 2][:5]
        if multi:
            texts.append(" ".join(multi))
        cases, used = [], set()
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for t in texts:
                ph, w, m = g(t)
                cases.append({"text": t, "ph_seq": list(ph), "word_seq": list(w), "map": [int(x) for x in m]})
                used.update(x for x in t.split(" ") if x in g.dictionary)
        res[name] = {"cases": cases, "n_entries": len(words),
                     "entries": {w: g.dictionary[w] for w in sorted(used)}}
    with open(os.path.join(HERE, "g2p_dicts.json"), "w") as f:
        json.dump(res, f, indent=1, ensure_ascii=False)
    print("g2p dictionaries done")


def gen_postproc():
    from tools.post_processing import post_processing

    r = synth.rng(5)
    cases = []
    # hand-made AP/SP gap cases + random jittered ones
    base = [
        (["a", "b", "c"], [[0.05, 0.5], [0.55, 1.0], [1.35, 2.0]], 2.05),
        (["AP", "b", "AP", "AP"], [[0.2, 0.5], [0.6, 1.0], [1.1, 1.4], [1.5, 1.9]], 2.0),
        (["a", "AP", "c"], [[0.0, 0.5], [0.58, 1.0], [1.2, 2.0]], 2.5),
        (["a"], [[0.3, 0.9]], 1.0),
        (["a", "b"], [[0.0, 0.5], [0.5, 1.0]], 1.0),
    ]
    for _ in range(6):
        n = int(r.integers(2, 9))
        edges = np.sort(r.uniform(0, 3.0, 2 * n))
        seq = [("AP" if r.uniform() < 0.3 else f"x{i}") for i in range(n)]
        base.append((seq, edges.reshape(n, 2).tolist(), float(edges[-1] + r.uniform(0, 0.3))))
    preds = []
    for i, (seq, iv, wl) in enumerate(base):
        preds.append((f"utt{i}.wav", wl, 0.5, np.array(seq), np.array(iv, np.float64), np.array(seq),
                      np.array(iv, np.float64)))
    res, log = post_processing(preds)
    for (seq, iv, wl), out in zip(base, res):
        cases.append({"seq": seq, "intervals": iv, "wav_length": wl,
                      "ph_seq": [str(x) for x in out[3]], "ph_intervals": np.asarray(out[4], float).tolist(),
                      "word_seq": [str(x) for x in out[5]],
                      "word_intervals": np.asarray(out[6], float).tolist()})
    with open(os.path.join(HERE, "postproc.json"), "w") as f:
        json.dump({"cases": cases, "n_errors": len(log)}, f, indent=1)
    print("postproc done", len(log), "errors")


def gen_gather_index():
    import torch

    out = {}
    for secs in (1.0, 5.0, 10.0, 300.0, 0.01):
        n44 = int(round(secs * 44100))
        hop_size, sample_rate = 512, 44100
        units = int(round(secs * 16000)) // 320 - 1  # Hubert frame count (any value: clamp bound)
        units = max(units, 1)
        # tools/encoder.py:56-58, executed verbatim as a torch expression
        n_frames = n44 // hop_size + 1
        ratio = (hop_size / sample_rate) / (320 / 16000)
        index = torch.clamp(torch.round(ratio * torch.arange(n_frames)).long(), max=units - 1)
        out[f"n{n44}_units{units}"] = index.numpy().astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "gather_index.npz"), **out)
    print("gather done")


def _to_torch_sd(sd):
    import torch
    return {k: torch.from_numpy(v.copy()) for k, v in sd.items()}


def gen_hubert():
    import torch
    from transformers import HubertConfig, HubertModel
    from networks.hubert.model import HubertSoft

    torch.manual_seed(0)
    wav = synth.synth_audio(16000, seed=3)
    out = {"wav": wav}
    # --- HF cnhubert base (12 layers), do_normalize applied on the host like Wav2Vec2FeatureExtractor ---
    arch = synth.arch_cnhubert_base()
    sd = synth.synth_hubert_state_dict(arch, seed=11)
    cfg = HubertConfig()
    cfg._attn_implementation = "eager"
    m = HubertModel(cfg).eval()
    tsd = _to_torch_sd(sd)
    # HF holds the weight-norm as a parametrization: original0 = g, original1 = v
    pre = "encoder.pos_conv_embed.conv."
    tsd[pre + "parametrizations.weight.original0"] = tsd.pop(pre + "weight_g")
    tsd[pre + "parametrizations.weight.original1"] = tsd.pop(pre + "weight_v")
    missing, unexpected = m.load_state_dict(tsd, strict=False)
    assert not unexpected and not [k for k in missing if "masked_spec" not in k], (missing, unexpected)
    x = torch.from_numpy(wav)[None]
    xn = (x - x.mean()) / torch.sqrt(x.var(unbiased=False) + 1e-7)
    with torch.inference_mode():
        feats = m.feature_extractor(xn)
        proj = m.feature_projection(feats.transpose(1, 2))
        hs = m(xn, output_hidden_states=True)
    out["hf_base_input"] = xn.numpy()[0]
    out["hf_base_feats"] = feats.numpy()[0]
    out["hf_base_proj"] = proj.numpy()[0]
    out["hf_base_layer1"] = hs.hidden_states[1].numpy()[0]
    out["hf_base_out"] = hs.last_hidden_state.numpy()[0]
    print("hf base out", hs.last_hidden_state.shape, float(hs.last_hidden_state.std()))
    np.savez_compressed(os.path.join(HERE, "hubert_hf_base.npz"), **out)

    # --- HF large-style (LN conv, stable LN), reduced to 2 layers to keep the fixture generator fast ---
    arch = synth.arch_cnhubert_large(layers=2)
    sd = synth.synth_hubert_state_dict(arch, seed=12)
    cfg = HubertConfig(hidden_size=1024, num_hidden_layers=2, num_attention_heads=16, intermediate_size=4096,
                       feat_extract_norm="layer", do_stable_layer_norm=True, conv_bias=True)
    cfg._attn_implementation = "eager"
    from transformers import HubertModel as HM
    m = HM(cfg).eval()
    tsd = _to_torch_sd(sd)
    tsd[pre + "parametrizations.weight.original0"] = tsd.pop(pre + "weight_g")
    tsd[pre + "parametrizations.weight.original1"] = tsd.pop(pre + "weight_v")
    missing, unexpected = m.load_state_dict(tsd, strict=False)
    assert not unexpected and not [k for k in missing if "masked_spec" not in k], (missing, unexpected)
    with torch.inference_mode():
        y = m(xn).last_hidden_state
    np.savez_compressed(os.path.join(HERE, "hubert_hf_large.npz"), input=xn.numpy()[0], out=y.numpy()[0])
    print("hf large out", y.shape, float(y.std()))

    # --- bshall HubertSoft.units (pads 40/40, projects to 256) ---
    arch = synth.arch_hubertsoft()
    sd = synth.synth_hubert_state_dict(arch, seed=13)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        hsoft = HubertSoft().eval()
    missing, unexpected = hsoft.load_state_dict(_to_torch_sd(sd), strict=True)
    with torch.inference_mode():
        u = hsoft.units(torch.from_numpy(wav)[None, None])
    np.savez_compressed(os.path.join(HERE, "hubert_soft.npz"), wav=wav, out=u.numpy()[0])
    print("hubertsoft out", u.shape, float(u.std()))


def gen_unet():
    import torch
    from networks.layer.backbone.unet import UNetBackbone
    from networks.layer.block.resnet_block import ResidualBasicBlock
    from networks.layer.scaling.stride_conv import DownSampling, UpSampling

    ua = synth.UNetArch()
    sd = synth.synth_unet_state_dict(ua, seed=21)
    bb = UNetBackbone(ua.input_dims, ua.output_dims, ua.hidden_dims, ResidualBasicBlock, DownSampling, UpSampling,
                      ua.factor, ua.times, ua.scaleup).eval()
    head = torch.nn.Linear(ua.output_dims, ua.vocab_size + 2).eval()
    bb.load_state_dict({k[len("backbone."):]: torch.from_numpy(v) for k, v in sd.items() if k.startswith("backbone.")})
    head.load_state_dict({k[len("head."):]: torch.from_numpy(v) for k, v in sd.items() if k.startswith("head.")})
    out = {}
    for T in (203, 862):
        x = synth.rng(31 + T).standard_normal((1, T, ua.input_dims)).astype(np.float32)
        with torch.inference_mode():
            h = bb(torch.from_numpy(x))
            logits = head(h)
        out[f"T{T}_logits"] = logits.numpy()[0]
        print("unet", T, logits.shape, float(logits.std()))
    np.savez_compressed(os.path.join(HERE, "unet_head.npz"), **out)


def _reference_encoder_module():
    """tools/encoder.py imports ``torchaudio.transforms.Resample`` at module level and torchaudio is absent here.
    A stub is installed for that one import and removed again (transformers probes torchaudio's presence later);
    the stub's Resample refuses to run.  The fixtures hand the reference's UnitsEncoder its 16 kHz wave through its
    own ``resample_kernel`` cache (encoder.py:44-48), so no resampling is ever executed and the resampler stays
    unpinned."""
    import transformers  # noqa: F401  (imported before the stub exists)
    if "tools.encoder" in sys.modules:
        return sys.modules["tools.encoder"]
    ta = types.ModuleType("torchaudio")
    tr = types.ModuleType("torchaudio.transforms")

    class Resample:
        def __init__(self, *a, **k):
            raise RuntimeError("torchaudio is absent: the fixtures never resample")
    tr.Resample = Resample
    ta.transforms = tr
    sys.modules["torchaudio"], sys.modules["torchaudio.transforms"] = ta, tr
    try:
        import tools.encoder as enc
    finally:
        del sys.modules["torchaudio"], sys.modules["torchaudio.transforms"]
    return enc


def _reference_lattice(units_encoder, wav16, n44, ua, usd, vocab, ph_seq, word_seq, p2w):
    """The reference's predict_step arithmetic after load_wav (forced_alignment.py:157-176), resampling excepted:
    UnitsEncoder.encode at the 44.1 kHz grid with the 16 kHz wave injected as its resampler's output, then
    UNetBackbone + head, the forward split (:284-292) and AlignmentDecoder.decode.  _decode's inputs are captured
    (ph_prob_log: the north star's per-frame log-probs)."""
    import torch
    from networks.layer.backbone.unet import UNetBackbone
    from networks.layer.block.resnet_block import ResidualBasicBlock
    from networks.layer.scaling.stride_conv import DownSampling, UpSampling
    from tools.alignment_decoder import AlignmentDecoder

    wav_t = torch.from_numpy(wav16)[None]
    units_encoder.resample_kernel["44100"] = lambda audio: wav_t       # the resampler's output, injected
    with torch.inference_mode():
        feat = units_encoder.encode(torch.zeros(1, n44), 44100, 512)    # [1, C, T] (encoder.py:36-60)
    bb = UNetBackbone(ua.input_dims, ua.output_dims, ua.hidden_dims, ResidualBasicBlock, DownSampling, UpSampling,
                      ua.factor, ua.times, ua.scaleup).eval()
    head = torch.nn.Linear(ua.output_dims, ua.vocab_size + 2).eval()
    bb.load_state_dict({k[len("backbone."):]: torch.from_numpy(v) for k, v in usd.items() if k.startswith("backbone.")})
    head.load_state_dict({k[len("head."):]: torch.from_numpy(v) for k, v in usd.items() if k.startswith("head.")})
    with torch.no_grad():
        logits = head(bb(feat.transpose(1, 2)))
    frame, edge = logits[:, :, 2:], logits[:, :, 0]
    ctc = torch.cat([logits[:, :, [1]], logits[:, :, 3:]], dim=-1)
    dec = AlignmentDecoder(vocab, {"hop_length": 512, "sample_rate": 44100})
    seen = {}
    inner = dec._decode

    def capture(ph_seq_id, ph_prob_log, edge_prob):
        seen.update(ph_prob_log=ph_prob_log.copy(), edge_prob=edge_prob.copy())   # edge_prob is f64 (:84)
        return inner(ph_seq_id, ph_prob_log, edge_prob)
    dec._decode = capture
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ph_pred, ph_int, w_pred, w_int, conf = dec.decode(frame, edge, ctc, n44 / 44100, ph_seq, word_seq, p2w)
    return dict(units=feat, ph_prob_log=seen["ph_prob_log"].astype(np.float32),
                edge_prob=seen["edge_prob"], ph_idx_seq=dec.ph_idx_seq.astype(np.int32),
                ph_time_int=dec.ph_time_int_pred.astype(np.int32),
                frame_confidence=dec.frame_confidence.astype(np.float32),
                ph_intervals=np.asarray(ph_int, np.float64), word_intervals=np.asarray(w_int, np.float64),
                ph_seq_pred=[str(x) for x in ph_pred], word_seq_pred=[str(x) for x in w_pred],
                confidence=float(conf))


def gen_e2e10s():
    """BASELINE config-2 geometry from the reference itself (VERDICT r02 'next' 1): one 10 s utterance (160 000
    samples at 16 kHz = the encoder's input; N44 = 441 000 -> 862 grid frames, T = 861) through the reference's
    UnitsEncoder (HF HubertModel base 12L, HF Hubert-large 24L stable-LN, bshall HubertSoft) -> reference UNet +
    head -> AlignmentDecoder.decode, with the product's default synthetic weights (synth:0 encoders, the
    synth_checkpoint(seed=1) UNet/head, V = 63) so the GPU box rebuilds them bit-identically.  Text: 30 words of
    the synthetic dictionary through the reference's DictionaryG2P (S = 91)."""
    import shutil
    import tempfile
    import torch
    from networks.g2p import DictionaryG2P
    import ckpt_files
    UnitsEncoder = _reference_encoder_module().UnitsEncoder

    wav16 = synth.synth_audio(160000, seed=2024)
    n44 = 441000
    vocab = synth.synth_vocab(62)
    g2p = DictionaryG2P(dictionary=os.path.join(HERE, "synth_dict.txt"))
    dic = synth.synth_dictionary(n_words=40)
    text = synth.synth_lab(30, dic, seed=2024)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        ph_seq, word_seq, p2w = g2p(text)
    p2w = [int(x) for x in p2w]
    meta = {"text": text, "ph_seq": list(ph_seq), "word_seq": list(word_seq), "ph_idx_to_word_idx": p2w,
            "n44": n44, "wav_seed": 2024, "encoders": {}}
    arrays = {"wav16_s16": np.round(wav16 * 32768).astype(np.int16)}
    tmp = tempfile.mkdtemp(prefix="hfa_gold_")
    try:
        for name, arch, enc in (("base", synth.arch_cnhubert_base(), "cnhubert"),
                                ("large", synth.arch_cnhubert_large(), "cnhubert"),
                                ("soft", synth.arch_hubertsoft(), "hubertsoft")):
            sd = synth.synth_hubert_state_dict(arch, seed=0)
            path = os.path.join(tmp, name)
            if enc == "cnhubert":
                ckpt_files.save_hf_folder(path, arch, sd, do_normalize=True)
            else:
                path += ".pt"
                torch.save({"hubert": {"module." + k: torch.from_numpy(v) for k, v in sd.items()}}, path)
            del sd
            ue = UnitsEncoder(enc, path, 16000, 320, device="cpu")
            ua = synth.UNetArch(input_dims=arch.out_channels, vocab_size=vocab["vocab_size"])
            usd = synth.synth_unet_state_dict(ua, seed=1)
            r = _reference_lattice(ue, wav16, n44, ua, usd, vocab, ph_seq, word_seq, p2w)
            del ue
            if name == "base":          # Hubert units at the grid, [C, 862] -> the [L, C] frames they gather
                arrays["base_units"] = r["units"][0].transpose(0, 1).numpy().astype(np.float32)
            for k in ("ph_prob_log", "edge_prob", "ph_idx_seq", "ph_time_int", "frame_confidence", "ph_intervals",
                      "word_intervals"):
                arrays[f"{name}_{k}"] = r[k]
            meta["encoders"][name] = {"encoder": enc, "channel": arch.out_channels,
                                      "ph_seq_pred": r["ph_seq_pred"], "word_seq_pred": r["word_seq_pred"],
                                      "confidence": r["confidence"], "n_ph": int(len(r["ph_idx_seq"]))}
            print(f"e2e 10 s {name}: T={r['ph_prob_log'].shape[0]} S={len(ph_seq)} n_ph={len(r['ph_idx_seq'])} "
                  f"conf={r['confidence']:.4f}")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    np.savez_compressed(os.path.join(HERE, "e2e_10s.npz"), **arrays)
    with open(os.path.join(HERE, "e2e_10s.json"), "w") as f:
        json.dump(meta, f, indent=1)


LOADER_SAMPLES = 16000      # loader fixtures: 1 s of audio through 2-layer encoders (tests/ckpt_files.py)


def gen_loaders():
    """Checkpoint-loader goldens (VERDICT r02 'next' 3).  The weight files themselves are rebuilt at test time by
    tests/ckpt_files.py from the same seeds (base-size conv stacks are ~17 MB of f32: too big to commit); what is
    stored is what the reference / transformers computed from each file:
      * HF folder written by HubertModel.save_pretrained (parametrized weight norm), preprocessor do_normalize
        true / false, and the legacy layout (pytorch_model.bin, weight_g/weight_v, "hubert." prefix), each loaded
        by the reference's Audio2CNHubert (HubertModel / Wav2Vec2FeatureExtractor.from_pretrained,
        encoder.py:86-96) -> units [1, 49, 768];
      * bshall {"hubert": {"module." + key: tensor}} loaded by the reference's Audio2HubertSoft (encoder.py:63-78,
        consume_prefix_in_state_dict_if_present) -> units [1, 50, 256];
      * a Lightning-layout .ckpt: state_dict = the reference modules' own keys (backbone / head, and every loss
        module's registered buffers, GHMLoss.py:18,64,123,126,225,227, under forced_alignment.py:82-108's
        attribute names) + hyper_parameters from configs/train_config.yaml; the reference UNet + head on a fixed
        input -> logits.  The buffer names/shapes are stored (the .ckpt is rebuilt at test time)."""
    import shutil
    import tempfile
    import torch
    import yaml
    import ckpt_files
    from networks.loss.BinaryEMDLoss import BinaryEMDLoss
    from networks.loss.GHMLoss import CTCGHMLoss, GHMLoss, MultiLabelGHMLoss
    UnitsEncoder = _reference_encoder_module().UnitsEncoder

    wav = synth.synth_audio(LOADER_SAMPLES, seed=5)
    out = {"wav": wav}
    tmp = tempfile.mkdtemp(prefix="hfa_gold_")
    try:
        units = {}
        for kind in ckpt_files.HF_KINDS:
            path = os.path.join(tmp, kind)
            ckpt_files.write_hf_folder(path, kind)
            ue = UnitsEncoder("cnhubert", path, 16000, 320, device="cpu")
            with torch.inference_mode():
                units[kind] = ue.model(torch.from_numpy(wav)[None])[0].numpy()
        assert np.array_equal(units["hf"], units["hf_legacy"]), "transformers loads both layouts to one model"
        out["hf_units"] = units["hf"]
        out["hf_nonorm_units"] = units["hf_nonorm"]
        path = os.path.join(tmp, "soft.pt")
        ckpt_files.write_bshall(path)
        ue = UnitsEncoder("hubertsoft", path, 16000, 320, device="cpu")
        with torch.inference_mode():
            out["soft_units"] = ue.model(torch.from_numpy(wav)[None])[0].numpy()
        print("loader units:", {k: v.shape for k, v in out.items()})
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    # the loss modules' buffers, as LitForcedAlignmentTask.__init__ builds them (forced_alignment.py:82-108)
    cfg = yaml.safe_load(open(os.path.join(REF, "configs", "train_config.yaml")))
    lf = cfg["loss_config"]["function"]
    vocab = synth.synth_vocab(62)
    V = vocab["vocab_size"]
    losses = {"ph_frame_GHM_loss_fn": GHMLoss(V, lf["num_bins"], lf["alpha"], lf["label_smoothing"]),
              "pseudo_label_GHM_loss_fn": MultiLabelGHMLoss(V, lf["num_bins"], lf["alpha"], lf["label_smoothing"]),
              "ph_edge_GHM_loss_fn": MultiLabelGHMLoss(1, lf["num_bins"], lf["alpha"], label_smoothing=0.0),
              "EMD_loss_fn": BinaryEMDLoss(),
              "ph_edge_diff_GHM_loss_fn": MultiLabelGHMLoss(1, lf["num_bins"], lf["alpha"], label_smoothing=0.0),
              "CTC_GHM_loss_fn": CTCGHMLoss(alpha=1 - 1e-3)}
    buffers = {f"{n}.{k}": list(v.shape) for n, m in losses.items() for k, v in m.state_dict().items()}
    # the reference UNet + head on a fixed input through the checkpoint's weights
    ua = synth.UNetArch(vocab_size=V)
    usd = synth.synth_unet_state_dict(ua, seed=ckpt_files.CKPT_SEED)
    from networks.layer.backbone.unet import UNetBackbone
    from networks.layer.block.resnet_block import ResidualBasicBlock
    from networks.layer.scaling.stride_conv import DownSampling, UpSampling
    bb = UNetBackbone(ua.input_dims, ua.output_dims, ua.hidden_dims, ResidualBasicBlock, DownSampling, UpSampling,
                      ua.factor, ua.times, ua.scaleup).eval()
    head = torch.nn.Linear(ua.output_dims, V + 2).eval()
    bb.load_state_dict({k[len("backbone."):]: torch.from_numpy(v) for k, v in usd.items() if k.startswith("backbone.")})
    head.load_state_dict({k[len("head."):]: torch.from_numpy(v) for k, v in usd.items() if k.startswith("head.")})
    x = synth.rng(77).standard_normal((1, 301, ua.input_dims)).astype(np.float32)
    with torch.no_grad():
        out["ckpt_logits"] = head(bb(torch.from_numpy(x))).numpy()[0]
    meta = {"loss_buffers": buffers, "model_config": cfg["model"], "hubert_config": cfg["hubert_config"],
            "melspec_config": cfg["melspec_config"], "optimizer_config": cfg["optimizer_config"],
            "loss_config": cfg["loss_config"], "unet_input_seed": 77, "unet_input_T": 301,
            "layers": ckpt_files.LOADER_LAYERS, "wav_seed": 5}
    np.savez_compressed(os.path.join(HERE, "loaders.npz"), **out)
    with open(os.path.join(HERE, "loaders.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("loaders done:", len(buffers), "loss buffers")


def main():
    if not os.path.isdir(REF):
        print("reference absent: fixtures are generated only in the survey/build container; skipping")
        return
    _import_reference()
    which = sys.argv[1:] or ["dp", "decode", "g2p", "postproc", "gather", "hubert", "unet", "e2e10s", "loaders"]
    for w in which:
        {"dp": gen_dp_cases, "decode": gen_decode_cases, "g2p": gen_g2p, "g2p_dicts": gen_g2p_dicts,
         "g2p_edges": gen_g2p_edges,
         "postproc": gen_postproc,
         "gather": gen_gather_index, "hubert": gen_hubert, "unet": gen_unet, "e2e10s": gen_e2e10s,
         "loaders": gen_loaders, "plot": gen_plot}[w]()


if __name__ == "__main__":
    main()
