"""Host-side drop-ins (CPU): G2P plugins and post-processing against the reference goldens, TextGrid/CSV writers,
WAV I/O, checkpoint round trip, and the multi-rank boundary gather over gloo (world size 2)."""
import json
import os
import warnings

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_g2p_plugins_match_reference():
    from hubertfa_amd.g2p import DictionaryG2P, NoneG2P, PhonemeG2P
    gold = json.load(open(os.path.join(GOLDEN, "g2p.json")))
    g = DictionaryG2P(dictionary=os.path.join(GOLDEN, gold["dictionary"]))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for case in gold["dict"]:
            if "error" in case:
                with pytest.raises(Exception):
                    g(case["text"])
                continue
            ph, w, m = g(case["text"])
            assert (ph, w, [int(x) for x in m]) == (case["ph_seq"], case["word_seq"], case["map"]), case["text"]
        for name, cls in (("none", NoneG2P), ("phoneme", PhonemeG2P)):
            for case in gold[name]:
                if "error" in case:
                    with pytest.raises(Exception):
                        cls()(case["text"])
                    continue
                ph, w, m = cls()(case["text"])
                assert list(ph) == case["ph_seq"] and list(w) == case["word_seq"], (name, case["text"])
                assert [int(x) for x in m] == case["map"]


def test_g2p_edge_inputs_and_lookup_errors_match_reference():
    """Edge texts (empty, blank, SP-only, repeated / leading / trailing spaces, tabs, unknown words) through the
    three G2P plugins give the reference's outputs, and the decoder's phone lookup raises the reference's KeyError
    on an unknown phone (alignment_decoder.py:35) before any device work (tests/golden/g2p_edges.json, made by the
    reference's own classes)."""
    import builtins

    import torch
    from hubertfa_amd.alignment_decoder import AlignmentDecoder
    from hubertfa_amd.g2p import DictionaryG2P, NoneG2P, PhonemeG2P
    gold = json.load(open(os.path.join(GOLDEN, "g2p_edges.json")))
    gs = {"dict": DictionaryG2P(dictionary=os.path.join(GOLDEN, gold["dictionary"])), "none": NoneG2P(),
          "phoneme": PhonemeG2P()}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for case in gold["cases"]:
            for name, g in gs.items():
                want = case[name]
                if "error" in want:
                    with pytest.raises(getattr(builtins, want["error"])):
                        g(case["text"])
                    continue
                ph, w, m = g(case["text"])
                assert (list(ph), list(w), [int(x) for x in m]) == (want["ph_seq"], want["word_seq"], want["map"]), \
                    (name, case["text"])
    lk = gold["decode_lookup"]
    dec = AlignmentDecoder(lk["vocab"], {"sample_rate": 44100, "hop_length": 512})
    lg = torch.zeros(1, 8, 3)
    for case in lk["cases"]:
        if case["error"] is None:
            assert list(dec.ph_ids(case["ph_seq"])) == [lk["vocab"]["vocab"][p] for p in case["ph_seq"]]
        else:
            assert case["error"] == "KeyError"
            with pytest.raises(KeyError):
                dec.decode(lg, torch.zeros(1, 8), lg, None, case["ph_seq"])


@pytest.mark.parametrize("name", ["opencpop-extension", "jyutping_dict", "japanese_dict_full"])
def test_g2p_reference_dictionaries(name, tmp_path):
    """DictionaryG2P over the reference's shipped dictionaries (the CLI's default -d opencpop-extension.txt,
    infer.py:37-41): parsed from the reference's own file when present (entry count must match), else from the
    entries the golden texts use (tests/golden/g2p_dicts.json, made by the reference's DictionaryG2P)."""
    from hubertfa_amd.g2p import DictionaryG2P
    gold = json.load(open(os.path.join(GOLDEN, "g2p_dicts.json"), encoding="utf-8"))[name]
    path = tmp_path / (name + ".txt")
    path.write_text("".join(f"{w}\t{' '.join(p)}\n" for w, p in gold["entries"].items()), encoding="utf-8")
    gs = [DictionaryG2P(dictionary=str(path))]
    ref_file = os.path.join("/root/reference/dictionary", name + ".txt")
    if os.path.exists(ref_file):
        gs.append(DictionaryG2P(dictionary=ref_file))
        assert len(gs[-1].dictionary) == gold["n_entries"]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for g in gs:
            for case in gold["cases"]:
                ph, w, m = g(case["text"])
                assert (list(ph), list(w), [int(x) for x in m]) == (case["ph_seq"], case["word_seq"], case["map"]), \
                    case["text"]


def test_post_processing_matches_reference():
    from hubertfa_amd.post_processing import post_processing
    gold = json.load(open(os.path.join(GOLDEN, "postproc.json")))
    preds = []
    for i, c in enumerate(gold["cases"]):
        iv = np.array(c["intervals"], np.float64)
        preds.append((f"utt{i}.wav", c["wav_length"], 0.5, np.array(c["seq"]), iv.copy(), np.array(c["seq"]),
                      iv.copy()))
    res, log = post_processing(preds)
    assert len(log) == gold["n_errors"]
    for c, r in zip(gold["cases"], res):
        assert [str(x) for x in r[3]] == c["ph_seq"] and [str(x) for x in r[5]] == c["word_seq"]
        np.testing.assert_array_equal(np.asarray(r[4], float), np.asarray(c["ph_intervals"], float))
        np.testing.assert_array_equal(np.asarray(r[6], float), np.asarray(c["word_intervals"], float))


def test_post_processing_collects_errors():
    from hubertfa_amd.post_processing import post_processing
    res, log = post_processing([("bad.wav", 1.0, 0.1, np.array([]), np.zeros((0, 2)), np.array([]),
                                 np.zeros((0, 2)))])
    assert res == [] and len(log) == 1


def test_textgrid_and_confidence_export(tmp_path):
    import pandas as pd
    from hubertfa_amd.export_tool import Exporter, read_textgrid
    from hubertfa_amd.post_processing import post_processing
    wav = tmp_path / "a" / "utt.wav"
    wav.parent.mkdir()
    wav.write_bytes(b"")
    ph_iv = np.array([[0.05, 0.4], [0.4, 0.9], [1.3, 1.5]])
    w_iv = np.array([[0.05, 0.9], [1.3, 1.5]])
    preds, log = post_processing([(wav, 2.0, np.float32(0.25), np.array(["a", "b", 'q"x']), ph_iv,
                                   np.array(["w1", "w2"]), w_iv)])
    Exporter(preds, log).export(["textgrid", "confidence"])
    tg = read_textgrid(tmp_path / "a" / "TextGrid" / "utt.TextGrid")
    assert [t[2] for t in tg["words"]] == ["w1", "SP", "w2", "SP"]
    assert [t[2] for t in tg["phones"]] == ["a", "b", "SP", 'q"x', "SP"]
    assert tg["phones"][0][0] == 0.0 and tg["phones"][-1][1] == 2.0
    for tier in tg.values():   # contiguous, non-overlapping
        assert all(abs(a[1] - b[0]) < 1e-12 for a, b in zip(tier[:-1], tier[1:]))
    df = pd.read_csv(tmp_path / "a" / "confidence" / "confidence.csv")
    assert list(df.columns) == ["name", "confidence"] and df["name"][0] == "utt"


def test_streaming_export_matches_batch_export(tmp_path):
    """infer.py's one-GPU streaming export (post-process + TextGrid per completed batch, batches out of dataset
    order) writes the same TextGrids, confidence table and error log as post-processing the whole folder."""
    import infer
    from hubertfa_amd.alignment_decoder import utterance_result
    from hubertfa_amd.export_tool import Exporter
    from hubertfa_amd.post_processing import post_processing
    rng = np.random.default_rng(3)
    rows, records = [], {}
    for i in range(7):
        wav = tmp_path / "seg" / f"u{i}.wav"
        wav.parent.mkdir(exist_ok=True)
        wav.write_bytes(b"")
        n_ph = 5 + i
        ph_seq = ["SP"] + [f"p{j}" for j in range(n_ph - 2)] + ["SP"]
        p2w = [-1] + [j // 2 for j in range(n_ph - 2)] + [-1]
        words = [f"w{j}" for j in range((n_ph - 2 + 1) // 2)]
        T = 200 + 30 * i
        cuts = np.sort(rng.choice(np.arange(1, T - 1), n_ph - 1, replace=False))
        rec = dict(n44=T * 512 + 100, T=T, ph_idx_seq=np.arange(n_ph), ph_time_int=np.concatenate([[0], cuts]),
                   frame_confidence=rng.uniform(0.2, 1.0, T).astype(np.float32),
                   edge_diff=rng.uniform(-1, 1, T).astype(np.float32))
        if i == 4:                                   # all SP: no intervals, post-processing fails -> error log
            ph_seq = ["SP"] * n_ph
        rows.append((str(wav), ph_seq, words, p2w))
        records[i] = rec
    sr, fl = 44100, 512 / 44100
    sink = infer._StreamingExport(rows, sr, fl, tmp_path / "stream")
    for ks in ([5, 6], [0, 3, 1], [2, 4]):
        sink(records, ks)
    s_preds, s_log = sink.results()
    preds = []
    for i, (wav, ph_seq, words, p2w) in enumerate(rows):
        r = utterance_result(records[i], ph_seq, words, p2w, fl)
        preds.append((wav, records[i]["n44"] / sr, r["confidence"], r["ph_seq"], r["ph_intervals"], r["word_seq"],
                      r["word_intervals"]))
    b_preds, b_log = post_processing(preds)
    Exporter(b_preds, b_log, tmp_path / "batch").export(["textgrid"])
    assert [p[0] for p in s_preds] == [p[0] for p in b_preds]
    assert [p[2] for p in s_preds] == [p[2] for p in b_preds]
    assert len(b_log) == 1 and [(e[0], repr(e[1])) for e in s_log] == [(e[0], repr(e[1])) for e in b_log]
    streamed = {p.name: p.read_bytes() for p in (tmp_path / "stream").rglob("*.TextGrid")}
    batch = {p.name: p.read_bytes() for p in (tmp_path / "batch").rglob("*.TextGrid")}
    assert streamed == batch and len(batch) == len(b_preds)


def test_textgrid_text_matches_tier_objects():
    """Exporter's direct formatter (textgrid_text) writes exactly what the IntervalTier/TextGrid objects write,
    for post-processed predictions (gaps, touching intervals, an int end from add_SP, quotes in marks), and
    declines (None) whatever the objects must sort or reject."""
    from hubertfa_amd.export_tool import IntervalTier, TextGrid, textgrid_text
    from hubertfa_amd.post_processing import post_processing

    def objects(ws, wiv, ps, piv):
        tg, wt, pt = TextGrid(), IntervalTier(name="words"), IntervalTier(name="phones")
        for w, (a, b) in zip(ws, wiv):
            wt.add(a, b, w)
        for ph, (a, b) in zip(ps, piv):
            pt.add(minTime=float(a), maxTime=b, mark=ph)
        tg.append(wt)
        tg.append(pt)
        return "\n".join(tg.lines()) + "\n"
    rng = np.random.default_rng(5)
    preds = []
    for i in range(40):
        n = int(rng.integers(1, 12))
        cuts = np.sort(rng.uniform(0.05, 9.5, 2 * n))
        ph_iv = cuts.reshape(n, 2).copy()
        if i % 3 == 0:
            ph_iv[1:, 0] = ph_iv[:-1, 1]                     # touching intervals
        marks = np.array([f'p{j}' if j % 5 else 'q"x' for j in range(n)])
        w_iv = ph_iv[::2].copy()
        w_iv[:, 1] = ph_iv[1::2, 1] if n > 1 and len(ph_iv[1::2]) == len(w_iv) else w_iv[:, 1]
        preds.append((f"u{i}.wav", 10 if i % 4 == 0 else 10.0, 0.5, marks, ph_iv, marks[::2], w_iv))
    res, log = post_processing(preds)
    assert len(res) > 30
    for _, _, _, ps, piv, ws, wiv in res:
        assert textgrid_text(ws, wiv, ps, piv) == objects(ws, wiv, ps, piv)
    iv = np.array([[0.5, 1.0], [0.2, 0.4]])                     # out of order: the objects sort it
    assert textgrid_text(["a", "b"], iv, ["a", "b"], iv) is None
    assert textgrid_text(["a"], np.array([[1.0, 1.0]]), ["a"], np.array([[0.0, 1.0]])) is None   # empty interval
    assert textgrid_text(["a"], np.array([[0.0, 1.0]], np.float32), ["a"], np.array([[0.0, 1.0]])) is None


def test_wav_roundtrip(tmp_path):
    from hubertfa_amd import synth
    from hubertfa_amd.wav_io import read_wav, write_wav
    x = synth.synth_audio(4000, seed=2)
    p = tmp_path / "x.wav"
    write_wav(p, x, 16000)
    y, sr = read_wav(p)
    assert sr == 16000 and y.shape == (1, 4000)
    np.testing.assert_array_equal(y[0], x)   # synth audio is already s16-quantised


def _wav_bytes(tag, bits, ch, payload, extensible=False, extra=False, data_size=None):
    import struct
    block = ch * bits // 8
    if extensible:
        fmt = struct.pack("<HHIIHHHHIH14s", 0xFFFE, ch, 22050, 22050 * block, block, bits, 22, bits, 0, tag,
                          b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71")
    else:
        fmt = struct.pack("<HHIIHH", tag, ch, 22050, 22050 * block, block, bits)
    body = b"fmt " + struct.pack("<I", len(fmt)) + fmt
    if extra:                                    # an odd-sized chunk (padded to even) before the data
        body += b"LIST" + struct.pack("<I", 5) + b"abcde" + b"\x00"
    body += b"data" + struct.pack("<I", len(payload) if data_size is None else data_size) + payload
    return b"RIFF" + struct.pack("<I", 4 + len(body)) + b"WAVE" + body


@pytest.mark.parametrize("tag,bits,dtype", [(1, 8, "u1"), (1, 16, "<i2"), (1, 24, None), (1, 32, "<i4"),
                                            (3, 32, "<f4"), (3, 64, "<f8")])
@pytest.mark.parametrize("ch,extensible,extra", [(1, False, False), (2, True, True), (3, False, True)])
def test_native_wav_reader_matches_restatement(tmp_path, tag, bits, dtype, ch, extensible, extra):
    """libhfa's hfa_wav_read / hfa_wav_info (csrc/wav.cpp) against the numpy restatement of torchaudio.load's
    normalisation (oracle/wav_read.py), bit for bit, every format and channel layout the reader accepts."""
    from hubertfa_amd.wav_io import read_wav, read_wav_into, wav_info
    from oracle.wav_read import read_wav_np, wav_info_np
    rng = np.random.default_rng(bits * 10 + ch)
    n = 70001                                    # > one 65 536-frame decode block
    if dtype is None:
        payload = rng.integers(0, 256, n * ch * 3, dtype=np.uint8).tobytes()
    elif dtype[-2] == "f":
        payload = (rng.standard_normal(n * ch) * 0.5).astype(dtype).tobytes()
    else:
        info = np.iinfo(np.dtype(dtype))
        v = rng.integers(info.min, info.max, n * ch, dtype=np.int64, endpoint=True)
        v[:4] = [info.min, info.max, 0, -1 if info.min < 0 else 128]
        payload = v.astype(dtype).tobytes()
    p = tmp_path / "x.wav"
    p.write_bytes(_wav_bytes(tag, bits, ch, payload, extensible, extra))
    x, sr = read_wav(p)
    y, sr2 = read_wav_np(p)
    assert sr == sr2 == 22050 and x.shape == y.shape == (ch, n)
    np.testing.assert_array_equal(x, y)
    assert wav_info(p) == wav_info_np(p) == (n, 22050, ch)
    row = np.full(n + 5, 7.0, np.float32)      # one channel into a longer row: the tail is left alone
    assert read_wav_into(p, row, channel=ch - 1) == (n, 22050)
    np.testing.assert_array_equal(row[:n], y[ch - 1])
    assert (row[n:] == 7.0).all()


def test_native_wav_reader_edges(tmp_path):
    from hubertfa_amd.wav_io import read_wav, read_wav_into, wav_info
    from oracle.wav_read import read_wav_np
    v = np.arange(-500, 501, dtype="<i2")
    p = tmp_path / "s.wav"
    p.write_bytes(_wav_bytes(1, 16, 1, v.tobytes(), data_size=0xFFFFFFFF))   # streaming writer's size
    x, _ = read_wav(p)
    np.testing.assert_array_equal(x, read_wav_np(p)[0])
    assert wav_info(p)[0] == 1001
    p.write_bytes(_wav_bytes(1, 16, 2, v.tobytes()[:-2]))                   # a trailing partial frame is dropped
    assert read_wav(p)[0].shape == (2, 500)
    bad = [(b"RIFX" + b"\0" * 40, "not a RIFF"), (_wav_bytes(1, 12, 1, b"\0" * 8), "unsupported"),
           (_wav_bytes(1, 16, 1, b"")[:36], "missing fmt or data")]
    for raw, msg in bad:
        p.write_bytes(raw)
        with pytest.raises(ValueError, match=msg):
            read_wav(p)
    with pytest.raises(ValueError, match="cannot open"):
        wav_info(tmp_path / "nope.wav")
    p.write_bytes(_wav_bytes(1, 16, 1, v.tobytes()))
    with pytest.raises(ValueError, match="do not fit"):
        read_wav_into(p, np.zeros(1000, np.float32))
    with pytest.raises(ValueError, match="channel 1 of 1"):
        read_wav_into(p, np.zeros(2000, np.float32), channel=1)


def test_native_wav_reader_hostile_headers(tmp_path):
    """Headers that claim 65535 channels of 64-bit floats (0.5 MB per frame): the staging buffer stays within its
    fixed budget whatever the header says, so an empty or short data chunk reads as such instead of asking for
    ~34 GB; a zero sample rate is rejected.  Every failure is a ValueError for that file, never an abort."""
    import struct
    from hubertfa_amd.wav_io import read_wav, read_wav_into, wav_info
    def hostile(payload):                                       # block align does not fit its 16 bits either
        fmt = struct.pack("<HHIIHH", 3, 65535, 22050, 0xFFFFFFFF, 0xFFFF, 64)
        body = b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(payload)) + payload
        return b"RIFF" + struct.pack("<I", 4 + len(body)) + b"WAVE" + body
    p = tmp_path / "h.wav"
    p.write_bytes(hostile(b""))
    assert wav_info(p) == (0, 22050, 65535)
    assert read_wav_into(p, np.zeros(4, np.float32), channel=3) == (0, 22050)
    frames = np.arange(3 * 65535, dtype="<f8") / 1e6            # three whole frames
    p.write_bytes(hostile(frames.tobytes()))
    row = np.zeros(3, np.float32)
    assert read_wav_into(p, row, channel=65534) == (3, 22050)
    np.testing.assert_array_equal(row, frames.reshape(3, 65535)[:, 65534].astype(np.float32))
    with pytest.raises(ValueError, match="do not fit"):
        read_wav_into(p, np.zeros(10, np.float32), channel=-1)
    raw = bytearray(_wav_bytes(1, 16, 1, b"\0\0" * 8))
    raw[24:28] = struct.pack("<I", 0)                            # sample rate 0
    p.write_bytes(bytes(raw))
    with pytest.raises(ValueError, match="0 Hz"):
        wav_info(p)


def test_checkpoint_roundtrip(tmp_path):
    import torch
    from hubertfa_amd.task import synth_checkpoint
    p = tmp_path / "m.ckpt"
    ck = synth_checkpoint(str(p))
    loaded = torch.load(p, map_location="cpu", weights_only=True)
    assert set(loaded["state_dict"]) == set(ck["state_dict"])
    assert loaded["hyper_parameters"]["hubert_config"]["encoder"] == "cnhubert"


def test_lpt_sharding_balances():
    from hubertfa_amd.distributed import shard_lpt
    costs = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    shards = shard_lpt(costs, 3)
    assert sorted(i for s in shards for i in s) == list(range(10))
    loads = [sum(costs[i] for i in s) for s in shards]
    assert max(loads) - min(loads) <= 2


def _records(rank):
    """Rank-local raw boundary records of different counts and lengths (rank 1 holds none of rank 0's sizes)."""
    rng = np.random.default_rng(rank)
    recs = {}
    for j in range(3 + 2 * rank):                      # 3 utterances on rank 0, 5 on rank 1
        T = int(rng.integers(5, 40)) + 17 * rank
        n = int(rng.integers(1, T))
        recs[10 * j + rank] = dict(n44=512 * T + j, T=T, ph_idx_seq=np.sort(rng.integers(0, 50, n)),
                                   ph_time_int=np.sort(rng.choice(T, n, replace=False)),
                                   frame_confidence=rng.random(T).astype(np.float32),
                                   edge_diff=rng.standard_normal(T).astype(np.float32))
    return recs


def _gloo_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from hubertfa_amd.distributed import gather_boundaries, gather_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, T = 3 + rank, 7 + 4 * rank                         # unequal local batch shapes
    dev_out = {"ph_idx_seq": torch.full((B, T), rank, dtype=torch.int32),
               "ph_time_int": torch.arange(B * T, dtype=torch.int32).view(B, T) + 100 * rank,
               "n": torch.full((B,), rank + 1, dtype=torch.int32),
               "frame_confidence": torch.full((B, T), float(rank))}
    g = gather_boundaries(dev_out)
    recs = gather_records(_records(rank))
    if rank == 0:
        q.put(({k: [v.numpy().tolist() for v in parts] for k, parts in g.items()},
               {k: {f: np.asarray(v).tolist() for f, v in r.items()} for k, r in recs.items()}))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_boundary_gather_world2_gloo_unequal_shapes(world):
    """all_gather of each rank's (B, Tmax), then a padded all_gather_into_tensor per array; ranks
    hold different batch sizes and lengths, and rank 0 gets every rank's arrays back unpadded (and the CLI's
    record tables survive the round trip bit for bit).  World 8 rehearses the driver's 8-GPU node on gloo."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res, recs = q.get(timeout=180)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        B, T = 3 + r, 7 + 4 * r
        assert np.array(res["ph_idx_seq"][r]).shape == (B, T) and bool((np.array(res["ph_idx_seq"][r]) == r).all())
        assert res["n"][r] == [r + 1] * B
        assert np.array(res["ph_time_int"][r])[0, 0] == 100 * r
        assert np.array(res["ph_time_int"][r])[B - 1, T - 1] == 100 * r + B * T - 1
    want = {}
    for r in range(world):
        want.update(_records(r))
    assert sorted(recs) == sorted(want)
    for k, r in want.items():
        for f, v in r.items():
            assert np.array_equal(np.asarray(recs[k][f]), np.asarray(v)), (k, f)


def test_record_table_pack_unpack_world1():
    from hubertfa_amd.distributed import gather_records
    want = _records(1)
    got = gather_records(want)
    for k, r in want.items():
        for f, v in r.items():
            assert np.array_equal(np.asarray(got[k][f]), np.asarray(v)), (k, f)
    assert gather_records({}) == {}


def test_wav_info_header_only(tmp_path):
    from hubertfa_amd.wav_io import wav_info, write_wav
    p = tmp_path / "a.wav"
    write_wav(p, np.zeros(22051, np.float32), 22050)
    assert wav_info(p) == (22051, 22050, 1)


def test_torchaudio_target_length_float32_ceil():
    """torchaudio's _apply_sinc_resample_kernel takes ceil(as_tensor(new * n / orig)): a float32 quotient, so just
    above an integer it rounds down (e.g. 44.1 kHz -> 16 kHz at n = 722562: 262154.0045... -> 262154)."""
    import torch
    from hubertfa_amd.resample import target_length
    for n, o, w in ((722562, 44100, 16000), (160000, 16000, 44100), (441000, 44100, 16000), (1, 16000, 44100),
                    (12345, 48000, 44100), (999999, 22050, 44100)):
        g = int(np.gcd(o, w))
        ta = int(torch.ceil(torch.as_tensor((w // g) * n / (o // g))).long())
        assert target_length(n, o, w) == ta
    assert target_length(722562, 44100, 16000) == 262154 == -(-160 * 722562 // 441) - 1


def test_resampled_and_encoder_lengths():
    from hubertfa_amd.batching import encoder_length, resampled_length
    assert resampled_length(160000, 16000, 44100) == 441000
    assert resampled_length(441000, 44100, 16000) == 160000
    assert resampled_length(1, 16000, 44100) == 3                   # ceil(441 / 160)
    assert resampled_length(12345, 44100, 44100) == 12345
    assert encoder_length(160000, 16000) == 160000
    assert encoder_length(48000, 48000) == resampled_length(resampled_length(48000, 48000, 44100), 44100, 16000)


def test_plan_batches_sorted_short_alone():
    from hubertfa_amd.batching import plan_batches
    items = [("a", 50000, 16000), ("b", 20000, 16000), ("c", 100, 16000), ("d", 90000, 16000),
             ("e", 30000, 44100), ("f", 70000, 16000), ("g", 60000, 16000)]
    plan = plan_batches(items, batch_size=2)
    assert (16000, ["c"]) in plan                                    # 100 samples -> < 400 at the encoder: alone
    b16 = [keys for sr, keys in plan if sr == 16000 and keys != ["c"]]
    assert b16 == [["b", "a"], ["g", "f"], ["d"]]                    # sorted by length, batch_size 2
    assert (44100, ["e"]) in plan
    assert sorted(k for _, ks in plan for k in ks) == sorted(i[0] for i in items)


def test_longform_window_plan_and_spans():
    from hubertfa_amd import synth
    from hubertfa_amd.encoder import plan_windows, window_samples
    from hubertfa_amd.hubert import frame_count
    for L, C, O in ((1499, 400, 100), (25839, 1000, 100), (1000, 1000, 50), (7, 3, 2)):
        wins = plan_windows(L, C, O)
        cores = [i for c0, c1, _, _ in wins for i in range(c0, c1)]
        assert cores == list(range(L))                                # cores tile [0, L) once, in order
        for c0, c1, a, b in wins:
            assert 0 <= a <= c0 < c1 <= b <= L and c0 - a <= O and b - c1 <= O
    for arch in (synth.arch_cnhubert_base(), synth.arch_cnhubert_large(), synth.arch_hubertsoft()):
        for a, b in ((0, 1), (0, 400), (300, 1601), (5, 6)):
            assert frame_count(arch, window_samples(a, b, pad=arch.wav_pad)) == b - a


def test_bench_config3_batch():
    """bench.py's N > 1 runs keep config 2's per-GPU batch for the weak-scaling line and add a BASELINE config-3
    measurement (global batch 512) after it: 256 / 128 / 64 per GPU at N = 2 / 4 / 8."""
    import argparse
    import bench
    a = argparse.Namespace(encoder="base", seconds=10.0, chunk_seconds=None, batch=32, no_config3=False)
    assert [bench.config3_batch(a, n) for n in (1, 2, 4, 8)] == [0, 256, 128, 64]
    assert bench.config3_batch(argparse.Namespace(**{**vars(a), "batch": 64}), 8) == 0     # already config 3
    assert bench.config3_batch(argparse.Namespace(**{**vars(a), "encoder": "large"}), 8) == 0
    assert bench.config3_batch(argparse.Namespace(**{**vars(a), "no_config3": True}), 8) == 0
    assert bench.config_name("base", 8, 64) == "config 3 geometry"


def test_bench_gpus_flag_launch_policy():
    """bench.py --gpus N (verdict r04 item 1): without WORLD_SIZE and N > 1 it starts N ranks under
    torch.distributed.run as a child; under a launcher the rank count must equal N; too few visible GPUs (and no
    --device rehearsal) is an error, never a silent one-rank line."""
    import argparse
    import bench
    a = lambda g, d=None: argparse.Namespace(gpus=g, device=d)  # noqa: E731
    assert bench.check_world(a(1), {}) is None
    assert bench.check_world(a(2, 0), {}) == "launch"
    assert bench.check_world(a(8, 0), {}) == "launch"
    assert bench.check_world(a(2), {"WORLD_SIZE": "2"}) is None
    assert "WORLD_SIZE=4" in bench.check_world(a(2), {"WORLD_SIZE": "4"})
    assert "WORLD_SIZE=1" in bench.check_world(a(8), {"WORLD_SIZE": "1"})
    assert "at least one" in bench.check_world(a(0), {})
    import torch
    if torch.cuda.device_count() < 2:
        assert "visible" in bench.check_world(a(2), {})
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "3"], 29511)
    assert cmd[1:4] == ["-u", "-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and "--master-port=29511" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_gpus_without_devices_exits_nonzero():
    """`python bench.py --gpus 2` on a node with fewer than 2 visible GPUs exits non-zero with a message and prints no
    JSON line (this container has none)."""
    import subprocess
    import sys
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this node has 2 GPUs")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env={k: v for k, v in os.environ.items()
                                                                      if k not in ("WORLD_SIZE", "RANK")})
    assert p.returncode != 0 and "visible" in p.stderr and "{" not in p.stdout


def test_bench_thread_cpu_breakdown():
    """bench.py's per-thread host CPU split (the bench line's host_cpu.threads_cpu_ms_per_step): the launching thread
    is reported as 'main' and a busy helper thread by its OS name (Python thread names are not OS names)."""
    import threading
    import time as _time
    import bench
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            pass
    a = bench.thread_cpu()
    t0 = _time.time()
    while _time.time() - t0 < 0.2:      # the main thread busy
        pass
    th = threading.Thread(target=spin, name="spinner")
    th.start()
    _time.sleep(0.3)                     # the helper busy, the main thread asleep
    b = bench.thread_cpu()
    stop.set()
    th.join()
    rows = bench.thread_cpu_diff(a, b, 1)
    assert dict(rows).get("main", 0) >= 100 and any(n != "main" and ms >= 100 for n, ms in rows), rows


def test_held_dp_policy():
    """task.submit's policy for holding a batch's forward DP (ForcedAlignmentTask.dp_ranges): one range per encoder
    layer from defer_dp_frames DP frames on (config 5's 300 s: 25 839 frames, 12 layers), one launch below it, for a
    one-layer encoder, or when holding is switched off."""
    from types import SimpleNamespace
    from hubertfa_amd.task import ForcedAlignmentTask

    def task(layers, defer=ForcedAlignmentTask.defer_dp_frames):
        return SimpleNamespace(defer_dp_frames=defer,
                               unitsEncoder=SimpleNamespace(model=SimpleNamespace(layers=[None] * layers)))
    rng = ForcedAlignmentTask.dp_ranges
    assert ForcedAlignmentTask.defer_dp_frames == 16384
    assert rng(task(12), 25840, 1808) == 12 and rng(task(24), 25840, 1808) == 24
    assert rng(task(12), 16384, 96) == 12 and rng(task(12), 16383, 96) == 1
    assert rng(task(12), 862, 96) == 1                      # config 2
    assert rng(task(1), 25840, 1808) == 1 and rng(task(12, None), 25840, 1808) == 1


def test_held_dp_failure_stays_with_its_batch():
    """a held batch's DP step that raises (here under the next batch's encoder, through the gate's
    _next, then through that encoder's drain) is kept by the held batch: the later steps and the completion do not
    run (no backtrack over a DP missing a time range), the next batch sees nothing, and the held batch's own
    resolve() -- its decoder.assemble -- raises the error.  A step is dropped only after it ran."""
    from types import SimpleNamespace
    from hubertfa_amd.task import _HeldDP
    ran, fetched = [], []

    def step(i, fail=False):
        def f():
            if fail:
                raise RuntimeError(f"step {i} failed")
            ran.append(i)
        return f
    task = SimpleNamespace(_side=None, decoder=SimpleNamespace(fetch=lambda d: fetched.append(d) or {"n": 1}))
    # healthy: every step once, in order, then the completion (fetch) fills the handle
    h = _HeldDP(task, {"deferred": [step(0), step(1), step(2)]}, None)
    task._held = h
    h._next()
    assert ran == [0] and h.steps and "resolve" in h.handle
    h.drain()
    assert ran == [0, 1, 2] and fetched and h.handle == {"n": 1} and task._held is None
    h.flush()                                        # nothing left, no error
    # failing middle step: the rest never runs, nothing is fetched, drain() (the next submit) does not raise
    ran.clear()
    fetched.clear()
    h = _HeldDP(task, {"deferred": [step(0), step(1, fail=True), step(2), step(3)]}, None)
    task._held = h
    h._next()
    h._next()                                        # the gate's call under the next encoder: captured
    assert ran == [0] and isinstance(h.error, RuntimeError) and not h.steps and task._held is None
    h.drain()
    assert ran == [0] and not fetched and "resolve" in h.handle
    with pytest.raises(RuntimeError, match="step 1 failed"):
        h.handle["resolve"]()                        # this batch's assemble raises it
    # a failing completion (on_device / fetch) is the batch's error too
    h = _HeldDP(task, {"deferred": [step(5)]}, lambda d: (_ for _ in ()).throw(ValueError("gather failed")))
    h.drain()
    with pytest.raises(ValueError, match="gather failed"):
        h.flush()


def test_held_dp_failure_reraised_on_retry_and_prompt_under_distributed(monkeypatch):
    """decoder.assemble keeps a held handle's resolve until it succeeds, so a caller that catches the
    held batch's error and assembles again gets the same error (not a KeyError); and in a multi-rank run whose
    on_device is the boundary collective, the failing step raises at once instead of leaving the peers in it."""
    from types import SimpleNamespace
    from hubertfa_amd import task as task_mod
    from hubertfa_amd.alignment_decoder import AlignmentDecoder
    from hubertfa_amd.task import _HeldDP

    def bad():
        raise RuntimeError("dp range failed")
    tk = SimpleNamespace(_side=None, decoder=SimpleNamespace(fetch=lambda d: {"n": 1}))
    h = _HeldDP(tk, {"deferred": [bad]}, None)
    h.drain()
    dec = AlignmentDecoder({"vocab": {"SP": 0, "a": 1}, "vocab_size": 2}, {"sample_rate": 44100, "hop_length": 512})
    for _ in range(2):
        with pytest.raises(RuntimeError, match="dp range failed"):
            dec.assemble(h.handle, [["SP", "a", "SP"]])
    assert "resolve" in h.handle
    # distributed with a collective completion: the gate's step raises immediately
    monkeypatch.setattr(task_mod, "_dist_world", lambda: 2)
    h = _HeldDP(tk, {"deferred": [bad]}, lambda d: None)
    with pytest.raises(RuntimeError, match="dp range failed"):
        h._next()
    assert h.error is not None and not h.steps
    # without a collective completion it stays deferred even at world 2
    h = _HeldDP(tk, {"deferred": [bad]}, None)
    h._next()
    assert h.error is not None


def test_interval_assembly_array_form_matches_loop():
    """intervals.assemble_intervals (array form) against the reference-order loop (assemble_intervals_loop,
    alignment_decoder.py:103-138) on random paths: SP-heavy and SP-free sequences, repeated word indices, a single
    phone, an all-SP path, an empty path, AP-like id-0 phones inside words; values and dtypes equal."""
    from hubertfa_amd.intervals import assemble_intervals, assemble_intervals_loop
    rng = np.random.default_rng(5)
    phones = ["a", "b", "cc", "ddd", "SP", "AP", "e"]
    for case in range(300):
        S = int(rng.integers(1, 60))
        ph_seq = [phones[int(k)] for k in rng.integers(0, len(phones), S)]
        if case % 7 == 0:
            ph_seq = ["SP"] * S
        words, p2w, w = [], [], -1
        for p in ph_seq:
            if p == "SP":
                p2w.append(-1)
                continue
            if w < 0 or rng.random() < 0.5:
                w += 1
                words.append(f"w{w}")
            p2w.append(w if rng.random() > 0.1 or w == 0 else w - 1)      # sometimes back to an earlier word
        T = int(rng.integers(max(S, 1), 300))
        n = int(rng.integers(0, S + 1)) if case % 11 else 0
        idx = np.sort(rng.choice(S, n, replace=False))
        tint = np.sort(rng.choice(T, n, replace=False))
        ed = rng.standard_normal(T)
        a = assemble_intervals(idx, tint, ed, T, 512 / 44100, ph_seq, words, p2w)
        b = assemble_intervals_loop(idx, tint, ed, T, 512 / 44100, ph_seq, words, p2w)
        for x, y in zip(a, b):
            assert x.dtype == y.dtype and x.shape == y.shape and np.array_equal(x, y), case


def test_batch_results_match_per_utterance():
    """intervals.batch_results (decoder.assemble's batched host assembly) gives every utterance exactly what
    utterance_result gives it from its own raw record: ragged n and T, a path ending on the last frame (its edge_diff
    entry replaced by 0), garbage past n and T in the padded buffers, default word sequences; with the transcript
    tables prebuilt (task.submit) for the same sequences, and for a copy of them (rebuilt, not used)."""
    from hubertfa_amd.intervals import batch_results, batch_tables, utterance_result
    rng = np.random.default_rng(9)
    phones = ["SP", "a", "b", "AP", "cc"]
    for trial in range(20):
        B = int(rng.integers(1, 9))
        Tmax, maxn = 300, 120
        Ts = [int(rng.integers(1, Tmax + 1)) for _ in range(B)]
        ph_seqs, word_seqs, p2ws, recs = [], [], [], []
        idx_h = rng.integers(-5, 99, (B, maxn)).astype(np.int32)          # garbage beyond n
        tint_h = rng.integers(-9, 10 ** 6, (B, maxn)).astype(np.int32)
        fc_h = rng.random((B, Tmax)).astype(np.float32)
        ed_h = rng.standard_normal((B, Tmax)).astype(np.float32)
        n_h = np.zeros(B, np.int32)
        for b in range(B):
            S = int(rng.integers(1, 40))
            ph = ["SP"] + [phones[int(k)] for k in rng.integers(0, len(phones), S)]
            words, p2w, w = [], [], -1
            for p in ph:
                if p == "SP":
                    p2w.append(-1)
                    continue
                if w < 0 or rng.random() < 0.6:
                    w += 1
                    words.append(f"w{w}")
                p2w.append(w)
            n = int(rng.integers(0, min(len(ph), Ts[b]) + 1))
            n_h[b] = n
            idx_h[b, :n] = np.sort(rng.choice(len(ph), n, replace=False))
            t = np.sort(rng.choice(Ts[b], n, replace=False))
            if n and trial % 2:
                t[-1] = Ts[b] - 1
            tint_h[b, :n] = t
            default = trial % 5 == 0
            ph_seqs.append(ph)
            word_seqs.append(None if default else words)
            p2ws.append(None if default else p2w)
        tabs = batch_tables(ph_seqs, word_seqs, p2ws) if trial % 2 else batch_tables(list(ph_seqs), word_seqs, p2ws)
        got = batch_results(Ts, idx_h, tint_h, n_h, fc_h, ed_h, ph_seqs, word_seqs, p2ws, 512 / 44100, tables=tabs)
        for b in range(B):
            k, T = int(n_h[b]), Ts[b]
            rec = dict(T=T, ph_idx_seq=idx_h[b, :k].astype(np.int64), ph_time_int=tint_h[b, :k].astype(np.int64),
                       frame_confidence=fc_h[b, :T].copy(), edge_diff=ed_h[b, :T].copy())
            ws = word_seqs[b] if word_seqs[b] is not None else ph_seqs[b]
            pw = p2ws[b] if p2ws[b] is not None else np.arange(len(ph_seqs[b]))
            ref = utterance_result(rec, ph_seqs[b], ws, pw, 512 / 44100)
            assert got[b].keys() == ref.keys()
            for key in ref:
                x, y = np.asarray(got[b][key]), np.asarray(ref[key])
                assert x.dtype == y.dtype and x.shape == y.shape and np.array_equal(x, y), (trial, b, key)


def test_batch_results_irregular_utterances():
    """batch_results on utterances the flat batch form cannot take (assembled alone, as the reference's loop would):
    a kept phone mapped to word -1 after a word (the loop reuses word_seq[-1]) and a word map longer than the phone
    list, beside regular utterances; and the errors the reference raises (a first kept phone without a word, a word
    index past the word list, a word map too short) raised the same."""
    from hubertfa_amd.intervals import batch_results, utterance_result
    ph = ["SP", "a", "b", "c", "SP", "d"]
    words = ["w0", "w1", "w2"]
    good = [[-1, 0, 0, 1, -1, 2], [-1, 0, 1, -1, -1, 2], [-1, 0, 0, 1, -1, 2, 2], [-1, 0, 1, 1, -1, 2]]
    T, n, B = 40, 6, 4
    idx_h = np.tile(np.arange(n, dtype=np.int32), (B, 1))
    tint_h = np.tile(np.array([0, 5, 9, 14, 22, 30], np.int32), (B, 1))
    rng = np.random.default_rng(3)
    fc_h = rng.random((B, T)).astype(np.float32)
    ed_h = rng.standard_normal((B, T)).astype(np.float32)
    n_h = np.full(B, n, np.int32)
    Ts, ph_seqs, word_seqs = [T] * B, [ph] * B, [words] * B
    got = batch_results(Ts, idx_h, tint_h, n_h, fc_h, ed_h, ph_seqs, word_seqs, good, 512 / 44100)
    for b in range(B):
        rec = dict(T=T, ph_idx_seq=idx_h[b].astype(np.int64), ph_time_int=tint_h[b].astype(np.int64),
                   frame_confidence=fc_h[b].copy(), edge_diff=ed_h[b].copy())
        ref = utterance_result(rec, ph, words, good[b], 512 / 44100)
        for key in ref:
            x, y = np.asarray(got[b][key]), np.asarray(ref[key])
            assert x.dtype == y.dtype and x.shape == y.shape and np.array_equal(x, y), (b, key)
    for bad in ([-1, -1, 0, 1, -1, 2], [-1, 0, 0, 1, -1, 7], [-1, 0, 0, 1, -1]):
        with pytest.raises(IndexError):
            utterance_result(dict(T=T, ph_idx_seq=idx_h[0].astype(np.int64), ph_time_int=tint_h[0].astype(np.int64),
                                  frame_confidence=fc_h[0].copy(), edge_diff=ed_h[0].copy()), ph, words, bad,
                             512 / 44100)
        with pytest.raises(IndexError):
            batch_results(Ts, idx_h, tint_h, n_h, fc_h, ed_h, ph_seqs, word_seqs, good[:2] + [bad] + good[3:],
                          512 / 44100)


def test_fill_small_gaps_rows_form_matches_element_form():
    """post_processing.fill_small_gaps (the reference's loop run on the rows as Python floats, written back in place)
    against the same loop on numpy elements (tools/post_processing.py:34-67's statement order), 600 random interval
    sets: AP neighbours on either / both sides, gaps under and over both thresholds, leading and trailing gaps,
    touching and overlapping intervals; values and the caller's array equal."""
    from hubertfa_amd.post_processing import MIN_SP_LENGTH, SP_MERGE_LENGTH, fill_small_gaps

    def element_form(seq, iv, wav_length):
        if iv[0, 0] > 0 and iv[0, 0] < MIN_SP_LENGTH:
            iv[0, 0] = 0
        for i in range(len(seq) - 1):
            if iv[i, 1] < iv[i + 1, 0] and iv[i + 1, 0] - iv[i, 1] < SP_MERGE_LENGTH:
                if seq[i] == "AP":
                    if seq[i + 1] == "AP":
                        iv[i, 1] = (iv[i, 1] + iv[i + 1, 0]) / 2
                        iv[i + 1, 0] = iv[i, 1]
                    else:
                        iv[i, 1] = iv[i + 1, 0]
                elif seq[i + 1] == "AP":
                    iv[i + 1, 0] = iv[i, 1]
                elif iv[i + 1, 0] - iv[i, 1] < MIN_SP_LENGTH:
                    iv[i, 1] = (iv[i, 1] + iv[i + 1, 0]) / 2
                    iv[i + 1, 0] = iv[i, 1]
        if iv[-1, 1] < wav_length and wav_length - iv[-1, 1] < MIN_SP_LENGTH:
            iv[-1, 1] = wav_length
        return seq, iv

    rng = np.random.default_rng(11)
    for case in range(600):
        n = int(rng.integers(1, 40))
        seq = [("AP" if rng.random() < 0.3 else f"p{int(rng.integers(0, 5))}") for _ in range(n)]
        starts = np.cumsum(rng.choice([0.0, 0.05, 0.15, 0.35, rng.uniform(0, 0.5)], n))
        lens = rng.uniform(0.01, 0.4, n)
        iv = np.stack([starts + np.arange(n) * 0.2, starts + np.arange(n) * 0.2 + lens], 1)
        if case % 5 == 0:
            iv[:, 0] -= rng.uniform(0, 0.1)                  # overlaps and touching ends
        wav_length = float(iv[-1, 1] + rng.choice([0.0, 0.05, 0.2]))
        a, b = iv.copy(), iv.copy()
        _, ra = fill_small_gaps(seq, a, wav_length)
        _, rb = element_form(seq, b, wav_length)
        assert ra is a and np.array_equal(a, b), case
