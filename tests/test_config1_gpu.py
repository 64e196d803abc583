"""BASELINE config 1, literally: one 5 s 16 kHz WAV + the opencpop-extension dictionary through the infer.py CLI
(reference: infer.py:43-72 with its default -g Dictionary and -d dictionary/opencpop-extension.txt).

The dictionary file is rebuilt from the opencpop-extension entries the reference's DictionaryG2P was run over
(tests/golden/g2p_dicts.json: 71 entries, 52 phones); the checkpoint's vocabulary is those phones + SP (= 0, AP
ignored) padded to the opencpop-extension size (62 phones, V = 63, as the binarizer would build it), with the
synthetic UNet/head and synth:0 Hubert-base weights.  Checked: the TextGrid's words equal the .lab, the phone tier
ends at 5 s, the CLI's file equals the one the reference-API path (predict_step -> post_processing -> Exporter)
writes byte for byte, and confidence.csv names the file."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _opencpop_setup(tmp_path):
    import yaml
    from hubertfa_amd import synth
    from hubertfa_amd.task import synth_checkpoint
    from hubertfa_amd.wav_io import write_wav
    gold = json.load(open(os.path.join(GOLDEN, "g2p_dicts.json"), encoding="utf-8"))["opencpop-extension"]
    entries = gold["entries"]
    dpath = tmp_path / "opencpop-extension.txt"
    dpath.write_text("".join(f"{w}\t{' '.join(p)}\n" for w, p in entries.items()), encoding="utf-8")
    phones = sorted({p for v in entries.values() for p in v})
    phones += [f"zz{i:02d}" for i in range(62 - len(phones))]          # opencpop-extension has 62 phones
    vocab = {"SP": 0, "AP": 0}
    vocab.update({p: i + 1 for i, p in enumerate(phones)})
    vocab = {"vocab": vocab, "vocab_size": 63, "ignored_phonemes": ["AP", "SP"]}
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    ck["hyper_parameters"]["vocab_text"] = yaml.safe_dump(vocab)
    ckpt = tmp_path / "model.ckpt"
    torch.save(ck, ckpt)
    seg = tmp_path / "segments"
    seg.mkdir()
    rng = np.random.default_rng(15)
    words = sorted(entries)
    lab = " ".join(words[int(i)] for i in rng.integers(0, len(words), 15))     # W = 15
    write_wav(seg / "utt.wav", synth.synth_audio(5 * 16000, seed=15), 16000)
    (seg / "utt.lab").write_text(lab, encoding="utf-8")
    return ckpt, dpath, seg, lab


def test_config1_cli_single_5s_wav_opencpop(tmp_path):
    from click.testing import CliRunner
    import infer
    import hubertfa_amd.g2p as g2p_mod
    from hubertfa_amd.export_tool import Exporter, read_textgrid
    from hubertfa_amd.post_processing import post_processing
    from hubertfa_amd.task import ForcedAlignmentTask
    ckpt, dpath, seg, lab = _opencpop_setup(tmp_path)
    r = CliRunner().invoke(infer.main, ["-c", str(ckpt), "-f", str(seg), "-d", str(dpath), "-sc",
                                        "--hubert_path", "synth:0"])
    assert r.exit_code == 0, r.output + repr(r.exception)
    tg_path = seg / "TextGrid" / "utt.TextGrid"
    tg = read_textgrid(tg_path)
    assert [t[2] for t in tg["words"] if t[2] != "SP"] == lab.split(" ")
    assert abs(tg["phones"][-1][1] - 5.0) < 1e-9 and tg["phones"][0][0] == 0.0
    g = g2p_mod.DictionaryG2P(dictionary=str(dpath))
    g.set_in_format("lab")
    rows = list(g.get_dataset(sorted(seg.rglob("*.wav"))))
    entries = json.load(open(os.path.join(GOLDEN, "g2p_dicts.json"), encoding="utf-8"))["opencpop-extension"]["entries"]
    assert len(rows) == 1 and len(rows[0][1]) == 1 + sum(len(entries[w]) + 1 for w in lab.split(" "))
    torch.set_grad_enabled(False)
    task = ForcedAlignmentTask.load_from_checkpoint(str(ckpt), device=torch.device("cuda"),
                                                    hubert_model_path="synth:0")
    task.on_predict_start()
    pred = task.predict_step(rows[0], 0)                            # the reference API's per-utterance path
    preds, log = post_processing([pred])
    assert not log
    out = tmp_path / "api"
    Exporter(preds, log, out).export(["textgrid"])
    assert (out / "TextGrid" / "utt.TextGrid").read_bytes() == tg_path.read_bytes()
    conf = (seg / "confidence" / "confidence.csv").read_text().splitlines()
    assert conf[0] == "name,confidence" and conf[1].startswith("utt,")
