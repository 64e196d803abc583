"""The infer.py drop-in CLI on a folder of synthetic wav/.lab pairs -> TextGrids + confidence.csv."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_infer_cli_end_to_end(tmp_path):
    from click.testing import CliRunner
    import infer
    from hubertfa_amd import synth
    from hubertfa_amd.export_tool import read_textgrid
    from hubertfa_amd.task import synth_checkpoint
    from hubertfa_amd.wav_io import write_wav
    d = synth.synth_dictionary(n_words=40)
    dpath = tmp_path / "dict.txt"
    dpath.write_text("".join(f"{w}\t{' '.join(p)}\n" for w, p in d.items()))
    seg = tmp_path / "segments"
    seg.mkdir()
    SECS = (2.0, 2.0, 3.5, 2.7, 1.3)
    for i, secs in enumerate(SECS):
        write_wav(seg / f"u{i}.wav", synth.synth_audio(int(secs * 16000), seed=i), 16000)
        (seg / f"u{i}.lab").write_text(synth.synth_lab(5, d, seed=i))
    ck = tmp_path / "m.ckpt"
    synth_checkpoint(str(ck))
    r = CliRunner().invoke(infer.main, ["-c", str(ck), "-f", str(seg), "-d", str(dpath), "-sc",
                                        "--hubert_path", "synth:0"])
    assert r.exit_code == 0, r.output + repr(r.exception)
    for i, secs in enumerate(SECS):
        tg = read_textgrid(seg / "TextGrid" / f"u{i}.TextGrid")
        words = [t for t in tg["words"] if t[2] != "SP"]
        assert [w[2] for w in words] == synth.synth_lab(5, d, seed=i).split(" ")
        assert abs(tg["phones"][-1][1] - secs) < 1e-3
    assert (seg / "confidence" / "confidence.csv").exists()
    # variable-length batches (default) write exactly what one-utterance batches (the reference's B=1) write
    batched = {i: (seg / "TextGrid" / f"u{i}.TextGrid").read_text() for i in range(len(SECS))}
    out1 = tmp_path / "one"
    r = CliRunner().invoke(infer.main, ["-c", str(ck), "-f", str(seg), "-d", str(dpath), "--hubert_path", "synth:0",
                                        "--batch_size", "1", "--out_path", str(out1)])
    assert r.exit_code == 0, r.output + repr(r.exception)
    for i in range(len(SECS)):
        one = next(out1.rglob(f"u{i}.TextGrid")).read_text()
        assert one == batched[i], f"u{i}: batched TextGrid differs from the B=1 run"
