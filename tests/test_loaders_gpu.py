"""The product's checkpoint loaders on the files the reference's loaders read (VERDICT r02 'next' 3).

tests/ckpt_files.py rebuilds each file from seeded weights (HF folders through transformers' save_pretrained, a
bshall .pt, a Lightning-layout .ckpt); tests/golden/loaders.npz holds what the reference computed from the same
files (gen_golden.py gen_loaders: its Audio2CNHubert / Audio2HubertSoft loaders, tools/encoder.py:63-96, and its
UNetBackbone + head).  Each file is loaded here by the product's own entry points —
``UnitsEncoder(encoder, path)`` (encoder.load_hubert) and ``ForcedAlignmentTask.load_from_checkpoint`` — and its
outputs are compared with the stored ones."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
UNITS_TOL = 2e-4            # 2-layer encoders (12 for hubertsoft) at 1 s, f32-class contractions


def _gold():
    return np.load(os.path.join(GOLDEN, "loaders.npz")), json.load(open(os.path.join(GOLDEN, "loaders.json")))


@pytest.mark.parametrize("kind", ["hf", "hf_nonorm", "hf_legacy"])
def test_hf_folder_loader(tmp_path, kind):
    """HubertModel folders: safetensors with parametrized weight norm, preprocessor do_normalize true/false, and
    the legacy pytorch_model.bin with weight_g/weight_v under a "hubert." prefix."""
    pytest.importorskip("transformers")
    import ckpt_files
    from hubertfa_amd.encoder import UnitsEncoder
    z, _ = _gold()
    path = str(tmp_path / kind)
    ckpt_files.write_hf_folder(path, kind)
    ue = UnitsEncoder("cnhubert", path, 16000, 320, device="cuda")
    assert ue.model.arch.do_normalize == (kind != "hf_nonorm")
    assert ue.model.arch.layers == ckpt_files.LOADER_LAYERS
    units = ue.model(torch.from_numpy(z["wav"])[None].cuda())[0].cpu().numpy()
    ref = z["hf_nonorm_units"] if kind == "hf_nonorm" else z["hf_units"]
    err = float(np.abs(units - ref).max())
    print(f"[{kind}] units error vs the reference loader: {err:.2e}")
    assert units.shape == ref.shape and err < UNITS_TOL


def test_bshall_loader(tmp_path):
    """torch.load(path)["hubert"] with DataParallel's "module." prefix (tools/encoder.py:69-71)."""
    import ckpt_files
    from hubertfa_amd.encoder import UnitsEncoder
    z, _ = _gold()
    path = str(tmp_path / "soft.pt")
    ckpt_files.write_bshall(path)
    ue = UnitsEncoder("hubertsoft", path, 16000, 320, device="cuda")
    units = ue.model(torch.from_numpy(z["wav"])[None].cuda())[0].cpu().numpy()
    err = float(np.abs(units - z["soft_units"]).max())
    print(f"[bshall] units error vs the reference loader: {err:.2e}")
    assert units.shape == z["soft_units"].shape and err < UNITS_TOL


def test_lightning_ckpt_loader(tmp_path):
    """A Lightning-layout .ckpt (loss-module buffers in the state_dict, trainer bookkeeping, hyper_parameters from
    configs/train_config.yaml) through load_from_checkpoint: the buffers are ignored, the UNet + head logits equal
    the reference modules' on the same input, and on_predict_start builds the units encoder named by the
    checkpoint's hubert_config (a HF folder)."""
    pytest.importorskip("transformers")
    import ckpt_files
    from hubertfa_amd import synth
    from hubertfa_amd.task import ForcedAlignmentTask
    z, meta = _gold()
    folder = str(tmp_path / "cnhubert")
    ckpt_files.write_hf_folder(folder, "hf")
    path = str(tmp_path / "model.ckpt")
    ck = ckpt_files.write_lightning_ckpt(path, meta, hubert_model_path=folder)
    assert any(k.startswith("CTC_GHM_loss_fn.") for k in ck["state_dict"])
    task = ForcedAlignmentTask.load_from_checkpoint(path, device=torch.device("cuda"))
    assert task.hubert_config["encoder"] == "cnhubert" and task.melspec_config["hop_length"] == 512
    x = synth.rng(meta["unet_input_seed"]).standard_normal((1, meta["unet_input_T"], 768)).astype(np.float32)
    frame, edge, ctc = task.forward(torch.from_numpy(x))
    ref = z["ckpt_logits"]
    err = max(float(np.abs(frame[0].cpu().numpy() - ref[:, 2:]).max()),
              float(np.abs(edge[0].cpu().numpy() - ref[:, 0]).max()),
              float(np.abs(ctc[0, :, 0].cpu().numpy() - ref[:, 1]).max()),
              float(np.abs(ctc[0, :, 1:].cpu().numpy() - ref[:, 3:]).max()))
    print(f"[ckpt] logits error vs the reference UNet + head: {err:.2e}")
    assert err < 2e-4
    task.on_predict_start()
    units = task.unitsEncoder.model(torch.from_numpy(z["wav"])[None].cuda())[0].cpu().numpy()
    assert float(np.abs(units - z["hf_units"]).max()) < UNITS_TOL
