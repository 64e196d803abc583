"""The RCCL code path of the boundary gather, executed on one GPU: a world-size-1 ``nccl`` process group (RCCL on
ROCm), gather_boundaries with the one-rank shortcut bypassed, issued from the side stream after the backtrack
exactly as bench.py's N > 1 step does (task.submit on_device), in both forms: the uniform-shape fast path (bench)
and the shape-exchange path (infer.py's gather_records over packed tables).  Multi-rank correctness is covered
over gloo (tests/test_host.py, tests/test_cli_gpu.py); this runs the same calls on the backend the 8-GPU run
uses."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture
def nccl_world1():
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_rccl_boundary_gather_from_side_stream(nccl_world1):
    import bench
    from hubertfa_amd import distributed as hd
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    assert nccl_world1.get_backend() == "nccl"
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=torch.device("cuda"))
    wav, ph, ws, pw = bench.make_inputs(3, 2.0, 6, 31)
    got = {}

    def on_device(dev_out):                     # runs on task.submit's side stream, after the backtrack
        assert torch.cuda.current_stream() != torch.cuda.default_stream()
        got["g"] = hd.gather_boundaries(dev_out, uniform=True, shortcut=False)
        got["local"] = {k: dev_out[k].clone() for k in hd.BOUNDARY_KEYS}
    handle = task.submit(torch.from_numpy(wav).cuda(), ph, ws, pw, wav_sr=16000, on_device=on_device)
    res = task.decoder.assemble(handle, ph, ws, pw)
    torch.cuda.synchronize()
    for k in hd.BOUNDARY_KEYS:
        assert len(got["g"][k]) == 1
        assert got["g"][k][0].is_cuda and torch.equal(got["g"][k][0], got["local"][k]), k
    n = got["g"]["n"][0].cpu().numpy()
    for b in range(3):
        assert np.array_equal(got["g"]["ph_time_int"][0][b, :n[b]].cpu().numpy(), res[b]["ph_time_int"])


def test_rccl_record_table_gather(nccl_world1):
    """infer.py's multi-GPU gather (packed per-utterance tables, shapes exchanged first) over RCCL."""
    from hubertfa_amd import distributed as hd
    rng = np.random.default_rng(0)
    records = {}
    for key in (4, 1, 9):
        T = int(rng.integers(50, 90))
        n = int(rng.integers(3, 12))
        records[key] = dict(n44=T * 512, T=T, ph_idx_seq=np.sort(rng.choice(40, n, replace=False)),
                            ph_time_int=np.sort(rng.choice(T, n, replace=False)),
                            frame_confidence=rng.random(T).astype(np.float32),
                            edge_diff=rng.random(T).astype(np.float32))
    tab = {k: v.cuda() for k, v in hd.pack_records(records).items()}
    out = hd.unpack_records(hd.gather_boundaries(tab, hd.TABLE_KEYS, shortcut=False))
    assert sorted(out) == sorted(records)
    for key, r in records.items():
        for f in ("ph_idx_seq", "ph_time_int", "frame_confidence", "edge_diff"):
            assert np.array_equal(out[key][f], r[f]), (key, f)
        assert out[key]["T"] == r["T"] and out[key]["n44"] == r["n44"]
