"""Drop-in CLI for the reference ``infer.py`` (reference: infer.py:13-72), running the MI355X path.

    python infer.py -c model.ckpt -f segments [-g Dictionary] [-d dictionary/opencpop-extension.txt] [-sc]

Same flags and defaults as the reference; extra flags: ``--hubert_path`` (override hubert_config.model_path, e.g.
``synth:0``), ``--batch_size`` (utterances per GPU batch: sorted by length, zero-padded, aligned with per-row
lengths so every result equals the one-utterance run), ``--out_path``.
Launched under ``torchrun --nproc-per-node N`` it shards the wav files across ranks by estimated cost (LPT);
rank 0 gathers the per-utterance results and writes the TextGrids / confidence.csv.
"""
from __future__ import annotations

import pathlib

import click


def _predict(task, dataset, batch_size: int):
    import torch
    from hubertfa_amd.batching import plan_batches, resampled_length
    from hubertfa_amd.wav_io import read_wav

    task.on_predict_start()
    sr = task.melspec_config["sample_rate"]
    items = []
    for wav_path, ph_seq, word_seq, p2w in dataset:
        x, file_sr = read_wav(wav_path)
        items.append((wav_path, x[0], file_sr, ph_seq, word_seq, p2w))
    # variable-length batches (hubertfa_amd.batching.plan_batches): per sample rate, sorted by length, rows
    # zero-padded and aligned with per-row lengths, which keeps every utterance's result identical to aligning it
    # alone (the reference's B=1); files too short for the encoder's 400-sample window are aligned alone
    out = {}
    by_key = {i: it for i, it in enumerate(items)}

    def finish(job):
        handle, chunk, n44s = job
        res = task.decoder.assemble(handle, [c[3] for c in chunk], [c[4] for c in chunk], [c[5] for c in chunk])
        for c, r, n44 in zip(chunk, res, n44s):
            out[str(c[0])] = (c[0], n44 / sr, r["confidence"], r["ph_seq"], r["ph_intervals"], r["word_seq"],
                              r["word_intervals"])

    def batches():
        plan = plan_batches([(i, len(it[1]), it[2]) for i, it in by_key.items()], batch_size, sr,
                            task.unitsEncoder.encoder_sample_rate)
        for file_sr, keys in plan:
            yield file_sr, [by_key[k] for k in keys]

    # one batch in flight: the host assembles batch i while the GPU runs batch i+1 (task.submit: encoder on the
    # main stream, head + Viterbi on a side stream)
    pending = None
    for file_sr, chunk in batches():
        lens = [len(c[1]) for c in chunk]
        wav_h = torch.zeros((len(chunk), max(lens)), dtype=torch.float32, pin_memory=True)
        wav_np = wav_h.numpy()           # rows written straight into pinned memory
        for r, c in enumerate(chunk):
            wav_np[r, :lens[r]] = c[1]
        wav = task.upload(wav_h)         # pinned non-blocking H2D: no host sync
        handle = task.submit(wav, [c[3] for c in chunk], [c[4] for c in chunk], [c[5] for c in chunk],
                             wav_sr=file_sr, lengths=lens if len(chunk) > 1 else None)
        n44s = [resampled_length(n, file_sr, sr) for n in lens]
        if pending is not None:
            finish(pending)
        pending = (handle, chunk, n44s)
    if pending is not None:
        finish(pending)
    return [out[str(it[0])] for it in items if str(it[0]) in out]


@click.command()
@click.option("--ckpt", "-c", default=None, required=True, type=str, help="path to the checkpoint")
@click.option("--folder", "-f", default="segments", type=str, help="path to the input folder")
@click.option("--g2p", "-g", default="Dictionary", type=str, help="name of the g2p class")
@click.option("--save_confidence", "-sc", is_flag=True, default=False, show_default=True, help="save confidence.csv")
@click.option("--dictionary", "-d", default="dictionary/opencpop-extension.txt", type=str,
              help="(only used when --g2p=='Dictionary') path to the dictionary")
@click.option("--hubert_path", default=None, type=str, help="override hubert_config.model_path")
@click.option("--batch_size", default=32, type=int, help="max utterances per GPU batch (variable lengths; results equal B=1)")
@click.option("--out_path", default=None, type=str, help="write TextGrids under this folder instead")
def main(ckpt, folder, g2p, save_confidence, hubert_path, batch_size, out_path, **kwargs):
    import os
    import torch
    import hubertfa_amd.g2p as g2p_mod
    from hubertfa_amd.distributed import env_rank_world, shard_lpt, utterance_cost
    from hubertfa_amd.export_tool import Exporter
    from hubertfa_amd.post_processing import post_processing
    from hubertfa_amd.task import ForcedAlignmentTask

    if not g2p.endswith("G2P"):
        g2p += "G2P"
    grapheme_to_phoneme = getattr(g2p_mod, g2p)(**kwargs)
    grapheme_to_phoneme.set_in_format("lab")
    dataset = grapheme_to_phoneme.get_dataset(sorted(pathlib.Path(folder).rglob("*.wav")))

    rank, world, local = env_rank_world()
    torch.cuda.set_device(local)
    rows = list(dataset)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        costs = [utterance_cost(os.path.getsize(r[0]) // 2, len(r[1])) for r in rows]
        rows = [rows[i] for i in shard_lpt(costs, world)[rank]]

    torch.set_grad_enabled(False)
    model = ForcedAlignmentTask.load_from_checkpoint(ckpt, device=torch.device("cuda", local),
                                                     hubert_model_path=hubert_path)
    predictions = _predict(model, rows, batch_size)
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, predictions)
        predictions = [p for part in gathered for p in part]
        if rank != 0:
            dist.destroy_process_group()
            return
    predictions, log = post_processing(predictions)
    exporter = Exporter(predictions, log, out_path)
    out_formats = ["textgrid"] + (["confidence"] if save_confidence else [])
    exporter.export(out_formats)
    print("Output files are saved to the same folder as the input wav files.")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
