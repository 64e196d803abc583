"""Drop-in CLI for the reference ``infer.py`` (reference: infer.py:13-72), running the MI355X path.

    python infer.py -c model.ckpt -f segments [-g Dictionary] [-d dictionary/opencpop-extension.txt] [-sc]

Same flags and defaults as the reference; extra flags: ``--hubert_path`` (override hubert_config.model_path, e.g.
``synth:0``), ``--batch_size`` (utterances per GPU batch: sorted by length, zero-padded, aligned with per-row
lengths so every result equals the one-utterance run), ``--out_path``.

Multi-GPU (``torchrun --nproc-per-node N infer.py ...``): every rank reads the folder and runs the
G2P, the files are sharded by an LPT on a cost estimate from each WAV header, each rank aligns its shard, and the
per-utterance boundary arrays are gathered to rank 0 (distributed.gather_records: shape all_gather + padded
all_gather_into_tensor over RCCL), which assembles intervals, post-processes and exports — byte-identical to a
one-GPU run.  A rank whose shard fails reports it over a gloo control group; its shard is re-run on the healthy
ranks.  A file that fails alone (a lattice beyond the DP kernel's limits, an unreadable WAV, ...) is recorded in
the error log and skipped instead of aborting the run.
"""
from __future__ import annotations

import os
import pathlib

import click


def _recoverable():
    """Errors that concern one input and leave the GPU healthy: a rejected argument (HFA_EINVAL: a lattice beyond
    the DP kernel's limits, an unreadable WAV), the reference's own per-utterance assertions and lookups.  A HIP
    error (libhfa rc = -(hipError_t)), a missing library or anything else fails the rank, so its shard is re-queued
    on a healthy rank instead of being logged file by file."""
    from hubertfa_amd._lib import HFAArgumentError
    return (HFAArgumentError, ValueError, AssertionError, KeyError, IndexError)


def _export_errors():
    """Errors of one file's post-processing / TextGrid write (e.g. IntervalTier's overlap check)."""
    return (ValueError, AssertionError, KeyError, IndexError, OSError)


class _StreamingExport:
    """One-GPU runs: post-process and write each batch's TextGrids as soon as the batch is back, on the host while
    the GPU runs the next batch, instead of after the whole folder.  The files written are the same; the
    confidence table and the error log are assembled at the end in dataset order, as the batch path does."""

    def __init__(self, rows, sr, frame_length, out_path):
        from hubertfa_amd.export_tool import Exporter
        self.rows, self.sr, self.frame_length = rows, sr, frame_length
        self.writer = Exporter([], [], out_path)
        self.done, self.log, self.made = {}, {}, set()
        print("Post-processing...")
        print("Saving TextGrids...")

    def __call__(self, records: dict, keys):
        from hubertfa_amd.intervals import utterance_result
        from hubertfa_amd.post_processing import post_process_one
        for i in keys:
            wav_path, ph_seq, word_seq, p2w = self.rows[i]
            rec = records[i]
            try:
                # records assembled by the batch (decoder.assemble's batch_results) carry their intervals already
                r = rec if "ph_seq" in rec else utterance_result(rec, ph_seq, word_seq, p2w, self.frame_length)
                pred, err = post_process_one((wav_path, rec["n44"] / self.sr, r["confidence"], r["ph_seq"],
                                              r["ph_intervals"], r["word_seq"], r["word_intervals"]))
                if err is None:
                    self.writer.write_textgrid(pred, self.made)
            except _export_errors() as e:            # this file's export failed: logged as an export error
                pred, err = None, [wav_path, e]
            if err is not None:
                self.log[i] = err
                continue
            self.done[i] = pred

    def results(self):
        """-> (predictions, post-processing log), both in dataset order."""
        return [self.done[i] for i in sorted(self.done)], [self.log[i] for i in sorted(self.log)]


def _predict(task, rows, keys, batch_size: int, errors: list, on_batch=None) -> dict:
    """Align ``rows`` (wav_path, ph_seq, word_seq, ph_idx_to_word_idx); ``keys`` their dataset indices.

    Returns {dataset index: raw boundary record} (alignment_decoder.utterance_result turns a record into the
    reference's decode outputs).  A batch that raises a recoverable error is re-run file by file; a file that
    fails alone goes to ``errors`` as [wav_path, exception] (the post-processing log).  ``on_batch(out, keys)``
    is called with each completed batch's dataset indices (the one-GPU streaming export)."""
    import time

    import torch
    from hubertfa_amd.batching import plan_batches, resampled_length
    from hubertfa_amd.wav_io import read_wav_into, wav_info

    if os.environ.get("HFA_FAULT_INJECT_RANK") == os.environ.get("RANK", "0"):
        raise RuntimeError("fault injected (HFA_FAULT_INJECT_RANK): this rank's shard fails")
    recoverable = _recoverable()
    task.on_predict_start()
    # one GPU (the streaming export): each batch's intervals assembled as one set of array operations when it lands
    # (decoder.assemble -> intervals.batch_results, transcript tables built at submit); multi-GPU: raw records,
    # gathered to rank 0, whose export assembles them (utterance_result: the same values)
    full = on_batch is not None
    task.host_tables = full
    sr = task.melspec_config["sample_rate"]
    items = {}

    def _info(path):
        try:
            return wav_info(path), None
        except (OSError, ValueError) as e:
            return None, e
    # Only the RIFF headers are read up front (lengths for the batch plan); each batch's files are decoded one batch
    # ahead of its launch, by libhfa's native reader straight into the batch's pinned buffer, so host memory holds
    # the batches in flight, not the folder (~70 us per 10 s file, on the loader thread below).
    for key, (wav_path, ph_seq, word_seq, p2w), (info, e) in zip(keys, rows, map(_info, [r[0] for r in rows])):
        if e is not None:
            errors.append([wav_path, e])
            continue
        n, file_sr, _ = info
        items[key] = (wav_path, n, file_sr, ph_seq, word_seq, p2w)
    out = {}

    def _decode(path, row, n):
        got, _ = read_wav_into(path, row, channel=0)     # channel 0, as the reference's waveform[0]
        if got != n:
            raise ValueError(f"{path}: {got} samples read, the header said {n}")
        row[n:] = 0.0                                    # the zero padding past this row's length

    def load(chunk):
        """The batch's files decoded straight into one pinned buffer (rows zero-padded past each length)."""
        lens = [c[1] for c in chunk]
        wav_h = torch.empty((len(chunk), max(lens)), dtype=torch.float32, pin_memory=True)
        wav_np = wav_h.numpy()
        for r, c in enumerate(chunk):
            _decode(c[0], wav_np[r], lens[r])
        return wav_h

    def submit(chunk, file_sr, wav_h=None):
        """-> (fetch handle, per-file sample counts at the melspec rate)."""
        lens = [c[1] for c in chunk]
        if wav_h is None:
            wav_h = load(chunk)
        wav = task.upload(wav_h)         # pinned non-blocking H2D: no host sync
        handle = task.submit(wav, [c[3] for c in chunk], [c[4] for c in chunk], [c[5] for c in chunk],
                             wav_sr=file_sr, lengths=lens if len(chunk) > 1 else None)
        return handle, [resampled_length(n, file_sr, sr) for n in lens]

    def finish(job):
        """Complete a batch's alignment (the export of its files is not part of it: see emit)."""
        handle, ks, n44s = job[:3]
        chunk = [items[k] for k in ks]
        res = task.decoder.assemble(handle, [c[3] for c in chunk], [c[4] for c in chunk], [c[5] for c in chunk],
                                    intervals=full)
        for k, r, n44 in zip(ks, res, n44s):
            out[k] = dict(r, n44=n44) if full else \
                dict(n44=n44, T=r["T"], ph_idx_seq=r["ph_idx_seq"], ph_time_int=r["ph_time_int"],
                     frame_confidence=r["frame_confidence"], edge_diff=r["edge_diff"])
        return ks

    def emit(ks):
        # outside the alignment guards: an export error is logged by on_batch, never taken for a GPU failure
        if on_batch is not None:
            on_batch(out, ks)

    # the next batch's files are decoded on a loader thread while this one is launched and the previous one
    # assembled and exported (the native reader runs outside the GIL); a decode error surfaces in run(), as inline
    from concurrent.futures import ThreadPoolExecutor
    loader, prefetched = ThreadPoolExecutor(max_workers=1, thread_name_prefix="hfa-wav"), {}

    trace = [] if os.environ.get("HFA_CLI_TRACE") else None     # (event, perf_counter) per batch, for profiling

    def run(ks, file_sr):
        if trace is not None:
            trace.append(("submit", time.perf_counter()))
        fut = prefetched.pop(tuple(ks), None)
        wav_h = fut.result() if fut is not None else None
        if trace is not None:
            trace.append(("loaded", time.perf_counter()))
        handle, n44s = submit([items[k] for k in ks], file_sr, wav_h)
        if trace is not None:
            trace.append(("submitted", time.perf_counter()))
        return handle, ks, n44s, file_sr

    def alone(k, file_sr):
        try:
            ks = finish(run([k], file_sr))
        except recoverable as e:
            errors.append([items[k][0], e])
            return
        emit(ks)

    def settle(job):
        """Complete a batch; a recoverable failure re-runs its files one by one."""
        if trace is not None:
            trace.append(("settle", time.perf_counter()))
        try:
            ks = finish(job)
        except recoverable as e:
            if len(job[1]) == 1:
                errors.append([items[job[1][0]][0], e])
            else:
                for k in job[1]:
                    alone(k, job[3])
            return
        if trace is not None:
            trace.append(("assembled", time.perf_counter()))
        emit(ks)
        if trace is not None:
            trace.append(("exported", time.perf_counter()))

    # variable-length batches (hubertfa_amd.batching.plan_batches): per sample rate, sorted by length, rows
    # zero-padded and aligned with per-row lengths, which keeps every utterance's result identical to aligning it
    # alone (the reference's B=1); files too short for the encoder's 400-sample window are aligned alone.
    # One batch in flight: the host assembles batch i while the GPU runs batch i+1 (task.submit: encoder on the
    # main stream, head + Viterbi on a side stream).  A batch whose DP task.submit holds for the next encoder's
    # attention launches (long files) completes only under that encoder, so it stays pending one batch longer
    # (as in bench.py): waiting for it right after the next submit would idle the GPU.
    plan = plan_batches([(k, it[1], it[2]) for k, it in items.items()], batch_size, sr,
                        task.unitsEncoder.encoder_sample_rate)
    pending = []
    try:
        for bi, (file_sr, ks) in enumerate(plan):
            if bi + 1 < len(plan):
                nks = plan[bi + 1][1]
                prefetched[tuple(nks)] = loader.submit(load, [items[k] for k in nks])
            job, err = None, None
            try:
                job = run(ks, file_sr)
            except recoverable as e:
                err = e
            depth = 2 if job is not None and "resolve" in job[0] else 1
            while len(pending) >= depth:
                settle(pending.pop(0))
            if job is not None:
                pending.append(job)
            elif len(ks) == 1:
                errors.append([items[ks[0]][0], err])
            else:
                for k in ks:
                    alone(k, file_sr)
        while pending:
            settle(pending.pop(0))
    finally:
        loader.shutdown(wait=True, cancel_futures=True)
    if trace is not None:
        import json
        with open(os.environ["HFA_CLI_TRACE"], "a", encoding="utf-8") as f:
            f.write(json.dumps(trace) + "\n")
    return out


def _run(task, rows, keys, batch_size, errors, on_batch=None):
    """_predict with the rank-level outcome: (records, ok).  A failed shard leaves ``errors`` as it found it: its
    files are re-run elsewhere, so the entries it logged would be duplicates (or wrong, for files aligned there)."""
    n_err = len(errors)
    try:
        return _predict(task, rows, keys, batch_size, errors, on_batch), True
    except Exception as e:  # noqa: BLE001 — reported to the control plane; the shard is re-queued elsewhere
        import traceback
        del errors[n_err:]
        traceback.print_exc()
        print(f"[rank {os.environ.get('RANK', '0')}] shard failed: {e!r}", flush=True)
        return {}, False


def _write_metrics(path, records, sr, world, n_files, n_errors, phases):
    """One JSON line per run (SURVEY §5 'Metrics / logging'): aligned audio seconds per wall second of the
    alignment phase (WAV reads + GPU + boundaries; the streamed export too on one GPU) and of the whole run, DP and
    Hubert frames per second, phase times."""
    import json
    import time
    audio_s = sum(r["n44"] for r in records.values()) / sr
    dp_frames = sum(int(r["T"]) for r in records.values())
    total = sum(phases.values())
    line = dict(time=time.time(), files=n_files, aligned=len(records), errors=n_errors, world=world,
                audio_s=audio_s, dp_frames=dp_frames, hubert_frames=int(round(audio_s * 50)),
                rtf_inv_align=audio_s / phases["align"] if phases["align"] > 0 else None,
                rtf_inv_total=audio_s / total if total > 0 else None,
                dp_frames_per_s=dp_frames / phases["align"] if phases["align"] > 0 else None,
                phases_s=phases)
    with open(path, "a", encoding="utf-8") as f:
        f.write(json.dumps(line) + "\n")


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
@click.option("--dist_backend", default="nccl", type=str, help="multi-GPU data backend: nccl (= RCCL); gloo for rehearsals")
@click.option("--device", default=None, type=int, help="force every rank onto this GPU (multi-rank rehearsal on one GPU)")
@click.option("--metrics", default=None, type=str, help="append one JSON line of run metrics to this file (SURVEY §5)")
def main(ckpt, folder, g2p, save_confidence, hubert_path, batch_size, out_path, dist_backend, device, metrics,
         **kwargs):
    import torch
    import hubertfa_amd.g2p as g2p_mod
    from hubertfa_amd.alignment_decoder import utterance_result
    from hubertfa_amd.distributed import env_rank_world, gather_records, shard_lpt, utterance_cost
    from hubertfa_amd.export_tool import Exporter
    from hubertfa_amd.post_processing import post_processing
    from hubertfa_amd.task import ForcedAlignmentTask
    from hubertfa_amd.wav_io import wav_info

    import time
    t_start = time.perf_counter()
    if not g2p.endswith("G2P"):
        g2p += "G2P"
    grapheme_to_phoneme = getattr(g2p_mod, g2p)(**kwargs)
    grapheme_to_phoneme.set_in_format("lab")
    rows = list(grapheme_to_phoneme.get_dataset(sorted(pathlib.Path(folder).rglob("*.wav"))))
    t_g2p = time.perf_counter()

    rank, world, local = env_rank_world()
    local = local if device is None else device
    torch.cuda.set_device(local)
    dist, ctrl, mine, costs, shards = None, None, list(range(len(rows))), None, None
    if world > 1:
        import torch.distributed as dist
        if dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(dist_backend)
        ctrl = dist.new_group(backend="gloo")            # control plane: host memory, survives a lost GPU
        costs = []
        for r in rows:
            try:
                n, file_sr, _ = wav_info(r[0])
            except (OSError, ValueError):
                n, file_sr = 0, 44100
            costs.append(utterance_cost(n, len(r[1]), file_sr))
        shards = shard_lpt(costs, world)
        mine = shards[rank]

    torch.set_grad_enabled(False)
    model = ForcedAlignmentTask.load_from_checkpoint(ckpt, device=torch.device("cuda", local),
                                                     hubert_model_path=hubert_path)
    model.on_predict_start()                             # the units encoder's weights (reference: predict start)
    # the loaded program's objects (torch, the model, the dataset rows) leave the cyclic collector's scans: a full
    # collection over them inside the batch loop stalled the host for 60-90 ms (the GPU idle meanwhile), once per
    # 1 024-file run (HFA_CLI_TRACE, scripts/archive/gpu_r06x.sh); objects made from here on are collected as usual
    import gc
    gc.collect()
    gc.freeze()
    errors = []
    t_load = time.perf_counter()
    sr = model.melspec_config["sample_rate"]
    # one GPU: each batch is post-processed and its TextGrids written while the GPU runs the next batch
    stream = _StreamingExport(rows, sr, model.decoder.frame_length, out_path) if world == 1 else None
    records, ok = _run(model, [rows[i] for i in mine], mine, batch_size, errors, stream)
    t_align = time.perf_counter()
    if world == 1 and not ok:
        raise SystemExit(1)
    if world > 1:
        status = [None] * world
        dist.all_gather_object(status, ok, group=ctrl)
        failed = [r for r in range(world) if not status[r]]
        if failed:
            healthy = [r for r in range(world) if status[r]]
            if not healthy:
                raise SystemExit("every rank failed its shard")
            todo = sorted(i for r in failed for i in shards[r])
            parts = shard_lpt([costs[i] for i in todo], len(healthy))
            if rank in healthy:
                again = [todo[j] for j in parts[healthy.index(rank)]]
                print(f"[rank {rank}] re-running {len(again)} file(s) of failed rank(s) {failed}", flush=True)
                more, ok2 = _run(model, [rows[i] for i in again], again, batch_size, errors)
                if not ok2:
                    raise SystemExit(f"rank {rank} failed re-running a re-queued shard")
                records.update(more)
        # boundary arrays to every rank: RCCL when every GPU is healthy, else the gloo control group
        records = gather_records(records, group=None if not failed and dist_backend == "nccl" else ctrl)
        all_errors = [None] * world
        dist.all_gather_object(all_errors, [[str(p), repr(e)] for p, e in errors], group=ctrl)
        errors = [e for part in all_errors for e in part]
        if rank != 0:
            dist.destroy_process_group()
            gc.unfreeze()
            return

    if stream is not None:
        predictions, log = stream.results()
    else:
        predictions = []
        for i, (wav_path, ph_seq, word_seq, p2w) in enumerate(rows):
            if i in records:
                rec = records[i]
                r = utterance_result(rec, ph_seq, word_seq, p2w, model.decoder.frame_length)
                predictions.append((wav_path, rec["n44"] / sr, r["confidence"], r["ph_seq"], r["ph_intervals"],
                                    r["word_seq"], r["word_intervals"]))
        predictions, log = post_processing(predictions)
    exporter = Exporter(predictions, errors + log, out_path)
    out_formats = ["textgrid"] + (["confidence"] if save_confidence else [])
    exporter.export(out_formats, textgrids=stream is None)
    t_end = time.perf_counter()
    print("Output files are saved to the same folder as the input wav files.")
    what = "align + post-processing + TextGrids (streamed)" if stream is not None else "align"
    print(f"[timing] g2p {t_g2p - t_start:.2f} s, model load {t_load - t_g2p:.2f} s, wav read + {what} "
          f"{t_align - t_load:.2f} s ({len(records)} files), gather + post-processing + export {t_end - t_align:.2f} s")
    if metrics:
        _write_metrics(metrics, records, sr, world, len(rows), len(errors) + len(log),
                       dict(g2p=t_g2p - t_start, load=t_load - t_g2p, align=t_align - t_load, export=t_end - t_align))
    if world > 1:
        dist.destroy_process_group()
    gc.unfreeze()                                        # (an in-process caller's later runs see a normal collector)


if __name__ == "__main__":
    main()
