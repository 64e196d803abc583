"""Host worker processes for the CLI's streamed export (infer.py, one GPU).

Interval assembly, post-processing (reference: tools/post_processing.py) and TextGrid writing
(tools/export_tool.py) are pure-Python work of ~0.7 ms per file.  On the main thread they made the CLI
host-bound: a 32-file batch's host work outlasted its ~17 ms on the GPU.  They run here in a small pool of
spawned processes instead, while the main thread only decodes WAVs, enqueues batches and fetches the boundary
arrays.  Workers import only the host modules (no torch, no GPU), and the pool is started before the caller
touches the GPU.  The files and results are the same as the inline path's
(tests/test_host.py::test_streaming_export_matches_batch_export runs both).
"""
from __future__ import annotations


def assemble_post_write(out_path, sr, frame_length, items):
    """[(dataset index, raw boundary record, (wav_path, ph_seq, word_seq, ph_idx_to_word_idx))] ->
    [(index, post-processed prediction or None, error-log entry or None)]: interval/word assembly
    (``intervals.utterance_result``), post-processing, and each successful prediction's TextGrid
    (``Exporter.write_textgrid``) -- the inline streamed export's steps, in a worker process."""
    from .export_tool import Exporter
    from .intervals import utterance_result
    from .post_processing import post_process_one
    writer = Exporter([], [], out_path)
    made = set()
    out = []
    for i, rec, (wav_path, ph_seq, word_seq, p2w) in items:
        r = utterance_result(rec, ph_seq, word_seq, p2w, frame_length)
        p, err = post_process_one((wav_path, rec["n44"] / sr, r["confidence"], r["ph_seq"], r["ph_intervals"],
                                   r["word_seq"], r["word_intervals"]))
        if err is None:
            writer.write_textgrid(p, made)
        out.append((i, p, err))
    return out


def start_pool(n_workers: int):
    """A spawn-context process pool whose workers are already started: Python 3.10 launches every worker on the
    first submit, and a spawned worker is a fresh interpreter (fork + exec at launch, nothing inherited from the
    caller's GPU context).  Not waited on: the workers import their modules while the caller loads the model.
    None when processes cannot be started here (the caller then exports inline)."""
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    try:
        pool = ProcessPoolExecutor(max_workers=n_workers, mp_context=multiprocessing.get_context("spawn"))
        pool.submit(int)
        return pool
    except Exception:  # noqa: BLE001 — no worker processes (restricted host): the inline path is used
        return None
