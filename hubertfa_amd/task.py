"""Inference surface of ``LitForcedAlignmentTask`` without Lightning (networks/task/forced_alignment.py).

Kept: ``load_from_checkpoint(path)`` (reads ``state_dict`` + ``hyper_parameters`` of a Lightning .ckpt),
``forward(x[B,T,C]) -> (ph_frame_logits, ph_edge_logits, ctc_logits)`` (:284-292), ``on_predict_start`` (:143-152),
``predict_step(batch, batch_idx)`` (:154-186) with the same 7-tuple result.  Training/validation/losses are out
of scope; loss-module buffers in the checkpoint are ignored.

Added: ``align_batch`` — B equal-length utterances through one pass of GPU kernels (resample, Hubert, gather,
UNet+head, lattice prologue, DP, backtrack), the path the benchmark and the batched CLI use.
"""
from __future__ import annotations


import numpy as np
import torch
import yaml

from . import ops, synth
from .alignment_decoder import AlignmentDecoder
from .encoder import UnitsEncoder
from .resample import ChainResampler, Resampler, target_length
from .hubert import dev_lengths
from .intervals import batch_tables
from .unet import LatticeHead
from .wav_io import read_wav


def guarded(module, flag, fn):
    """Run ``fn`` (one pass of ``module``'s kernels) under the split-f16 range guard, synchronously: clear
    ``flag``, run, and if a split producer raised it, clear it and run ``fn`` again with ``module.precision`` =
    "f32".  Used by the reference-surface entries that return tensors (forward, UnitsEncoder.encode); the
    pipelined path snapshots the flags on the device instead (ForcedAlignmentTask._guard)."""
    if getattr(module, "precision", "f32") != "split" or flag is None:
        return fn()
    flag.zero_()
    out = fn()
    if int(flag.item()):
        flag.zero_()
        module.precision = "f32"
        try:
            out = fn()
        finally:
            module.precision = "split"
    return out


class ForcedAlignmentTask:
    def __init__(self, vocab_text, vowel_text, model_config, hubert_config, melspec_config, optimizer_config=None,
                 loss_config=None, *, state_dict=None, device="cuda"):
        self.hparams = dict(vocab_text=vocab_text, vowel_text=vowel_text, model_config=model_config,
                            hubert_config=hubert_config, melspec_config=melspec_config,
                            optimizer_config=optimizer_config, loss_config=loss_config)
        self.device = torch.device(device)
        self.vocab = yaml.safe_load(vocab_text)
        self.vowel = yaml.safe_load(vowel_text) if vowel_text else None
        self.ignored_phones = self.vocab.get("ignored_phonemes", [])
        self.melspec_config = melspec_config
        self.hubert_config = hubert_config
        arch = synth.UNetArch(input_dims=hubert_config["channel"], hidden_dims=model_config["hidden_dims"],
                              output_dims=model_config["hidden_dims"],
                              factor=model_config["down_sampling_factor"], times=model_config["down_sampling_times"],
                              scaleup=model_config["channels_scaleup_factor"], vocab_size=self.vocab["vocab_size"])
        if state_dict is None:
            raise ValueError("state_dict (backbone.*, head.*) is required")
        sd = {k: v for k, v in state_dict.items() if k.startswith("backbone.") or k.startswith("head.")}
        self.head = LatticeHead(arch, sd, self.device)
        self.decoder = AlignmentDecoder(self.vocab, self.melspec_config)
        self.unitsEncoder = None
        self._upsamplers = {}
        self._chains = {}

    # -- checkpoint ---------------------------------------------------------------------------------------------
    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, device="cuda", hubert_model_path=None):
        ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        hp = dict(ckpt["hyper_parameters"])
        if hubert_model_path is not None:
            hp["hubert_config"] = dict(hp["hubert_config"], model_path=hubert_model_path)
        return cls(hp["vocab_text"], hp.get("vowel_text"), hp["model_config"], hp["hubert_config"],
                   hp["melspec_config"], hp.get("optimizer_config"), hp.get("loss_config"),
                   state_dict=ckpt["state_dict"], device=device)

    # -- reference surface --------------------------------------------------------------------------------------
    def on_predict_start(self):
        if self.unitsEncoder is None:
            hc = self.hubert_config
            self.unitsEncoder = UnitsEncoder(hc["encoder"], hc["model_path"], hc["sample_rate"], hc["hop_size"],
                                             self.device)

    @torch.no_grad()
    def forward(self, x):
        """x [B, T, C] -> (ph_frame_logits [B,T,V], ph_edge_logits [B,T], ctc_logits [B,T,V]).

        Range guard as on the batched path: if a split-f16 operand of the head left f16 range, the logits are
        recomputed on the f32 GEMMs (this entry returns tensors, so it checks the head's flag synchronously)."""
        x = x.to(self.device).float()
        T = x.shape[1]
        Tp = self.head.padded_len(T)
        if Tp != T:
            x = torch.nn.functional.pad(x, (0, 0, 0, Tp - T))
        x = x.contiguous()
        logits = guarded(self.head, self.head.flag, lambda: self.head.logits(x))[:, :T]
        return LatticeHead.split(logits)

    __call__ = forward

    def predict_step(self, batch, batch_idx=0):
        """forced_alignment.py:154-186.  load_wav's resample to the melspec rate (load_wav.py:6-7) runs inside
        align_batch (``wav_sr``), on the same kernels as the batched CLI, so one file gives identical results on
        both paths."""
        wav_path, ph_seq, word_seq, ph_idx_to_word_idx = batch
        sr = self.melspec_config["sample_rate"]
        x, file_sr = read_wav(str(wav_path))
        wave = self.upload(np.ascontiguousarray(x[:1]))                     # channel 0 (load_wav.py:8)
        wav_length = target_length(x.shape[1], file_sr, sr) / sr           # waveform.shape[0] / sample_rate
        res = self.align_batch(wave, [ph_seq], [word_seq], [ph_idx_to_word_idx], wav_sr=file_sr)[0]
        return (wav_path, wav_length, res["confidence"], res["ph_seq"], res["ph_intervals"], res["word_seq"],
                res["word_intervals"])

    # -- batched GPU path ---------------------------------------------------------------------------------------
    def upsampler(self, sr: int):
        target = self.melspec_config["sample_rate"]
        if sr not in self._upsamplers:
            self._upsamplers[sr] = Resampler(sr, target, 6, self.device)
        return self._upsamplers[sr]

    @torch.no_grad()
    def encode_batch(self, waves: torch.Tensor, wav_sr: int | None = None, lengths=None,
                     chunk_seconds: float | None = None, gate=None):
        """Device half 1 (current stream): waves [B, N] -> (features [B, T_pad, C], DP frames, wav lengths).

        ``lengths`` (optional host ints [B]): samples per row of a variable-length batch, rows zero-padded to N
        at ``wav_sr``; then DP frames is a per-row list and every row aligns exactly as it would alone.
        ``chunk_seconds`` (one long utterance): encode overlapping windows of that length as one batch
        (UnitsEncoder.units_chunked) — long-form speed at the cost of per-window attention context."""
        self.on_predict_start()
        sr = self.melspec_config["sample_rate"]
        hop = self.melspec_config["hop_length"]
        waves = waves.to(self.device).float()
        if lengths is not None and all(int(n) == waves.shape[-1] for n in lengths):
            lengths = None
        resampled = None
        if wav_sr is not None and wav_sr != sr:
            chain = self.chain_resampler(wav_sr, waves.shape[-1], lengths)
            if chain is not None:        # input rate -> sr -> encoder rate as one pass; the sr wave is never formed
                if waves.stride(-1) != 1:
                    waves = waves.contiguous()
                enc = chain(waves, dev_lengths(lengths, waves.device) if lengths is not None else None)
                resampled = (enc, target_length(waves.shape[-1], wav_sr, sr))
            else:
                up = self.upsampler(wav_sr)
                waves = up(waves, split=self.unitsEncoder.split_resample)
            if lengths is not None:
                lengths = [target_length(int(n), wav_sr, sr) for n in lengths]
                if chain is None:
                    waves = waves.contiguous()
                    ops.mask_rows(waves, dev_lengths(lengths, waves.device))   # sinc tails past each row's end
        n = waves.shape[-1] if resampled is None else resampled[1]
        chunk = None if chunk_seconds is None else max(1, int(round(chunk_seconds * 50)))
        feats, n_frames = self.unitsEncoder.encode_frames(waves if resampled is None else None, sr, hop,
                                                          pad_to=self.head.divisible, lengths=lengths,
                                                          chunk_frames=chunk, gate=gate, resampled=resampled)
        wl = [n / sr] * waves.shape[0] if lengths is None else [int(m) / sr for m in lengths]
        return feats, n_frames, wl

    # the input rate -> melspec rate -> encoder rate chain as one pass (resample.ChainResampler) when the input is
    # at the encoder rate (16 kHz files) and the encoder runs split; False: always the two stages
    chain_resample = True

    def chain_resampler(self, wav_sr: int, n: int, lengths=None):
        """The one-pass ChainResampler for a batch at ``wav_sr``, or None where the two stages must run: another
        input rate, the f32 re-run of the range guard, or a row whose encoder-rate length is under the 400 samples
        where the reference pads the melspec-rate wave (encoder.py:51-52)."""
        ue = self.unitsEncoder
        if not self.chain_resample or not ue.split_resample or int(wav_sr) != int(ue.encoder_sample_rate):
            return None
        key = int(wav_sr)
        if key not in self._chains:
            try:
                self._chains[key] = ChainResampler(wav_sr, self.melspec_config["sample_rate"], 6, 128, self.device)
            except ValueError:
                self._chains[key] = None
        chain = self._chains[key]
        if chain is None or chain.out_length(min(int(m) for m in lengths) if lengths is not None else n) < 400:
            return None
        return chain

    def head_logits(self, feats, n_frames):
        """UNet head (current stream): features -> (logits [B, T, V+2], the head's range-flag snapshot or None)."""
        if isinstance(n_frames, (list, tuple)):          # variable-length batch
            t_pad = [self.head.padded_len(int(t)) for t in n_frames]
            logits = self.head.logits(feats, t_pad)[:, :max(n_frames)]
        else:
            logits = self.head.logits(feats)[:, :n_frames]
        flag = None
        if self.head.precision == "split":      # the head's own range flag, snapshot on the stream that ran it
            flag = ops.flag_take(self.head.flag)
        return logits, flag

    def lattice_dp(self, logits, flag, wav_lengths, ph_seqs, word_seqs=None, p2ws=None, dp_ranges=None):
        """Lattice prologue + Viterbi + backtrack (current stream) -> the decoder's device outputs (with
        ``dp_ranges``, possibly the DP left as deferred steps: AlignmentDecoder.decode_batch)."""
        frame, edge = logits[:, :, 2:], logits[:, :, 0]      # LatticeHead.split without the unused ctc logits
        dev_out = self.decoder.decode_batch(frame, edge, wav_lengths, ph_seqs, word_seqs, p2ws, host=False,
                                            dp_ranges=dp_ranges)
        if flag is not None:
            dev_out["split_oflow_head"] = flag
        return dev_out

    def decode_device(self, feats, n_frames, wav_lengths, ph_seqs, word_seqs=None, p2ws=None, dp_ranges=None):
        """Device half 2 (current stream): UNet head + lattice + Viterbi -> the decoder's device outputs."""
        logits, flag = self.head_logits(feats, n_frames)
        return self.lattice_dp(logits, flag, wav_lengths, ph_seqs, word_seqs, p2ws, dp_ranges)

    def _guard(self, dev_out, redo_args):
        """Split-precision range guard: snapshot (and clear) the split-f16 overflow flag the batch's producers
        raise (ops.split_flag) into the batch's outputs, and attach a re-run of the batch on the f32 GEMMs that
        ``decoder.assemble`` takes instead when the flag is set."""
        enc = getattr(self.unitsEncoder, "model", None)
        enc_split = getattr(enc, "precision", "f32") == "split"
        if not enc_split and self.head.precision != "split":
            return dev_out
        if enc_split:
            dev_out["split_oflow"] = ops.flag_take(ops.split_flag(self.device))
        dev_out["redo"] = lambda: self._align_f32(*redo_args)
        return dev_out

    def _align_f32(self, waves, ph_seqs, word_seqs, p2ws, wav_sr, lengths, chunk_seconds):
        enc = self.unitsEncoder.model
        saved = (getattr(enc, "precision", "f32"), self.head.precision)
        if hasattr(enc, "precision"):
            enc.precision = "f32"
        self.head.precision = "f32"
        try:
            return self.align_batch(waves, ph_seqs, word_seqs, p2ws, wav_sr=wav_sr, lengths=lengths,
                                    chunk_seconds=chunk_seconds)
        finally:
            if hasattr(enc, "precision"):
                enc.precision = saved[0]
            self.head.precision = saved[1]

    def align_batch(self, waves: torch.Tensor, ph_seqs, word_seqs=None, p2ws=None, wav_sr: int | None = None,
                    host: bool = True, lengths=None, chunk_seconds: float | None = None):
        """B waveforms [B, N] (at melspec sample_rate, or ``wav_sr`` to resample first, like load_wav) ->
        list of decode results (dicts with ph_seq / ph_intervals / word_seq / word_intervals / confidence / raw
        path).  Rows of different lengths: zero-pad to N and pass ``lengths``."""
        feats, n_frames, wl = self.encode_batch(waves, wav_sr, lengths, chunk_seconds)
        dev_out = self.decode_device(feats, n_frames, wl, ph_seqs, word_seqs, p2ws)
        dev_out = self._guard(dev_out, (waves, ph_seqs, word_seqs, p2ws, wav_sr, lengths, chunk_seconds))
        if not host:
            return dev_out
        return self.decoder.assemble(dev_out, ph_seqs, word_seqs, p2ws)

    def upload(self, waves) -> torch.Tensor:
        """Host waves (numpy or CPU tensor [B, N]; pinned f32 avoids a staging copy) -> f32 device tensor: a pinned
        non-blocking H2D on the caller's current stream (no host sync).  A dedicated copy stream, which would let
        the copy run under the previous batch's encoder, measured slower on MI355X."""
        if isinstance(waves, torch.Tensor) and waves.is_cuda:
            return waves.to(self.device, torch.float32)
        x = torch.as_tensor(waves, dtype=torch.float32)
        pinned = x if x.is_pinned() else x.contiguous().pin_memory()
        return pinned.to(self.device, non_blocking=True)   # (the pinned block is held until this copy ends)

    def submit(self, waves: torch.Tensor, ph_seqs, word_seqs=None, p2ws=None, wav_sr: int | None = None,
               on_device=None, lengths=None, chunk_seconds: float | None = None):
        """Two-stream pipelined device pass; returns the decoder's fetch handle (``decoder.assemble`` completes it).

        The encoder runs on the caller's current stream and the head + lattice + Viterbi on a side stream that
        waits for it, so a batch's small-grid tail (UNet GEMMs on a few hundred workgroups, one DP workgroup per
        utterance) overlaps the next batch's extractor instead of idling most of the chip.  (Enqueuing the side
        pass in steps at the next encoder's FFN2 launches, whose one round of tiles leaves CUs idle, measured 13 %
        slower: the steps spill into the full-chip kernels that follow)  A long lattice
        (``defer_dp_frames``) is the exception: its forward DP holds one CU for milliseconds, and every one-round
        GEMM grid it overlaps waits for the tile that CU could not start, so its DP is held back and run in step
        ranges, one right before each attention launch of the NEXT batch's encoder (multi-round grids), the rest
        when the next encoder has been enqueued or when the handle is assembled (config 5: the DP's cost to the
        encoder 2.4 -> 0.5 ms, profiles/r04/dp_gate_ab.txt).  ``on_device`` (e.g. the RCCL boundary gather) runs
        on the side stream after the backtrack."""
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        held, self._held = getattr(self, "_held", None), None
        feats, n_frames, wl = self.encode_batch(waves, wav_sr, lengths, chunk_seconds,
                                                gate=held.gate(main) if held is not None else None)
        if held is not None:
            held.drain()        # a failure there belongs to the held batch: its handle's resolve() re-raises it
        guard = self._guard({}, (waves, ph_seqs, word_seqs, p2ws, wav_sr, lengths, chunk_seconds))
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            feats.record_stream(self._side)      # the caching allocator must not recycle it under the side stream
            with ops.grid_cap(self.side_grid_cap):
                dev_out = self.decode_device(feats, n_frames, wl, ph_seqs, word_seqs, p2ws,
                                             dp_ranges=self.dp_ranges if chunk_seconds is None else None)
            if "split_oflow" in guard:
                guard["split_oflow"].record_stream(self._side)
            dev_out.update(guard)
            work = _HeldDP(self, dev_out, on_device)
            if work.steps:
                self._held = work
            else:
                work.complete()
        if self.host_tables:         # the host assembly's transcript tables, built while the GPU runs this batch
            work.handle["tables"] = batch_tables(ph_seqs, word_seqs, p2ws)
        return work.handle

    # submit builds the batch's transcript tables for decoder.assemble's batch_results (False: a caller that takes
    # raw records, assemble(intervals=False), as the CLI's export workers do)
    host_tables = True

    # workgroups at most per launch of the side pass's row-streaming kernels (ops.grid_cap; 0: uncapped): beside the
    # next batch's encoder, their one-row workgroups cost the encoder more than their work
    side_grid_cap = 512

    # a lattice of at least this many DP frames (config 5's 300 s: 25 839) runs its forward DP beside the next
    # batch's attention launches, one step range per encoder layer; None: never.  A range must fit in one
    # attention launch: the DP's steps grow with the wave's length L, the attention's time with L^2, and at
    # 16 384 frames (~190 s) a twelfth of the DP (~0.7 ms) is about one unchunked attention launch.  Windowed
    # long-form (chunk_seconds) never holds: its attention launches are far shorter (profiles/r04/held_dp_ab.txt)
    defer_dp_frames = 16384

    def dp_ranges(self, Tmax: int, Smax: int) -> int:
        """How many step ranges submit() cuts a batch's forward DP into (1: one launch, now)."""
        n_layers = len(getattr(self.unitsEncoder.model, "layers", ()))
        if self.defer_dp_frames is None or Tmax < self.defer_dp_frames or n_layers < 2:
            return 1
        return n_layers

    def flush(self):
        """Enqueue a held batch's remaining DP steps now (the pipeline's last batch; assemble also does this).  An
        error in them stays with that batch: its handle's resolve() (decoder.assemble) raises it."""
        held, self._held = getattr(self, "_held", None), None
        if held is not None:
            held.drain()


class _HeldDP:
    """A batch's deferred forward-DP ranges + backtrack (AlignmentDecoder.decode_batch ``deferred``) and the
    completion after them: ``on_device``, then the D2H fetch whose handle ``submit`` returned early (its "resolve"
    entry, which ``decoder.assemble`` calls, runs whatever is still held).

    Failures stay with this batch: a step is dropped only after it ran, the first error stops the rest
    (a DP missing a time range must never reach the backtrack) and is kept, and ``resolve`` -- this batch's
    assemble -- raises it (on every call); the next batch's encoder, whose attention launches gate the steps, never
    sees it.  Exception: in a multi-rank run whose ``on_device`` is a collective, the error is raised at once
    (ADVICE r05): the peers would otherwise wait in the gather this rank never reaches."""

    def __init__(self, task, dev_out, on_device):
        self.task, self.dev_out, self.on_device = task, dev_out, on_device
        self.steps = dev_out.pop("deferred", [])
        self.error = None
        self.handle = {"resolve": self.flush}

    def complete(self):
        """(side stream) the batch's outputs are enqueued: run on_device and the fetch; fill the handle."""
        if self.on_device is not None:
            self.on_device(self.dev_out)
        h = self.task.decoder.fetch(self.dev_out)
        self.handle.pop("resolve", None)
        self.handle.update(h)

    def _next(self):
        if self.error is not None or not self.steps:
            return
        try:
            self.steps[0]()
            self.steps.pop(0)
            if not self.steps:
                self.complete()
        except Exception as e:  # noqa: BLE001 — kept for this batch's resolve(); see the class note
            self.error = e
            self.steps = []
            if getattr(self.task, "_held", None) is self:
                self.task._held = None
            if self.on_device is not None and _dist_world() > 1:
                # on_device is this batch's collective (the boundary gather): deferring the error would leave the
                # peer ranks blocked in it until the process-group timeout and hide the cause.  Raise now, so this
                # rank exits and the launcher (torch.distributed.run) tears the job down with this error in its log
                raise

    def gate(self, main):
        """The next encoder's attention gate: the side stream waits for the main stream to reach the launch, then
        takes the next step."""
        side = self.task._side

        def g():
            if self.steps and self.error is None:
                ev = torch.cuda.Event()
                ev.record(main)
                with torch.cuda.stream(side):
                    side.wait_event(ev)
                    self._next()
        return g

    def drain(self):
        """Enqueue every remaining step (on the side stream); errors are kept, not raised."""
        with torch.cuda.stream(self.task._side):
            while self.steps and self.error is None:
                self._next()
        if getattr(self.task, "_held", None) is self:
            self.task._held = None

    def flush(self):
        """The handle's resolve(): drain, then raise this batch's error if one of its steps failed."""
        self.drain()
        if self.error is not None:
            raise self.error


def _dist_world() -> int:
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def synth_checkpoint(path: str | None = None, *, encoder="cnhubert", model_path="synth:0", seed=1,
                     n_phones: int = 62) -> dict:
    """A Lightning-layout checkpoint dict with seeded weights (optionally saved to ``path``)."""
    vocab = synth.synth_vocab(n_phones)
    channel = 256 if encoder == "hubertsoft" else (1024 if encoder == "cnhubert-large" else 768)
    ua = synth.UNetArch(input_dims=channel, vocab_size=vocab["vocab_size"])
    sd = {k: torch.from_numpy(v) for k, v in synth.synth_unet_state_dict(ua, seed=seed).items()}
    hp = {
        "vocab_text": yaml.safe_dump(vocab),
        "vowel_text": yaml.safe_dump({"vowel": []}),
        "model_config": {"hidden_dims": ua.hidden_dims, "down_sampling_factor": ua.factor,
                         "down_sampling_times": ua.times, "channels_scaleup_factor": ua.scaleup},
        "hubert_config": {"encoder": encoder, "model_path": model_path, "sample_rate": 16000, "hop_size": 320,
                          "channel": channel},
        "melspec_config": {"n_mels": 128, "sample_rate": 44100, "win_length": 1024, "hop_length": 512,
                           "n_fft": 2048, "fmin": 40, "fmax": 16000, "clamp": 0.00001},
        "optimizer_config": {}, "loss_config": {},
    }
    ckpt = {"state_dict": sd, "hyper_parameters": hp}
    if path is not None:
        torch.save(ckpt, path)
    return ckpt
