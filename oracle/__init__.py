"""TEST INFRASTRUCTURE ONLY — CPU restatements of the reference hot path, used as the parity checker.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this package.
The product (``hubertfa_amd``) never imports it and fails loudly when its HIP library is missing.

Contents
  * ``viterbi_oracle.c`` (+ ``Makefile`` -> ``_build/liboracle.so``): AlignmentDecoder.forward_pass + backtrack
    (tools/alignment_decoder.py:170-230, 263-288).  Pinned bit-exact against tests/golden/dp_cases.npz.
  * ``decode.py``: numpy restatement of AlignmentDecoder.decode/_decode (tools/alignment_decoder.py:26-143,
    232-294).  Pinned against tests/golden/decode_cases.{npz,json}.
  * ``hubert_cpu.py``: torch-CPU fp32 restatement of the Hubert encoders, UNet backbone and head
    (networks/hubert/model.py, transformers HubertModel, networks/layer/*).  Pinned against
    tests/golden/hubert_*.npz and unet_head.npz.
  * ``resample.py``: torchaudio sinc resampler restatement (tools/load_wav.py:7, tools/encoder.py:46-48).
    torchaudio is absent here: parity UNPINNED (no reference output exists for it in this container).
"""
