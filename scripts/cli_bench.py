"""End-to-end CLI throughput (GPU box): N synthetic 16-bit WAV + .lab pairs (8-12 s), infer.py over the folder
in-process, phase times (G2P + WAV reads, GPU pass, post-processing + TextGrid export) and audio s per wall s.
python scripts/cli_bench.py [--n 512] [--batch 32]"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--profile", action="store_true", help="cProfile the second run (host time by function)")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--seconds", type=float, nargs=2, default=(8.0, 12.0), help="utterance length range (s)")
    ap.add_argument("--metrics", default=None, help="infer.py --metrics: append each run's JSON line to this file")
    args = ap.parse_args()
    import numpy as np
    from click.testing import CliRunner
    import infer
    from hubertfa_amd import synth
    from hubertfa_amd.task import synth_checkpoint
    from hubertfa_amd.wav_io import write_wav
    with tempfile.TemporaryDirectory() as td:
        d = synth.synth_dictionary(n_words=200)
        dpath = os.path.join(td, "dict.txt")
        with open(dpath, "w") as f:
            f.write("".join(f"{w}\t{' '.join(p)}\n" for w, p in d.items()))
        seg = os.path.join(td, "segments")
        os.makedirs(seg)
        rng = np.random.default_rng(0)
        secs = rng.uniform(args.seconds[0], args.seconds[1], args.n)
        base = synth.synth_audio(int(args.seconds[1] * 16000), seed=1)
        for i, s in enumerate(secs):
            write_wav(os.path.join(seg, f"u{i:05d}.wav"), base[: int(s * 16000)], 16000)
            with open(os.path.join(seg, f"u{i:05d}.lab"), "w") as f:
                f.write(synth.synth_lab(int(3 * s), d, seed=i))
        ck = os.path.join(td, "m.ckpt")
        synth_checkpoint(ck)
        argv0 = ["-c", ck, "-f", seg, "-d", dpath, "-sc", "--hubert_path", "synth:0", "--batch_size", str(args.batch)]
        if args.metrics:
            argv0 += ["--metrics", os.path.abspath(args.metrics)]
        for rep in range(args.reps):              # the first run also pays kernel loading and warm-up
            argv = argv0
            prof = None
            if args.profile and rep == 1:
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            t0 = time.perf_counter()
            r = CliRunner().invoke(infer.main, argv)
            el = time.perf_counter() - t0
            if prof is not None:
                import pstats
                prof.disable()
                pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(25)
                pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(40)
            if r.exit_code != 0:
                print(r.output[-2000:], repr(r.exception))
                raise SystemExit(1)
            timing = [ln for ln in r.output.splitlines() if ln.startswith("[timing]")]
            print(f"run {rep}: {args.n} files, {secs.sum():.0f} s of audio in {el:.2f} s wall -> "
                  f"{secs.sum() / el:.0f} x realtime; " + "; ".join(timing), flush=True)


if __name__ == "__main__":
    main()
