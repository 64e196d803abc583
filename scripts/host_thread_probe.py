"""Which host thread burns CPU in the pipelined config-2 step, and what it is doing (GPU box, verdict r05 item 4).

One process per run; ``--device-flags`` sets the HIP device schedule (hipSetDeviceFlags on torch's own
libamdhip64.so.7, before anything initialises the device): default | spin | yield | blocking.  Over ``--steps``
pipelined steps (bench.py's loop: task.submit + assemble one batch behind) a sampler thread reads every thread's
/proc/self/task/<tid>/{stat,syscall,wchan} at ~500 Hz.  Prints one JSON line: ms per step, and per thread the CPU ms
per step, the share of samples in state R (on a CPU: a user-space spin when the syscall file says "running"), the
most frequent syscalls (number -> share) and kernel wait channels.

    python scripts/host_thread_probe.py --device-flags default
"""
import argparse
import collections
import ctypes
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FLAGS = {"default": None, "spin": 1, "yield": 2, "blocking": 4}
SYSCALLS = {0: "read", 1: "write", 7: "poll", 16: "ioctl", 23: "select", 24: "sched_yield", 35: "nanosleep",
            202: "futex", 230: "clock_nanosleep", 232: "epoll_wait", 270: "pselect6", 271: "ppoll", 281: "epoll_pwait"}


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


def _maps():
    """[(lo, hi, perms, offset, path)] of this process's mappings."""
    out = []
    for ln in _read(f"/proc/{os.getpid()}/maps").splitlines():
        f = ln.split(None, 5)
        lo, hi = (int(x, 16) for x in f[0].split("-"))
        out.append((lo, hi, f[1], int(f[2], 16), f[5] if len(f) > 5 else ""))
    return out


def stack_scan(sp, pc, maps, depth=32768):
    """Poor man's backtrace of a thread parked in a syscall (no ptrace, no gdb on the box): the syscall's user pc,
    then every 8-byte word in [sp, sp + depth) of the thread's own stack mapping that points into an executable
    file mapping of this process, as (library, file offset) -- return addresses, plus some stale words."""
    import ctypes
    out = []

    def where(a):
        for lo, hi, perms, off, path in maps:
            if lo <= a < hi and "x" in perms and path.startswith("/"):
                return os.path.basename(path), a - lo + off
        return None
    w = where(pc)
    if w:
        out.append(w)
    top = next((hi for lo, hi, perms, _o, _p in maps if lo <= sp < hi), None)
    if top is None:
        return out
    n = min(depth, top - sp) // 8
    raw = ctypes.string_at(sp, n * 8)
    for i in range(n):
        a = int.from_bytes(raw[8 * i:8 * i + 8], "little")
        w = where(a)
        if w:
            out.append(w)
    return out


def symbolize(frames):
    """(library, offset) -> 'library!symbol+0x..' from the library's dynamic and static symbol tables (nm)."""
    import bisect
    import subprocess
    tables = {}
    libs = {}
    for lo, hi, perms, off, path in _maps():
        if path.startswith("/"):
            libs.setdefault(os.path.basename(path), path)
    res = []
    for lib, off in frames:
        if lib not in tables:
            syms = []
            for extra in (["-D"], []):
                try:
                    txt = subprocess.run(["nm", "-C", "--defined-only", *extra, libs[lib]], capture_output=True,
                                         text=True, timeout=60).stdout
                except Exception:  # noqa: BLE001
                    txt = ""
                for ln in txt.splitlines():
                    f = ln.split(" ", 2)
                    if len(f) == 3 and f[1] in "tTwW":
                        syms.append((int(f[0], 16), f[2]))
            syms.sort()
            tables[lib] = ([a for a, _ in syms], [n for _, n in syms])
        addrs, names = tables[lib]
        i = bisect.bisect_right(addrs, off) - 1
        res.append(f"{lib}!{names[i][:90]}+{off - addrs[i]:#x}" if i >= 0 else f"{lib}+{off:#x}")
    return res


class Sampler(threading.Thread):
    def __init__(self, period=0.002):
        super().__init__(daemon=True)
        self.period, self.stop, self.me = period, threading.Event(), None
        self.state = collections.defaultdict(collections.Counter)
        self.sysc = collections.defaultdict(collections.Counter)
        self.wchan = collections.defaultdict(collections.Counter)
        self.n = 0
        self.stacks = collections.defaultdict(list)      # tid -> [(sp, pc, frames)] of samples parked in a syscall
        self.maps = _maps()

    def run(self):
        self.me = threading.get_native_id()
        base = f"/proc/{os.getpid()}/task"
        while not self.stop.is_set():
            for t in os.listdir(base):
                tid = int(t)
                if tid == self.me:
                    continue
                st = _read(f"{base}/{t}/stat")
                if not st:
                    continue
                s = st[st.rindex(")") + 2]
                self.state[tid][s] += 1
                sc = _read(f"{base}/{t}/syscall").split()
                key = "running" if sc[:1] == ["running"] else (SYSCALLS.get(int(sc[0]), sc[0]) if sc and sc[0].lstrip("-").isdigit() else "?")
                self.sysc[tid][key] += 1
                if key not in ("running", "?") and len(sc) >= 3 and len(self.stacks[tid]) < 6:
                    try:
                        sp, pc = int(sc[-2], 16), int(sc[-1], 16)
                        self.stacks[tid].append(stack_scan(sp, pc, self.maps))
                    except Exception:  # noqa: BLE001 — a diagnostic: a torn read just drops the sample
                        pass
                w = _read(f"{base}/{t}/wchan").strip() or "0"
                self.wchan[tid][w] += 1
            self.n += 1
            time.sleep(self.period)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device-flags", default="default", choices=sorted(FLAGS))
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--env", action="append", default=[], help="K=V set before the HIP runtime starts")
    a = ap.parse_args()
    for kv in a.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    import torch
    if FLAGS[a.device_flags] is not None:
        hip = ctypes.CDLL("libamdhip64.so.7")          # the runtime torch loaded (same soname: one instance)
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(FLAGS[a.device_flags]))
        assert rc == 0, f"hipSetDeviceFlags rc={rc}"
    import bench
    from hubertfa_amd.task import ForcedAlignmentTask, synth_checkpoint
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    ck = synth_checkpoint(model_path="synth:0", seed=1)
    task = ForcedAlignmentTask(**ck["hyper_parameters"], state_dict=ck["state_dict"], device=d)
    task.on_predict_start()
    wav_np, ph, ws, pw = bench.make_inputs(32, 10.0, 30, seed0=1000)
    wav = torch.from_numpy(wav_np).to(d)

    def steps(k):
        pending = None
        for _ in range(k):
            h = task.submit(wav, ph, ws, pw, wav_sr=16000)
            if pending is not None:
                task.decoder.assemble(pending, ph, ws, pw)
            pending = h
        task.decoder.assemble(pending, ph, ws, pw)
        torch.cuda.synchronize()
    steps(5)
    # timing and per-thread CPU without the sampler (its reads would share the GIL with the launching thread) ...
    a0, t0 = bench.thread_cpu(), time.perf_counter()
    steps(a.steps)
    el = time.perf_counter() - t0
    a1 = bench.thread_cpu()
    # ... then the same steps again under the sampler, for the threads' states
    smp = Sampler()
    smp.start()
    time.sleep(0.05)
    steps(a.steps)
    smp.stop.set()
    smp.join()
    main_id = threading.get_native_id()
    rows = []
    for tid, (name, c1) in a1.items():
        ms = 1e3 * (c1 - a0.get(tid, (name, 0.0))[1]) / a.steps
        if ms <= 0.05 or tid == smp.me:
            continue
        tot = sum(smp.state[tid].values()) or 1
        st = _read(f"/proc/{os.getpid()}/task/{tid}/status")
        vcs = next((int(ln.split()[1]) for ln in st.splitlines() if ln.startswith("voluntary_ctxt_switches")), None)
        rows.append({"tid": tid, "name": "main" if tid == main_id else name, "cpu_ms_per_step": round(ms, 2),
                     "voluntary_ctxt_switches_total": vcs,
                     "share_R": round(smp.state[tid]["R"] / tot, 3),
                     "syscalls": {k: round(v / tot, 3) for k, v in smp.sysc[tid].most_common(4)},
                     "wchan": {k: round(v / tot, 3) for k, v in smp.wchan[tid].most_common(3)}})
    rows.sort(key=lambda r: -r["cpu_ms_per_step"])
    for r in rows[:3]:              # the busiest threads' parked stacks, deduplicated frames in first-seen order
        seen, frames = set(), []
        for fr in smp.stacks.get(r["tid"], []):
            for f in fr[:40]:
                if f not in seen:
                    seen.add(f)
                    frames.append(f)
        r["stack_frames"] = symbolize(frames[:40])
    print(json.dumps({"device_flags": a.device_flags, "env": a.env, "steps": a.steps, "ms_per_step": 1e3 * el / a.steps,
                      "process_cpu_ms_per_step": sum(r["cpu_ms_per_step"] for r in rows), "samples": smp.n,
                      "threads": rows[:8], "n_threads": len(a1)}), flush=True)


if __name__ == "__main__":
    main()
