"""Which HIP operation keeps the HSA runtime's async-events thread spinning (verdict r05 item 4; scripts/
host_thread_probe.py names the thread).  Each pattern runs for ~2 s while a stream of small kernels keeps the GPU
busy; reported: CPU ms per second of every non-main thread (the busiest one is the HSA thread) and of the main thread.

    python scripts/host_thread_micro.py
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", action="append", default=[], help="K=V set before the HIP runtime starts")
    ap.add_argument("--only", default=None, help="comma-separated pattern names")
    a = ap.parse_args()
    for kv in a.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    import ctypes
    import torch
    import bench
    d = torch.device("cuda", 0)
    torch.cuda.set_device(d)
    x = torch.randn(1 << 20, device=d)
    side = torch.cuda.Stream()
    pin = torch.empty(1 << 12, dtype=torch.float32).pin_memory()
    hsrc = torch.randn(1 << 12).pin_memory()
    main_id = threading.get_native_id()

    def busy(k=1):              # ~10-20 us of GPU work per call
        for _ in range(k):
            x.mul_(1.0000001)

    def p_idle():
        time.sleep(0.002)

    def p_kernels():
        busy(4)

    def p_event():
        busy(4)
        e = torch.cuda.Event()
        e.record()

    def p_event_query():
        busy(4)
        e = torch.cuda.Event()
        e.record()
        e.query()

    def p_wait_event():
        busy(4)
        e = torch.cuda.Event()
        e.record()
        side.wait_event(e)
        with torch.cuda.stream(side):
            x[:16].add_(0)

    def p_d2h_pinned():
        busy(4)
        pin.copy_(x[:1 << 12], non_blocking=True)

    def p_h2d_pinned():
        busy(4)
        x[:1 << 12].copy_(hsrc, non_blocking=True)

    def p_pin_alloc_h2d():       # decode_batch's meta upload: a fresh pinned tensor per call (caching host allocator)
        busy(4)
        m = torch.arange(300, dtype=torch.int32).pin_memory()
        x[:300].copy_(m, non_blocking=True)

    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint,
                                         ctypes.c_uint32]
    hip.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint]
    flag = torch.zeros(1, dtype=torch.int32, device=d)
    cnt = [0]

    def p_wait_value():          # the same cross-stream dependency through a device word (stream memory operations)
        busy(4)
        cnt[0] += 1
        rc = hip.hipStreamWriteValue32(torch.cuda.current_stream().cuda_stream, flag.data_ptr(), cnt[0], 0)
        rc |= hip.hipStreamWaitValue32(side.cuda_stream, flag.data_ptr(), cnt[0], 0, 0xFFFFFFFF)   # >=
        assert rc == 0, rc
        with torch.cuda.stream(side):
            x[:16].add_(0)

    pats = {"idle": p_idle, "wait_value32": p_wait_value, "kernels": p_kernels, "event_record": p_event, "event_record_query": p_event_query,
            "side_wait_event": p_wait_event, "d2h_pinned": p_d2h_pinned, "h2d_pinned": p_h2d_pinned,
            "pin_alloc_h2d": p_pin_alloc_h2d}
    if a.only:
        pats = {k: v for k, v in pats.items() if k in a.only.split(",")}
    out = {"env": a.env}
    for name, fn in pats.items():
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        a0, t0, n = bench.thread_cpu(), time.perf_counter(), 0
        while time.perf_counter() - t0 < 2.0:
            fn()
            n += 1
            if n % 64 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        a1 = bench.thread_cpu()
        rows = []
        for tid, (nm, c1) in a1.items():
            ms = 1e3 * (c1 - a0.get(tid, (nm, 0.0))[1]) / el
            if ms > 1:
                rows.append(("main" if tid == main_id else f"{nm}:{tid}", round(ms, 1)))
        rows.sort(key=lambda r: -r[1])
        out[name] = {"ops_per_s": n / el, "thread_cpu_ms_per_s": rows[:4]}
        print(name, json.dumps(out[name]), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
