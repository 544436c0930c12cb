"""Host CPU cost of the HIP stream-ordering operations the ZeRO-3 runtime issues per gather /
reduce-scatter bucket (event record on the compute stream, the side stream's wait, event record on
the side stream, the compute stream's wait), per thread — main thread vs the HIP / HSA runtime's
own threads (named from /proc/self/task/<tid>/comm).  Diagnostic for VERDICT r3 next #4: the
simulated ws=8 C5 iteration spends ~6 ms per iteration of CPU on a runtime thread.

Usage: python tools/hip_event_cost.py [--n 2000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))


def thread_names():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            out[int(tid)] = Path(f"/proc/self/task/{tid}/comm").read_text().strip()
        except OSError:
            pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    args = ap.parse_args()

    import psutil
    import torch

    from zero_amd import _lib

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    s1 = torch.cuda.current_stream(dev)
    s2 = torch.cuda.Stream(device=dev)
    proc = psutil.Process()
    main_tid = threading.get_native_id()
    ev = [torch.cuda.Event() for _ in range(4)]
    for e in ev:
        e.record(s1)
    evt = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in evt:
        e.record(s1)
    x = torch.zeros(16, device=dev)
    torch.cuda.synchronize()

    def snap():
        return {t.id: t.user_time + t.system_time for t in proc.threads()}

    cases = {
        "record (no timing)": lambda: ev[0].record(s1),
        "record (timing)": lambda: evt[0].record(s1),
        "record + cross-stream wait": lambda: (ev[0].record(s1), s2.wait_event(ev[0])),
        "zs_stream_wait_event only": lambda: _lib.lib.zs_stream_wait_event(s2.cuda_stream, ev[1].cuda_event),
        "ordered pattern (4 ops)": lambda: (ev[0].record(s1), s2.wait_event(ev[0]), ev[1].record(s2),
                                            s1.wait_event(ev[1])),
        "small kernel launch": lambda: x.add_(1.0),
    }
    rows = []
    for name, fn in cases.items():
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        s0, w0 = snap(), time.perf_counter()
        for _ in range(args.n):
            fn()
        torch.cuda.synchronize()
        w, s_1 = time.perf_counter() - w0, snap()
        names = thread_names()
        d = {t: s_1[t] - s0.get(t, 0.0) for t in s_1}
        others = sorted(((v, t) for t, v in d.items() if t != main_tid and v > 0), reverse=True)[:4]
        rows.append({"case": name, "wall_us": round(w / args.n * 1e6, 2),
                     "main_thread_us": round(d.get(main_tid, 0.0) / args.n * 1e6, 2),
                     "other_threads_us": {f"{names.get(t, '?')}[{t}]": round(v / args.n * 1e6, 2)
                                          for v, t in others}})
        print(json.dumps(rows[-1]), flush=True)
    # time-based or count-based?  ONE cross-stream wait on an event behind ~`long_ms` of work on
    # the other stream, the host idle meanwhile (torch.cuda.synchronize): the runtime threads'
    # CPU over the whole span, vs the same work with no cross-stream wait
    big = torch.empty(1 << 28, device=dev)  # 1 GiB
    big2 = torch.empty_like(big)
    for wait in (False, True, False, True):
        torch.cuda.synchronize()
        s0, w0 = snap(), time.perf_counter()
        for _ in range(5):
            for _ in range(20):
                big2.copy_(big)  # ~20 x 0.35 ms on s1
            ev[2].record(s1)
            if wait:
                s2.wait_event(ev[2])
                ev[3].record(s2)
            torch.cuda.synchronize()
        w, s_1 = time.perf_counter() - w0, snap()
        d = {t: s_1[t] - s0.get(t, 0.0) for t in s_1}
        other = sum(v for t, v in d.items() if t != main_tid)
        print(json.dumps({"case": f"long work on s1, cross-stream wait on it: {wait}",
                          "wall_ms_per_rep": round(w / 5 * 1e3, 3),
                          "other_threads_ms_per_rep": round(other / 5 * 1e3, 3),
                          "main_thread_ms_per_rep": round(d.get(main_tid, 0.0) / 5 * 1e3, 3)}),
              flush=True)
    print(json.dumps({"threads": sorted(set(thread_names().values()))}), flush=True)


if __name__ == "__main__":
    main()
