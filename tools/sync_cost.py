"""Host cost of the primitives a two-stream ZeRO-3 gather adds over a single-stream one (VERDICT r4
#2): per call, wall time of the calling thread and process CPU (all threads), for a sync record,
a sync wait (flag and event; producer idle, and producer far behind the host), the side-stream
allocation, ``record_stream``, ``hipStreamQuery`` and one ordered library call with no collective
(the simulated gather's whole device work).  Each primitive runs in blocks of ``--n`` calls; the median block is
reported.

Usage: python tools/sync_cost.py [--n 2000] [--blocks 5] [--out profiles/r05_sync_cost.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--blocks", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import numpy as np
    import torch

    import bench
    from zero_amd import _lib
    from zero_amd.comm import Sync

    dev = torch.device("cuda:0")
    side, cons = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    sh, ch = side.cuda_stream, cons.cuda_stream
    side_ids = (side.stream_id, side.device_index, side.device_type)
    syncs = {k: Sync(getattr(_lib, f"ZS_SYNC_{k.upper()}")) for k in ("flag", "event")}
    nc = bench._NoComm(8)
    send, recv = np.zeros(1, np.uint64), np.zeros(1, np.uint64)
    count = np.zeros(1, np.int64)
    ordered = nc.all_gather_group_synced_bound(send, recv, count, 0)
    flag_ready, flag_done = Sync(_lib.ZS_SYNC_FLAG), Sync(_lib.ZS_SYNC_FLAG)
    x = torch.empty(1 << 20, dtype=torch.bfloat16, device=dev)
    import ctypes
    import os

    hip_path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    hip = ctypes.CDLL(hip_path if os.path.exists(hip_path) else "libamdhip64.so")
    hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
    cons_obj = torch.cuda.ExternalStream(ch, device=dev)

    def side_empty():
        prev = torch._C._cuda_getCurrentStream(0)
        torch._C._cuda_setStream(*side_ids)
        try:
            return torch.empty(1 << 20, dtype=torch.bfloat16, device=dev)
        finally:
            torch._C._cuda_setStream(*prev)

    prims = {
        "flag record": lambda: syncs["flag"].record(sh),
        "flag wait": lambda: syncs["flag"].wait(ch),
        "event record": lambda: syncs["event"].record(sh),
        "event wait": lambda: syncs["event"].wait(ch),
        "ordered call, done only (flag)": lambda: ordered(ch, 0, sh, flag_done.h),
        "ordered call, ready + done (flag)": lambda: ordered(ch, flag_ready.h, sh, flag_done.h),
        "ordered call, no syncs": lambda: ordered(ch, 0, sh, 0),
        "torch.empty (current stream)": lambda: torch.empty(1 << 20, dtype=torch.bfloat16,
                                                            device=dev),
        "torch.empty on the side stream": side_empty,
        "record_stream": lambda: x.record_stream(cons_obj),
        "current raw stream handle": lambda: torch._C._cuda_getCurrentRawStream(0),
        "hipStreamQuery (producer stream)": lambda: hip.hipStreamQuery(sh),
    }
    rows = []
    for behind in (False, True):
        for name, fn in prims.items():
            per = []
            for b in range(args.blocks):
                torch.cuda.synchronize()
                if behind:  # the producer (side stream) ~far behind the host
                    with torch.cuda.stream(side):
                        torch.cuda._sleep(20_000_000)
                    syncs["flag"].record(sh)
                    syncs["event"].record(sh)
                w0, c0 = time.perf_counter(), time.process_time()
                for _ in range(args.n):
                    fn()
                w, c = time.perf_counter() - w0, time.process_time() - c0
                per.append((w / args.n * 1e6, c / args.n * 1e6))
                torch.cuda.synchronize()
            per.sort()
            rows.append({"primitive": name, "producer_behind": behind,
                         "wall_us": round(per[len(per) // 2][0], 3),
                         "cpu_us": round(sorted(p[1] for p in per)[len(per) // 2], 3)})
            print(json.dumps(rows[-1]), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"n": args.n, "blocks": args.blocks, "rows": rows},
                                             indent=1) + "\n")


if __name__ == "__main__":
    main()
