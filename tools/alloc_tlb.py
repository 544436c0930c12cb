"""Why does a streaming kernel's bandwidth depend on WHICH allocation it streams?

Round 1 saw the same Adam launch at 5.3-6.2 TB/s depending on the allocation of its state and
kept the fastest of 5 candidates (engine.probed_zeros).  This probe measures, in one process:

  torch   — K buffers from torch's caching allocator (plain hipMalloc underneath), held together;
  contig  — K buffers from hipExtMallocWithFlags(hipDeviceMallocContiguous): physically
            contiguous VRAM, so the GPU page tables can use the largest fragments;
  default — K buffers from hipExtMallocWithFlags(hipDeviceMallocDefault) via the same path
            (control for the raw-pointer path).

For each buffer: the gfx950 segment-copy kernel (copy_segments_kernel) streams it in place
(read + write every byte) 3 times; the best time → GB/s.  Prints one JSON line per buffer.
Run with PYTORCH_HIP_ALLOC_CONF=expandable_segments:True to see torch's VMM allocator instead.

    python tools/alloc_tlb.py [--gib 8] [--k 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))

hipDeviceMallocDefault = 0x0
hipDeviceMallocContiguous = 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--modes", default="torch,contig,default")
    ap.add_argument("--warm-s", type=float, default=0.0,
                    help="stream the first buffer continuously this long before measuring "
                         "(lets the clocks settle)")
    ap.add_argument("--sizes", default=None,
                    help="comma list of GiB: one buffer per size, interleaved rounds")
    ap.add_argument("--rounds", type=int, default=1,
                    help="measure every held buffer round-robin this many times")
    ap.add_argument("--many", default=None,
                    help="MiB,count: hold `count` buffers of MiB each (torch allocator and raw "
                         "hipMalloc), print every buffer's GB/s and address")
    a = ap.parse_args()

    import torch

    from zero_amd.kernels import CopySet

    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipExtMallocWithFlags.restype = ctypes.c_int
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipMalloc.restype = ctypes.c_int
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    nbytes = int(a.gib * (1 << 30)) // 256 * 256
    st = torch.cuda.current_stream(dev)

    def measure(ptr):
        cs = CopySet([ptr], [ptr], [nbytes])
        cs.run(st)  # first touch / warm
        best = None
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            cs.run(st)
            e1.record(st)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return 2 * nbytes / (best / 1e3) / 1e9

    import time

    if a.many:
        mib, count = (int(x) for x in a.many.split(","))
        nb = mib << 20
        for mode in ("torch", "hipMalloc"):
            held, rows = [], []
            for k in range(count):
                if mode == "torch":
                    t = torch.empty(nb // 4, dtype=torch.float32, device=dev)
                    held.append(t)
                    ptr = t.data_ptr()
                else:
                    q = ctypes.c_void_p()
                    if hip.hipMalloc(ctypes.byref(q), ctypes.c_size_t(nb)) != 0:
                        break
                    held.append(q)
                    ptr = q.value
                cs = CopySet([ptr], [ptr], [nb])
                cs.run(st)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(10):
                    cs.run(st)
                e1.record(st)
                e1.synchronize()
                gbs = 10 * 2 * nb / (e0.elapsed_time(e1) / 1e3) / 1e9
                rows.append((k, ptr, round(gbs)))
            for k, ptr, gbs in rows:
                print(json.dumps({"mode": mode, "mib": mib, "k": k, "addr_hex": hex(ptr),
                                  "addr_mod_2m": ptr % (2 << 20), "gbs": gbs}), flush=True)
            torch.cuda.synchronize()
            for h in held:
                if isinstance(h, ctypes.c_void_p):
                    hip.hipFree(h)
            del held
            torch.cuda.empty_cache()
        return

    if a.sizes:  # buffer-size effect: one buffer per size, each streamed with its own size
        sizes = [int(float(x) * (1 << 30)) // 256 * 256 for x in a.sizes.split(",")]
        bufs = [torch.zeros(n // 4, dtype=torch.float32, device=dev) for n in sizes]
        for r in range(max(a.rounds, 1)):
            row = {}
            for n, b in zip(sizes, bufs):
                nonlocal_n = n
                cs = CopySet([b.data_ptr()], [b.data_ptr()], [nonlocal_n])
                cs.run(st)
                best = None
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    cs.run(st)
                    e1.record(st)
                    e1.synchronize()
                    ms = e0.elapsed_time(e1)
                    best = ms if best is None else min(best, ms)
                row[f"{n / (1 << 30):.1f}GiB"] = round(2 * n / (best / 1e3) / 1e9, 1)
            print(json.dumps({"mode": "sizes", "round": r, "copy_gbs": row}), flush=True)
        return

    alloc_conf = os.environ.get("PYTORCH_HIP_ALLOC_CONF", "")
    for mode in a.modes.split(","):
        if a.rounds > 1:  # interleaved: buffer effect vs time (clock) effect
            bufs = [torch.zeros(nbytes // 4, dtype=torch.float32, device=dev) for _ in range(a.k)]
            if a.warm_s > 0:
                cs = CopySet([bufs[0].data_ptr()], [bufs[0].data_ptr()], [nbytes])
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < a.warm_s:
                    for _ in range(20):
                        cs.run(st)
                    st.synchronize()
            for r in range(a.rounds):
                row = [round(measure(b.data_ptr()), 1) for b in bufs]
                print(json.dumps({"mode": f"{mode}-interleaved", "round": r, "warm_s": a.warm_s,
                                  "copy_gbs_per_buffer": row}), flush=True)
            del bufs
            torch.cuda.empty_cache()
            continue
        held = []
        for k in range(a.k):
            free, _ = torch.cuda.mem_get_info(dev)
            if free < nbytes + (4 << 30):
                break
            if mode == "torch":
                t = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
                held.append(t)
                ptr, rc = t.data_ptr(), 0
            else:
                p = ctypes.c_void_p()
                flag = hipDeviceMallocContiguous if mode == "contig" else hipDeviceMallocDefault
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flag)
                if rc != 0:
                    print(json.dumps({"mode": mode, "k": k, "error": f"hipExtMallocWithFlags rc={rc}"}),
                          flush=True)
                    break
                hip.hipMemset(p, 0, nbytes)
                held.append(p)
                ptr = p.value
            gbs = measure(ptr)
            print(json.dumps({"mode": mode, "alloc_conf": alloc_conf, "k": k, "gib": a.gib,
                              "addr_gib": round(ptr / (1 << 30), 2), "copy_gbs": round(gbs, 1)}),
                  flush=True)
        torch.cuda.synchronize()
        for h in held:
            if isinstance(h, ctypes.c_void_p):
                hip.hipFree(h)
        del held
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
