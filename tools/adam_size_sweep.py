"""Why C2's fused Adam reaches a lower fraction of 8 TB/s than C3/C4/C5.

One launch over n fp32 elements (C2's precision: fp32 params, grads, m, v — 28 B/element) is timed
with HIP events at n = C2 x {1/8 ... 16}, interleaved, on one contiguous segment and on C2's own 12
segments (6 x 4096^2 + 6 x 4096).  A straight-line fit t(n) = a + bytes(n) / B separates the fixed
cost of a launch (a: ramp-up of 32k workgroups over 256 CUs plus the drain of the last ones) from
the steady streaming rate B; C2's achieved fraction is then B's fraction diluted by a.  The same
for an in-place float4 copy of the same bytes (the streaming ceiling), and C2 through grids of 8 to
128 workgroups per CU (``zs_tune adam_wg_per_cu``).

Usage: python tools/adam_size_sweep.py [--reps 3] [--iters 30] [--out profiles/r05_c2_adam_sweep.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))

HBM_PEAK_GBS = 8000.0
C2_ELEMS = 6 * 4096 * 4096 + 6 * 4096


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import numpy as np
    import torch

    from zero_amd import _lib
    from zero_amd.kernels import AdamSet, CopySet, adam_hparams

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    nmax = C2_ELEMS * 16
    # one buffer per stream, sized for the largest n (fp32: p, g, m, v)
    P, G, M, V = (torch.zeros(nmax, dtype=torch.float32, device=dev) for _ in range(4))
    G.normal_(0.0, 1e-3)
    hp = adam_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, 1)

    def rows_for(lengths):
        rows, o = [], 0
        assert sum(-(-n // 64) * 64 for n in lengths) <= nmax  # every segment inside the buffers
        for n in lengths:
            rows.append([G.data_ptr() + 4 * o, P.data_ptr() + 4 * o, P.data_ptr() + 4 * o, 0,
                         M.data_ptr() + 4 * o, V.data_ptr() + 4 * o, 0, 0, n])
            o += -(-n // 64) * 64
        return np.array(rows, np.uint64)

    def time_launch(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / args.iters

    fracs = [1 / 8, 1 / 4, 1 / 2, 1, 2, 4, 8, 16]
    sets = {f: AdamSet(rows_for([int(C2_ELEMS * f) // 64 * 64]), _lib.ZS_F32) for f in fracs}
    c2_segs = [4096 * 4096, 4096] * 6
    c2 = AdamSet(rows_for(c2_segs), _lib.ZS_F32)
    # in place over a buffer of its own, 14 B per Adam element copied: read + write = 28 B
    C = torch.zeros(14 * nmax // 4, dtype=torch.float32, device=dev)
    copies = {}
    for f in fracs:
        nb = 14 * (int(C2_ELEMS * f) // 64 * 64)
        assert nb <= C.numel() * 4
        copies[f] = CopySet([C.data_ptr()], [C.data_ptr()], [nb])
    rows = []
    for rep in range(args.reps):
        for f in (fracs if rep % 2 == 0 else fracs[::-1]):
            ms = time_launch(lambda s=sets[f]: s.run(hp, st))
            cms = time_launch(lambda c=copies[f]: c.run(st))
            n = int(C2_ELEMS * f) // 64 * 64
            rows.append({"rep": rep, "scale": f, "elems": n, "adam_ms": ms, "copy_ms": cms,
                         "adam_gbs": 28 * n / ms / 1e6, "copy_gbs": 28 * n / cms / 1e6})
            print(json.dumps(rows[-1]), flush=True)
    grid_rows = []
    for rep in range(args.reps):
        for wg in (0, 8, 16, 32, 64, 128):
            _lib.call("zs_tune", b"adam_wg_per_cu", wg, None)
            ms = time_launch(lambda: c2.run(hp, st))
            grid_rows.append({"rep": rep, "wg_per_cu": wg or 128, "c2_segments_ms": ms,
                              "frac": 28 * C2_ELEMS / ms / 1e6 / HBM_PEAK_GBS})
            print(json.dumps(grid_rows[-1]), flush=True)
    _lib.call("zs_tune", b"adam_wg_per_cu", 0, None)

    def fit(key):
        x = np.array([28 * r["elems"] for r in rows], np.float64)
        y = np.array([r[key] for r in rows], np.float64)
        slope, icpt = np.polyfit(x, y, 1)
        return {"fixed_us": icpt * 1e3, "steady_gbs": 1 / slope / 1e6,
                "steady_frac": 1 / slope / 1e6 / HBM_PEAK_GBS}

    med = lambda v: float(np.median(v))  # noqa: E731
    c2_ms = med([r["adam_ms"] for r in rows if r["scale"] == 1])
    fa, fc = fit("adam_ms"), fit("copy_ms")
    summary = {
        "c2_elems": C2_ELEMS, "c2_adam_bytes": 28 * C2_ELEMS, "c2_one_segment_ms": c2_ms,
        "c2_one_segment_frac": 28 * C2_ELEMS / c2_ms / 1e6 / HBM_PEAK_GBS,
        "c2_12_segments_ms_by_grid": {str(w): med([r["c2_segments_ms"] for r in grid_rows
                                                   if r["wg_per_cu"] == w]) for w in (128, 8, 16, 32, 64)},
        "fit_adam": fa, "fit_copy": fc,
        "c2_fixed_share": fa["fixed_us"] / 1e3 / c2_ms,
        "c2_frac_if_no_fixed_cost": fa["steady_frac"],
    }
    print(json.dumps(summary), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"summary": summary, "sizes": rows, "grids": grid_rows},
                                             indent=1) + "\n")


if __name__ == "__main__":
    main()
