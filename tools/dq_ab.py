"""In-process A/B of the fp8 gathered-dequantise variants (zs_tune knobs) on one C5 decoder layer
(VERDICT r3 next #3), interleaved so placement and clock drift hit every variant alike: accesses in
flight per lane (4 / 8 / 16), non-temporal vs plain stores, one wave per row vs k workgroups per
CU; ws = 1 layout (the kernel table's) and the ws = 8 layout (each matrix's rows gathered from 8
rank chunks).  Every variant's output must equal the default's bit for bit.  The in-place float4
copy over the same output buffer is timed beside them (this memory's streaming ceiling).

Usage: python tools/dq_ab.py [--iters 20] [--blocks 4] [--out FILE]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))

VARIANTS = [  # (dq_unroll, dq_nt_store, dq_wg_per_cu); the first is the library default
    (4, 1, 0), (8, 1, 0), (16, 1, 0), (4, 0, 0), (8, 0, 0), (4, 1, 8), (8, 1, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import numpy as np
    import torch

    from zero_amd import _lib
    from zero_amd.engine import probed_zeros
    from zero_amd.kernels import CopySet, stream_handle
    from zero_amd.shapes import decoder_shapes

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    layer = [s for s in decoder_shapes("C5", 1)[1:10] if len(s) == 2]
    elems = sum(int(np.prod(s)) for s in layer)
    nrows = sum(s[0] for s in layer)
    alg = 3 * elems + 4 * nrows
    q_buf, _ = probed_zeros(max(elems + 64 * len(layer), 1 << 30), torch.uint8, dev)
    out_buf, _ = probed_zeros(max(elems, 1 << 29), torch.bfloat16, dev)
    sc = torch.rand(nrows + 64, device=dev) * 0.01 + 1e-3
    g = torch.Generator(device=dev).manual_seed(0)
    q_buf[:elems].copy_(torch.randint(0, 256, (elems,), device=dev, dtype=torch.uint8, generator=g)
                        & 0x7E)  # finite E4M3 codes only (no NaN 0x7F / 0xFF)

    def layout(ws):
        rows = np.array([r for r, _ in layer], np.int64)
        cs = rows // ws
        row_len = np.array([c for _, c in layer], np.int64)
        q_off = np.cumsum(np.concatenate([[0], cs * row_len]))[:-1].astype(np.int64)
        sc_off = np.cumsum(np.concatenate([[0], cs]))[:-1].astype(np.int64)
        q_rank, sc_rank = int((cs * row_len).sum()), int(cs.sum())
        o = np.cumsum(np.concatenate([[0], rows * row_len]))[:-1].astype(np.uint64)
        dst = np.uint64(out_buf.data_ptr()) + o * np.uint64(2)
        return cs, row_len, q_off, sc_off, q_rank, sc_rank, dst

    def run(lay, ws):
        cs, row_len, q_off, sc_off, q_rank, sc_rank, dst = lay
        _lib.call("zs_fp8_dequantize_gathered", len(cs), q_buf.data_ptr(), sc.data_ptr(), ws,
                  q_rank, sc_rank, q_off.ctypes.data, sc_off.ctypes.data, cs.ctypes.data,
                  row_len.ctypes.data, dst.ctypes.data, _lib.ZS_BF16, stream_handle(st))

    def tune(v):
        for k, x in zip(("dq_unroll", "dq_nt_store", "dq_wg_per_cu"), v):
            _lib.call("zs_tune", k.encode(), x, None)

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / args.iters

    nb = out_buf.numel() * 2
    cp = CopySet([out_buf.data_ptr()], [out_buf.data_ptr()], [nb])
    res = {}
    ref = {}
    for ws in (1, 8):
        lay = layout(ws)
        tune(VARIANTS[0])
        run(lay, ws)
        torch.cuda.synchronize()
        ref[ws] = out_buf[:elems].view(torch.int16).clone()
        for v in VARIANTS:
            tune(v)
            out_buf[:elems].zero_()
            run(lay, ws)
            torch.cuda.synchronize()
            assert torch.equal(out_buf[:elems].view(torch.int16), ref[ws]), ("bits differ", ws, v)
    for b in range(args.blocks):
        order = VARIANTS if b % 2 == 0 else VARIANTS[::-1]
        for ws in (1, 8):
            lay = layout(ws)
            for v in order:
                tune(v)
                ms = timed(lambda: run(lay, ws))
                res.setdefault(f"ws{ws} unroll{v[0]} nt{v[1]} wgcu{v[2]}", []).append(ms)
        res.setdefault("copy in place (out buffer)", []).append(timed(lambda: cp.run(st)))
    tune(VARIANTS[0])
    rows = []
    for k, v in res.items():
        ms = sorted(v)[len(v) // 2]
        b = 2 * nb if k.startswith("copy") else alg
        rows.append({"variant": k, "median_ms": ms, "gbs": b / (ms / 1e3) / 1e9,
                     "frac": b / (ms / 1e3) / 1e9 / 8000.0, "ms_blocks": v})
        print(json.dumps({kk: (round(x, 4) if isinstance(x, float) else x) for kk, x in rows[-1].items()
                          if kk != "ms_blocks"}), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"alg_bytes": alg, "iters": args.iters, "rows": rows},
                                             indent=1) + "\n")


if __name__ == "__main__":
    main()
