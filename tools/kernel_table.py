"""Roofline table of the gfx950 kernels beside Adam: each kernel at the size the
product launches it with, its algorithmic HBM bytes per launch, the average launch time from HIP
events on the launch stream, achieved GB/s and the fraction of the 8 TB/s HBM peak.  Run it under
``rocprofv3 --kernel-trace --stats`` as well; the two must agree on the per-kernel durations.

  convert_kernel<true>   fp32 -> bf16 RNE, C3-size gradient (983,116,800 elements): the
                         grad_comm="bf16" conversion before the exchange; 4 + 2 B/element
  convert_kernel<false>  bf16 -> fp32, same size; 2 + 4 B/element
  fp8_quantize_rowset    one C5 decoder layer's matrices (bf16, row-scaled E4M3, the ZeRO-3
                         gather_dtype="fp8" send side, one launch per register class):
                         2 + 1 B/element + 4 B/row
  fp8_dequantize_gathered  the same layer gathered (receive side, one launch): 1 + 2 B/element
                         + 4 B/row.  (Round 5: the per-matrix zs_fp8_*_rows forms are off the
                         product path — a standalone Zero3ParamManager runs these two kernels as a
                         one-matrix set — so they are not in the table.)
  scale_kernel           DDP's grad /= ws, in place, bf16 and fp32: a 256 MiB bucket (MALL-sized)
                         and a 4 GiB buffer (HBM): 2 x element size per element
  copy_segments_kernel   pack of the C4 set's grads into one rank-major arena (every tensor a
                         segment, bf16): 2 x 2 B/element

Usage: python tools/kernel_table.py [--iters 20] [--out profiles/r03_kernels_table.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import numpy as np
    import torch

    from zero_amd import _lib
    from zero_amd.engine import probed_zeros
    from zero_amd.kernels import CopySet, convert, stream_handle
    from zero_amd.shapes import decoder_shapes, mlp_shapes, smollm3_3b_shapes

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    rows = []

    def timed(name, launch, alg_bytes, note, rocprof=None, per_call=1):
        launch()  # warm
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            launch()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        gbs = alg_bytes / (ms / 1e3) / 1e9
        row = {"kernel": name, "avg_launch_ms": ms, "alg_bytes_per_launch": int(alg_bytes),
               "achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS, "workload": note,
               # for tools/kernel_pmc.py: the rocprof kernel-name prefix and dispatches per call
               "rocprof_kernel": rocprof, "dispatches_per_call": per_call}
        rows.append(row)
        print(json.dumps(row), flush=True)

    # convert: C3-size gradient (6 x Linear(12800, 12800) + biases)
    n = int(sum(int(np.prod(s)) for s in mlp_shapes(12800)))
    src, _ = probed_zeros(n, torch.float32, dev)
    dst, _ = probed_zeros(n, torch.bfloat16, dev)
    src.normal_()
    timed("convert_kernel<true> (fp32->bf16)", lambda: convert(src, dst, st), 6 * n,
          f"C3 gradient, {n:,} elements (grad_comm='bf16')", "convert_kernel<true,")
    timed("convert_kernel<false> (bf16->fp32)", lambda: convert(dst, src, st), 6 * n,
          f"C3 gradient, {n:,} elements", "convert_kernel<false,")
    del src, dst
    torch.cuda.empty_cache()

    # fp8 row quantise / dequantise: one C5 decoder layer's matrices (bf16), in placed buffers
    # (engine.probed_zeros, as every HBM-sized buffer of the product path) so the kernels are
    # measured on the same kind of memory as Adam; the in-place copy rows at the end give the
    # streaming rate of these very buffers (the ceiling the kernels can reach here)
    layer = [s for s in decoder_shapes("C5", 1)[1:10] if len(s) == 2]
    elems = sum(int(np.prod(s)) for s in layer)
    nrows = sum(s[0] for s in layer)
    gib = 1 << 30
    src_buf, _ = probed_zeros(max(elems, gib // 2), torch.bfloat16, dev)
    q_buf, _ = probed_zeros(max(elems + 64 * len(layer), gib), torch.uint8, dev)
    out_buf, _ = probed_zeros(max(elems, gib // 2), torch.bfloat16, dev)
    sc_buf = torch.empty(nrows + 64 * len(layer), dtype=torch.float32, device=dev)
    mats, qs, scs, outs, o = [], [], [], [], 0
    so = 0
    for s_ in layer:
        k = int(np.prod(s_))
        mats.append(src_buf[o:o + k].view(s_))
        qs.append(q_buf[o:o + k].view(s_))
        outs.append(out_buf[o:o + k].view(s_))
        scs.append(sc_buf[so:so + s_[0]])
        o += k
        so += s_[0]
    for x in mats:
        x.normal_()

    # the gather group's fused forms: one quantise launch per register class into one
    # concatenated send buffer, one dequantise launch from it (ws = 1 layout: the gathered buffer
    # is the send buffer)
    shp = [tuple(x.shape) for x in mats]
    q_off = np.cumsum([0] + [r * c for r, c in shp])[:-1].astype(np.int64)
    sc_off = np.cumsum([0] + [r for r, _ in shp])[:-1].astype(np.int64)
    qtot, sctot = int(sum(r * c for r, c in shp)), int(sum(r for r, _ in shp))
    src = np.array([x.data_ptr() for x in mats], np.uint64)
    qp = np.uint64(q_buf.data_ptr()) + q_off.astype(np.uint64)
    sp = np.uint64(sc_buf.data_ptr()) + (sc_off * 4).astype(np.uint64)
    rows_a = np.array([r for r, _ in shp], np.int64)
    len_a = np.array([c for _, c in shp], np.int64)
    dst = np.array([y.data_ptr() for y in outs], np.uint64)
    nreg = sorted({8 if c <= 4096 else 16 if c <= 8192 else 32 for c in len_a})
    timed(f"fp8_quantize_rowset_kernel<bf16> ({len(mats)} matrices, one launch per register class)",
          lambda: _lib.call("zs_fp8_quantize_rowset", len(mats), src.ctypes.data, qp.ctypes.data,
                            sp.ctypes.data, rows_a.ctypes.data, rows_a.ctypes.data,
                            len_a.ctypes.data, _lib.ZS_BF16, stream_handle(st)),
          3 * elems + 4 * nrows, f"one C5 decoder layer, {elems:,} bf16 elements",
          "fp8_quantize_rowset_kernel<unsigned short,", len(nreg))
    timed(f"fp8_dequantize_gathered_kernel<bf16> ({len(mats)} matrices, one launch)",
          lambda: _lib.call("zs_fp8_dequantize_gathered", len(mats), q_buf.data_ptr(),
                            sc_buf.data_ptr(), 1, qtot, sctot, q_off.ctypes.data, sc_off.ctypes.data,
                            rows_a.ctypes.data, len_a.ctypes.data, dst.ctypes.data, _lib.ZS_BF16,
                            stream_handle(st)),
          3 * elems + 4 * nrows, f"one C5 decoder layer, {elems:,} elements",
          "fp8_dequantize_gathered_kernel<unsigned short,", 1)
    # (the in-place copies over these buffers run at the very end: see below)

    # DDP scale, in place: a 256 MiB bucket (fits the 256 MB MALL, so repeated launches partly hit
    # it — the figure is not an HBM rate) and a 4 GiB buffer (HBM-bound, placed by the probe)
    for mib in (64, 256, 4096):
        for dt, code, es in ((torch.bfloat16, _lib.ZS_BF16, 2), (torch.float32, _lib.ZS_F32, 4)):
            m = (mib << 20) // es
            if mib >= 1024:  # placed like the other rows' HBM-sized buffers (engine.probed_zeros)
                b, _ = probed_zeros(m, dt, dev)
                b.normal_()
            else:
                b = torch.randn(m, device=dev).to(dt)
            timed(f"scale_kernel<{'bf16' if es == 2 else 'f32'}> (/3, in place, {mib} MiB)",
                  lambda b=b, code=code: _lib.call("zs_scale", b.data_ptr(), b.numel(), code, 3.0,
                                                   stream_handle(st)),
                  2 * es * m, f"DDP bucket, {mib} MiB {dt}" + (" (MALL-resident)" if mib <= 256 else ""),
                  f"scale_kernel<{'unsigned short' if es == 2 else 'float'},")  # (either cache policy)
            del b
            torch.cuda.empty_cache()

    # pack: the C4 set's bf16 grads (326 segments) into one rank-major arena
    shapes = smollm3_3b_shapes()
    total = int(sum(int(np.prod(s)) for s in shapes))
    grads, _ = probed_zeros(total, torch.bfloat16, dev)
    arena, _ = probed_zeros(total + 64 * len(shapes), torch.bfloat16, dev)
    src, dst, nb, o, a = [], [], [], 0, 0
    for s in shapes:
        k = int(np.prod(s))
        src.append(grads.data_ptr() + 2 * o)
        dst.append(arena.data_ptr() + 2 * a)
        nb.append(2 * k)
        o += k
        a += -(-k // 64) * 64
    cs = CopySet(src, dst, nb)
    timed("copy_segments_kernel (pack, 326 segments)", lambda: cs.run(st), 2 * cs.nbytes,
          f"C4 bf16 grads, {total:,} elements, one launch", "copy_segments_kernel<")
    del grads, arena, cs
    # the streaming rate of the fp8 rows' own buffers (in-place float4 copy, read + write): the
    # ceiling those kernels can reach on this memory
    for nm, buf in (("fp8 layer output buffer", out_buf), ("fp8 layer q buffer", q_buf)):
        nb = buf.numel() * buf.element_size()
        cp = CopySet([buf.data_ptr()], [buf.data_ptr()], [nb])
        timed(f"copy_segments_kernel (in place, {nm})", lambda cp=cp: cp.run(st), 2 * nb,
              f"{nb:,} B, the buffer the fp8 rows use", "copy_segments_kernel<")
    if args.out:
        Path(args.out).write_text(json.dumps({"iters": args.iters, "peak_gbs": HBM_PEAK_GBS,
                                              "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
