"""In-process A/B of the cache policy of zs_scale, zs_convert and the segment copy (zs_tune
"scale_nt" / "convert_nt" / "copy_nt": 0 default policy, 1 non-temporal loads and stores) over buffer sizes either side of
the 256 MB MALL, interleaved so placement and clock drift hit both alike.  Every buffer is a placed
one (probed_zeros), and the in-place float4 copy over the same buffer is timed beside them (this
memory's streaming ceiling).  Both policies must give the same bits.

Usage: python tools/scale_ab.py [--iters 20] [--blocks 4] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))

SIZES_MIB = (64, 256, 1024, 4096)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    from zero_amd import _lib
    from zero_amd.engine import probed_zeros
    from zero_amd.kernels import CopySet, stream_handle

    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    h = stream_handle(st)
    nbytes = max(SIZES_MIB) << 20
    buf, _ = probed_zeros(nbytes // 4, torch.float32, dev)
    half, _ = probed_zeros(nbytes // 4, torch.bfloat16, dev)  # the bf16 side of the conversions
    g = torch.Generator(device=dev).manual_seed(0)
    buf.normal_(generator=g)
    base = buf.clone()

    def tune(v, key=b"scale_nt"):
        _lib.call("zs_tune", key, v, None)

    def conv(src, dst):
        _lib.call("zs_convert", src.data_ptr(), _lib.ZS_F32 if src.dtype == torch.float32 else _lib.ZS_BF16,
                  dst.data_ptr(), _lib.ZS_F32 if dst.dtype == torch.float32 else _lib.ZS_BF16,
                  src.numel(), h)

    def run(t, n):
        _lib.call("zs_scale", t.data_ptr(), n, _lib.ZS_F32 if t.dtype == torch.float32 else _lib.ZS_BF16,
                  3.0, h)

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) / args.iters

    # same bits under both policies (one scale of a fresh copy each)
    for dt in (torch.float32, torch.bfloat16):
        outs = []
        for v in (0, 1):
            tune(v)
            buf.copy_(base)
            t = buf.view(torch.uint8)[: 64 << 20].view(dt)
            run(t, t.numel())
            torch.cuda.synchronize()
            outs.append(t.view(torch.int16 if dt == torch.bfloat16 else torch.int32).clone())
        assert torch.equal(outs[0], outs[1]), ("bits differ", dt)
    for v in (0, 1):
        tune(v, b"convert_nt")
        conv(base[: 16 << 20], half[: 16 << 20])
        torch.cuda.synchronize()
        outs.append(half[: 16 << 20].view(torch.int16).clone())
    assert torch.equal(outs[-2], outs[-1]), "convert bits differ"
    res = {}
    for b in range(args.blocks):
        for mib in SIZES_MIB:
            nb = mib << 20
            raw = buf.view(torch.uint8)[:nb]
            for dt in (torch.float32, torch.bfloat16):
                t = raw.view(dt)
                for v in ((0, 1) if b % 2 == 0 else (1, 0)):
                    tune(v)
                    ms = timed(lambda: run(t, t.numel()))
                    res.setdefault(f"{mib} MiB {str(dt)[6:]} nt{v}", []).append(ms)
            cp = CopySet([raw.data_ptr()], [raw.data_ptr()], [nb])
            tune(1, b"copy_nt")  # the ceiling reference: the policy every earlier table used
            res.setdefault(f"{mib} MiB copy in place", []).append(timed(lambda: cp.run(st)))
            # a pack-shaped copy: half of it from the fp32 buffer into the other buffer
            pk = CopySet([raw.data_ptr()], [half.data_ptr()], [nb // 2])
            for v in ((0, 1) if b % 2 == 0 else (1, 0)):
                tune(v, b"copy_nt")
                ms = timed(lambda: pk.run(st))
                res.setdefault(f"{mib} MiB copy (half) to another buffer nt{v}", []).append(ms)
            tune(-1, b"copy_nt")
            f32, b16 = raw.view(torch.float32), half[: nb // 4]
            for name, a, c in (("convert f32->bf16", f32, b16), ("convert bf16->f32", b16, f32)):
                for v in ((0, 1) if b % 2 == 0 else (1, 0)):
                    tune(v, b"convert_nt")
                    ms = timed(lambda: conv(a, c))
                    res.setdefault(f"{mib} MiB {name} nt{v}", []).append(ms)
    tune(-1)
    tune(-1, b"convert_nt")
    rows = []
    for k, v in res.items():
        ms = sorted(v)[len(v) // 2]
        nb = int(k.split()[0]) << 20
        # convert: the fp32 side + the bf16 side; the half copy: nb / 2 read + nb / 2 written
        moved = 1.5 * nb if "convert" in k else (nb if "(half)" in k else 2 * nb)
        gbs = moved / (ms / 1e3) / 1e9
        rows.append({"variant": k, "median_ms": ms, "gbs": gbs, "frac": gbs / 8000.0, "ms_blocks": v})
        print(json.dumps({kk: (round(x, 4) if isinstance(x, float) else x) for kk, x in rows[-1].items()
                          if kk != "ms_blocks"}), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"iters": args.iters, "rows": rows}, indent=1) + "\n")


if __name__ == "__main__":
    main()
