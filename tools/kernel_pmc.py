"""HBM traffic of the kernels beside Adam: combine separate rocprofv3
``--pmc FETCH_SIZE`` and ``--pmc WRITE_SIZE`` passes over ``tools/kernel_table.py`` with the table's
own rows into traffic ÷ algorithmic bytes per kernel.

Matching: every table row names its rocprof kernel-name prefix and its dispatches per call; the
table makes (iters + 1) calls per row (one warm).  For each prefix, the LAST
Σ_rows (iters + 1) × dispatches_per_call dispatches with that prefix are the rows' own (placement
probes that share the copy kernel's name run before the rows that use it), split in row order, and
a row's traffic is the sum over the dispatches of its last call.

Units and corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB per dispatch;
on gfx950 FETCH_SIZE reports 1/2 of a wide (16 B/lane) coalesced streaming read, so reads of
16 B/lane are doubled.  WRITE_SIZE is exact for 16 B/lane stores.  8-B/lane reads and stores are
not calibrated by the guide; they are calibrated here on known byte counts in the same run: the
bf16 -> fp32 conversion reads exactly 2 B x n with 8-B lanes (FETCH_SIZE = 1/2 of it, like the
16-B reads: doubled as well), and the fp32 -> bf16 conversion writes exactly 2 B x n with 8-B
lanes (WRITE_SIZE = all of it).  The raw counters are kept beside every corrected figure.

usage: python tools/kernel_pmc.py <kernel_table.json> <fetch_dir> <write_dir> <out.json> [timed.json]
(timed.json: an unprofiled kernel_table.py run whose launch times and fractions are reported —
the profiled passes run few iterations and their times are not the kernels')
"""
import csv
import json
import sys
from pathlib import Path

# lane width of each kernel's global reads / writes (bytes per lane per access)
READ_WIDTH = {"convert_kernel<true,": 16, "convert_kernel<false,": 8,
              "fp8_quantize_rows_wave_kernel<unsigned short,": 16,
              "fp8_quantize_rowset_kernel<unsigned short,": 16,
              "fp8_dequantize_gathered_kernel<unsigned short,": 8,
              "scale_kernel<unsigned short,": 16, "scale_kernel<float,": 16,
              "copy_segments_kernel<": 16}
WRITE_WIDTH = {"convert_kernel<true,": 8, "convert_kernel<false,": 16,
               "fp8_quantize_rows_wave_kernel<unsigned short,": 8,
               "fp8_quantize_rowset_kernel<unsigned short,": 8,
               "fp8_dequantize_gathered_kernel<unsigned short,": 16,
               "scale_kernel<unsigned short,": 16, "scale_kernel<float,": 16,
               "copy_segments_kernel<": 16}


def _norm(name: str) -> str:
    for pre in ("void ", "(anonymous namespace)::"):
        if name.startswith(pre):
            name = name[len(pre):]
    return name.replace("(anonymous namespace)::", "")


def _dispatches(d, counter):
    rows = [r for r in csv.DictReader(open(Path(d) / "run_counter_collection.csv"))
            if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(_norm(r["Kernel_Name"]), float(r["Counter_Value"])) for r in rows]


def per_row(table, disp):
    iters = table["iters"]
    out = {}
    prefixes = []
    for r in table["rows"]:
        if r.get("rocprof_kernel") and r["rocprof_kernel"] not in prefixes:
            prefixes.append(r["rocprof_kernel"])
    for pre in prefixes:
        rows = [r for r in table["rows"] if r.get("rocprof_kernel") == pre]
        need = sum((iters + 1) * r["dispatches_per_call"] for r in rows)
        vals = [v for k, v in disp if k.startswith(pre)]
        if len(vals) < need:
            raise SystemExit(f"{pre}: {len(vals)} dispatches in the trace, the table needs {need}")
        vals = vals[len(vals) - need:]
        i = 0
        for r in rows:
            n = (iters + 1) * r["dispatches_per_call"]
            mine = vals[i:i + n]
            i += n
            out[r["kernel"]] = sum(mine[-r["dispatches_per_call"]:])  # the last call
    return out


def main():
    tab, fdir, wdir, out = sys.argv[1:5]
    table = json.loads(Path(tab).read_text())
    timed = {r["kernel"]: r for r in json.loads(Path(sys.argv[5]).read_text())["rows"]} \
        if len(sys.argv) > 5 else {}
    fetch = per_row(table, _dispatches(fdir, "FETCH_SIZE"))
    write = per_row(table, _dispatches(wdir, "WRITE_SIZE"))
    rows = []
    for r in table["rows"]:
        k = r["kernel"]
        if k not in fetch:
            continue
        pre = r["rocprof_kernel"]
        fk, wk = fetch[k], write[k]
        rw, ww = READ_WIDTH.get(pre), WRITE_WIDTH.get(pre)
        fetch_b = fk * 1024 * (2 if rw in (8, 16) else 1)
        hbm = fetch_b + wk * 1024
        t = timed.get(k, r)
        rows.append({
            "kernel": k, "workload": r["workload"], "avg_launch_ms": t["avg_launch_ms"],
            "frac": t["frac"], "achieved_gbs": t.get("achieved_gbs"),
            "alg_bytes_per_call": r["alg_bytes_per_launch"],
            "fetch_size_kib": fk, "write_size_kib": wk, "read_bytes_per_lane": rw,
            "write_bytes_per_lane": ww,
            "fetch_bytes": fetch_b, "write_bytes": wk * 1024, "hbm_bytes_per_call": hbm,
            "traffic_over_algorithmic": hbm / r["alg_bytes_per_launch"],
            "fetch_correction": "x2 (16 B/lane reads, guide §HBM)" if rw == 16 else
                                "x2 (8 B/lane reads: calibrated on the bf16->fp32 conversion's "
                                "known 2 B/element read in this run)" if rw == 8 else "none"})
    doc = {"source": f"{tab} + rocprofv3 --pmc FETCH_SIZE ({fdir}) / --pmc WRITE_SIZE ({wdir}), "
                     "separate passes" + (f"; times and fractions from {sys.argv[5]}" if timed else ""),
           "units": "FETCH_SIZE / WRITE_SIZE: KiB per dispatch",
           "rows": rows}
    Path(out).write_text(json.dumps(doc, indent=1) + "\n")
    for x in rows:
        print(f"{x['kernel'][:70]:70s} frac {x['frac']:.3f} traffic/alg {x['traffic_over_algorithmic']:.3f}"
              f" (fetch {x['fetch_size_kib']:.0f} KiB, write {x['write_size_kib']:.0f} KiB)")


if __name__ == "__main__":
    main()
