"""Summarise separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py into the JSON
bench.py reads for roofline.traffic (profiles/*_adam_pmc.json).

FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE reports 1/2 of a wide coalesced
(16 B/lane) streaming read, so it is doubled (MI355X_MICROARCH.md §HBM; calibrated on a 4 GiB copy,
profiles/r01_c4_n1_adam_pmc.json "calibration").  The timed launches are the last ones of the run.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <kernel substring> <out.json> \
           <alg_bytes_per_launch> <config json> <command>
"""
import csv
import json
import sys
from pathlib import Path


def values(d, counter, kernel):
    rows = list(csv.DictReader(open(Path(d) / "run_counter_collection.csv")))
    sel = [r for r in rows if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return [float(r["Counter_Value"]) for r in sel], (sel[0]["Kernel_Name"] if sel else None)


def main():
    fdir, wdir, kernel, out, alg, cfg, cmd = sys.argv[1:8]
    f, name = values(fdir, "FETCH_SIZE", kernel)
    w, _ = values(wdir, "WRITE_SIZE", kernel)
    fk, wk = f[-1], w[-1]
    hbm = fk * 2 * 1024 + wk * 1024
    prev = {}
    p = Path(out)
    if p.exists():
        prev = json.loads(p.read_text())
    d = {
        "config": json.loads(cfg), "kernel": name[name.index(kernel):].split("(")[0],
        "command": cmd, "units": "FETCH_SIZE / WRITE_SIZE are KiB per dispatch",
        "fetch_size_kib": fk, "write_size_kib": wk, "fetch_bytes_corrected": fk * 2 * 1024,
        "write_bytes": wk * 1024, "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": int(float(alg)),
        "traffic_over_algorithmic": hbm / float(alg),
        "dispatches_seen": {"fetch": len(f), "write": len(w)},
        "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM: gfx950 FETCH_SIZE reports 1/2 of a "
                      "wide coalesced stream); WRITE_SIZE exact",
    }
    for k in ("calibration", "first_kernel_r01"):
        if k in prev:
            d[k] = prev[k]
    p.write_text(json.dumps(d, indent=1) + "\n")
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
