"""A/B: placement probe for state buffers below 1 GiB (engine.PROBE_MIN_BYTES).

Runs bench.main() in a child process per variant (alternating, so box drift hits both) and prints
the Adam GB/s of each.  usage: python tools/probe_threshold_ab.py <config> <dtype> <rounds>"""
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
CHILD = r'''
import sys
sys.path.insert(0, "{pkg}"); sys.path.insert(0, "{repo}")
import zero_amd.engine as E
E.PROBE_MIN_BYTES = {thr}
import bench
sys.argv = ["bench.py", "--config", "{cfg}", "--dtype", "{dt}", "--no-cpu-baseline", "--steps", "50"]
bench.main()
'''


def main():
    cfg, dt, rounds = sys.argv[1], sys.argv[2], int(sys.argv[3])
    for r in range(rounds):
        for name, thr in (("1GiB", 1 << 30), ("64MiB", 64 << 20)):
            code = CHILD.format(pkg=REPO / "distributed-training-sandbox_amd", repo=REPO, thr=thr,
                                cfg=cfg, dt=dt)
            out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                                 timeout=300, cwd=REPO)
            line = [l for l in out.stdout.splitlines() if l.startswith("{")]
            if out.returncode != 0 or not line:
                print(name, "FAILED", out.returncode, out.stderr[-500:], flush=True)
                sys.exit(1)
            d = json.loads(line[0])
            print(f"round {r} {name:6s} step {d['ms_per_step']:.4f} ms  adam "
                  f"{d['roofline']['achieved']:.0f} GB/s  placement {d['placement']['state']}",
                  flush=True)


if __name__ == "__main__":
    main()
