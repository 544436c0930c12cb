"""Run bench.py in this process with zero_amd's diagnostic zs_tune knobs set first (A/B of the
library's defaults, e.g. the stream-flag record / wait kernels).

Usage: python tools/tune_run.py sync_wait_kernel=1 sync_write_fence=0 -- <bench.py arguments>
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "distributed-training-sandbox_amd"))
sys.path.insert(0, str(REPO))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    knobs, rest = argv[:cut], argv[cut + 1:]
    import torch  # noqa: F401  (the library binds to torch's HIP runtime)

    from zero_amd import _lib

    for kv in knobs:
        k, v = kv.split("=")
        _lib.call("zs_tune", k.encode(), int(v), None)
        print(f"[tune_run] {k} = {v}", file=sys.stderr, flush=True)
    import bench

    bench.main(rest)


if __name__ == "__main__":
    main()
