"""Interleaved A/B of library builds on the kernel alone (tools/run_kernel.py --time in a fresh
process per measurement, builds alternating; cdna_hip_programming.md §5.4 rule 24).

    python tools/kernel_ab.py --config cfg3 --rounds 4 ab/base/libmsv_hip.so ab/new/libmsv_hip.so
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--warm", type=int, default=15)
    ap.add_argument("--time", type=int, default=20)
    ap.add_argument("--profile", default="")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, MSV_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "run_kernel.py"), "--config", a.config,
                                  "--launches", str(a.warm), "--time", str(a.time)]
                                 + (["--profile", a.profile] if a.profile else []) + (["--n", str(a.n)] if a.n else []), env=env, capture_output=True,
                                 text=True, timeout=240, check=True).stdout.strip().splitlines()[-1]
            d = json.loads(out)
            d["round"] = r
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
