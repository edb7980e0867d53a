"""Interleaved A/B of library builds on the Viterbi stage: tools/vit_tune.py in a fresh process per
measurement (MSV_LIB_PATH = each build in turn), rounds alternating, one JSON line per (round, build).

    python tools/vit_ab.py --config cfg3 --variant vit_s22_t5a --rounds 3 abx/base/libmsv_hip.so abx/new/libmsv_hip.so
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
    ap.add_argument("--variant", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=0, help="random 1400.hmm-style batch of n sequences instead of --config")
    ap.add_argument("--profile", default="1400.hmm")
    ap.add_argument("--lmin", type=int, default=300)
    ap.add_argument("--lmax", type=int, default=500)
    ap.add_argument("--in-place", action="store_true", help="bench.py's setting (vit_tune.py --in-place)")
    ap.add_argument("--config-n", type=int, default=0, help="the config's first N sequences (vit_tune.py)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, MSV_LIB_PATH=os.path.abspath(lib))
            batch = (["--profile", a.profile, "--n", str(a.n), "--lmin", str(a.lmin), "--lmax", str(a.lmax)] if a.n
                     else ["--config", a.config] + (["--config-n", str(a.config_n)] if a.config_n else []))
            order = ["--in-place"] if a.in_place else ["--longest-first"]
            out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "vit_tune.py"), *batch, *order,
                                  "--rounds", "1", "--reps", "5", "--variants", a.variant],
                                 env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                sys.exit(out.stderr[-2000:])
            d = json.loads(out.stdout.strip().splitlines()[-1])
            print(json.dumps({"round": r, "lib": lib, "config": None if a.n else a.config, "n": d["sequences"],
                              "profile": d["profile"], "variant": a.variant,
                              "ms_med": d["ms_med"], "valu_frac": d["valu_frac"]}), flush=True)


if __name__ == "__main__":
    main()
