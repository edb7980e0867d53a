"""Scores of a BASELINE config's rank-0 batch from the library build named by MSV_LIB_PATH (A/B builds:
tools/ab_build.sh), saved as raw float32 bits for a bitwise comparison between builds.

    MSV_LIB_PATH=abx/x/libmsv_hip.so python tools/lib_scores.py --config cfg2 --out gpurun_out/x.npy
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import homolog_batch, random_batch, concat_batches
    from bench import CONFIGS
    prof, n, lmin, lmax, seed, scaling = CONFIGS[a.config]
    h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof))
    codes, offsets = concat_batches(random_batch(seed * 1000 if scaling == "weak" else seed, n, lmin, lmax),
                                    homolog_batch(h.match_emissions, 7, 2000, lmin, lmax))
    sc = msv.MSV_HMM(h).score_batch(codes=codes, offsets=offsets)
    np.save(a.out, sc.view(np.uint32))
    print(a.out, len(sc))


if __name__ == "__main__":
    main()
