"""MSV P-values against the calibration HMMER3 stored in every profile (STATS LOCAL MSV mu, lambda):
score N iid background sequences of length 200 on the GPU (what p7_MSVMu scores to fit mu), refit mu to
our bit scores with lambda fixed, and report the tail fractions of our P-values (uniform if the pipeline
matches the calibration).  One JSON line per profile.

    python tools/pvalue_calibration.py [--n 20000]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process)
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import background_batch

    profs = sorted((f for f in os.listdir(os.path.join(ROOT, "data", "profile_HMMs")) if f.endswith(".hmm")),
                   key=lambda f: int(f.split(".")[0]))
    codes, offsets = background_batch(2024, a.n, 200)
    for p in profs:
        h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", p))
        e = msv.MSV_HMM(h)
        sc = e.score_batch(codes=codes, offsets=offsets)
        pv = e.pvalues(sc, offsets)
        mu, lam = e.msv_mu, e.msv_lambda
        bits = mu - np.log(-np.log1p(-pv)) / lam
        mu_fit = float(-np.log(np.mean(np.exp(-lam * bits))) / lam)
        print(json.dumps({"profile": p, "mu_file": mu, "lambda_file": lam, "mu_fit": round(mu_fit, 4),
                          "mu_fit_minus_file_bits": round(mu_fit - mu, 4),
                          "frac_p_lt": {str(t): float(np.mean(pv < t)) for t in (0.5, 0.1, 0.01, 0.001)}}),
              flush=True)
        e.close()


if __name__ == "__main__":
    main()
