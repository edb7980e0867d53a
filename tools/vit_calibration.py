"""Statistical pin of the Viterbi stage against the calibration HMMER3 stored in every profile:
HMMER fits STATS LOCAL VITERBI mu (lambda fixed) to the Viterbi bit scores of iid background sequences of
length 200 (p7_ViterbiMu).  For each profile: score N such sequences (seed 2024), P-values against the file's
mu/lambda (msv_pvalues), the refitted mu (ML with lambda fixed) and tail fractions; the MSV stage beside it
(STATS LOCAL MSV) for comparison.  Scores come from the serial restatement (oracle_vit_run_codes, bitwise
equal to the kernel: tests/test_gpu_viterbi.py); the GPU test repeats the fit on the kernel's scores.

    python tools/vit_calibration.py --n 20000 --out profiles/r04_vit_calibration.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def fit(scores, offsets, mu, lam):
    from hmm_fasta_viterbi_amd import _native
    pv = np.zeros(len(scores), np.float64)
    assert _native.lib().msv_pvalues(scores.ctypes.data, offsets.ctypes.data, len(scores), mu, lam,
                                     pv.ctypes.data) == 0
    b = mu - np.log(-np.log1p(-pv)) / lam
    mu_fit = -np.log(np.mean(np.exp(-lam * b))) / lam
    return {"file_mu": round(float(mu), 4), "refit_mu": round(float(mu_fit), 4),
            "refit_minus_file_bits": round(float(mu_fit - mu), 4),
            "p_lt_0.5": round(float(np.mean(pv < 0.5)), 4), "p_lt_0.1": round(float(np.mean(pv < 0.1)), 4),
            "p_lt_0.01": round(float(np.mean(pv < 0.01)), 5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import background_batch
    from oracle_lib import PROFILES, OracleProfile, profile_path
    codes, offsets = background_batch(2024, a.n, 200)
    lines = []
    for prof in PROFILES:
        o = OracleProfile(prof)
        h = msv.Profile_HMM(profile_path(prof))
        vit = o.vit_score_batch(codes, offsets, 0, threads=a.threads)
        ms = o.score_batch(codes, offsets, threads=a.threads)
        d = {"profile": prof, "sequences": a.n, "length": 200, "seed": 2024, "scores": "oracle_vit_run_codes",
             "viterbi": fit(vit, offsets, h.stats_local_viterbi_mu, h.stats_local_viterbi_lambda),
             "msv": fit(ms, offsets, h.stats_local_msv_mu, h.stats_local_msv_lambda)}
        lines.append(json.dumps(d))
        print(lines[-1], flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
