"""The MSV filter and the Viterbi stage against their calibration (STATS LOCAL MSV / VITERBI) at the lengths
the bench uses, for both input compositions.  HMMER3 fits both mus on iid *background*
sequences of length 200; the bench's synthetic batches are uniform over the 20 letters
(random_FASTA_generator.py's format).  For every profile, length L in --lengths and composition in
{background, uniform}: N sequences scored on the GPU (MSV: msv_score_batch, Viterbi: msv_vit_score_batch),
P-values against the file's mu/lambda, tail fractions and the mu refitted with lambda fixed.  One JSON line
per (profile, L, composition, stage).

    python tools/filter_drift.py --out profiles/r05_filter_length_composition.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def uniform_batch(seed, n, length):
    rng = np.random.Generator(np.random.PCG64(seed))
    codes = rng.integers(0, 20, n * length).astype(np.uint8)
    return codes, np.arange(0, n * length + 1, length, dtype=np.uint64)


def fit(pv, mu, lam):
    b = mu - np.log(-np.log1p(-pv)) / lam
    mu_fit = -np.log(np.mean(np.exp(-lam * b))) / lam
    return {"refit_minus_file_bits": round(float(mu_fit - mu), 4),
            **{f"p_lt_{t}": round(float(np.mean(pv < t)), 5) for t in (0.5, 0.1, 0.02, 0.01)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lengths", default="200,400,2000")
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--profiles", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process)
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import background_batch

    profs = a.profiles.split(",") if a.profiles else sorted(
        (f for f in os.listdir(os.path.join(ROOT, "data", "profile_HMMs")) if f.endswith(".hmm")),
        key=lambda f: int(f.split(".")[0]))
    out = open(a.out, "w") if a.out else None
    batches = {}
    for L in (int(x) for x in a.lengths.split(",")):
        n = a.n if L <= 400 else max(1000, a.n // 4)
        batches[(L, "background")] = background_batch(2024 + L, n, L)
        batches[(L, "uniform")] = uniform_batch(2024 + L, n, L)
    for p in profs:
        h = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", p))
        m, v = msv.MSV_HMM(h), msv.Viterbi_HMM(h)
        for (L, comp), (codes, offsets) in batches.items():
            for stage, eng, mu, lam in (("msv", m, m.msv_mu, m.msv_lambda),
                                        ("viterbi", v, v.viterbi_mu, v.viterbi_lambda)):
                pv = eng.pvalues(eng.score_batch(codes=codes, offsets=offsets), offsets)
                line = {"profile": p, "length": L, "composition": comp, "stage": stage, "n": len(offsets) - 1,
                        **fit(pv, mu, lam)}
                print(json.dumps(line), flush=True)
                if out:
                    out.write(json.dumps(line) + "\n")
        m.close()
    if out:
        out.close()


if __name__ == "__main__":
    main()
