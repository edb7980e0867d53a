"""The reference's own benchmark programs, on this engine (informational; BASELINE.md: the reference
publishes no numbers and its OpenCL path does not run here).

    python tools/bench_reference_programs.py

  benchmark_MSV_1400  1400.hmm x FASTA_files/random_FASTA.fsa (3 x 3500 residues), best of 2
                      (algorithms/benchmark_MSV_1400.cpp:5-15, benchmark_helper.hpp:9-38): the per-sequence
                      call parallel_run_on_sequence timed per sequence and summed, as the reference does;
                      also the whole file as one score_batch launch.
  benchmark_MSV       every profile x random_FASTA.fsa (algorithms/benchmark_MSV.cpp:12-41): summed
                      per-profile best times, and the whole grid as one score_grid call.
GPU only (the reference CPU path is timed beside the headline metric by bench.py's cpu_baseline).
Scores are checked bitwise against the reference's golden values (tests/golden/random_fasta_scores.tsv).
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# score_grid forks one launch per profile onto the profiles' own streams; HIP's default of 4 hardware
# queues runs at most 4 of the 24 small launches at once (as bench.py, raise it before HIP starts).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
PROFILES = sorted((f for f in os.listdir(os.path.join(ROOT, "data", "profile_HMMs")) if f.endswith(".hmm")),
                  key=lambda f: int(f.split(".")[0]))


def read_golden_tsv(name):
    """Rows (profile, index, length, score) of a committed golden file (data, written by the reference)."""
    rows = []
    with open(os.path.join(ROOT, "tests", "golden", name)) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            prof, idx, L, hx, _ = line.rstrip("\n").split("\t")
            rows.append((prof, int(idx), int(L), np.float32(float.fromhex(hx))))
    return rows


def best_of(fn, n=2):
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    import torch  # noqa: F401  (one HIP runtime per process)
    import hmm_fasta_viterbi_amd as msv

    fasta_path = os.path.join(ROOT, "data", "FASTA_files", "random_FASTA.fsa")
    fa = msv.FASTA_protein_sequences(fasta_path)
    golden = read_golden_tsv("random_fasta_scores.tsv")
    engines = {p: msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", p))) for p in PROFILES}
    for e in engines.values():  # warm: table upload, first launch
        e.score_batch(fa.sequences)

    def per_sequence(e):
        return lambda: [e.parallel_run_on_sequence(s) for s in fa.sequences]

    ok = True
    for p in PROFILES:
        want = np.array([w for q, i, L, w in golden if q == p], np.float32)
        ok &= bool(np.array_equal(engines[p].score_batch(fa.sequences).view(np.uint32), want.view(np.uint32)))

    e1400 = engines["1400.hmm"]
    res = {
        "fasta": "random_FASTA.fsa (3 x 3500 residues)",
        "bitwise_equal_to_reference_golden": ok,
        "benchmark_MSV_1400": {
            "gpu_per_sequence_ms": round(best_of(per_sequence(e1400)) * 1e3, 3),
            "gpu_one_batch_ms": round(best_of(lambda: e1400.score_batch(fa.sequences)) * 1e3, 3),
        },
        "benchmark_MSV": {
            "gpu_per_sequence_sum_ms": round(sum(best_of(per_sequence(engines[p])) for p in PROFILES) * 1e3, 3),
            "gpu_per_profile_batch_sum_ms": round(
                sum(best_of(lambda e=engines[p]: e.score_batch(fa.sequences)) for p in PROFILES) * 1e3, 3),
            "gpu_grid_ms": round(best_of(lambda: msv.score_grid(list(engines.values()), fa.sequences)) * 1e3, 3),
        },
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
