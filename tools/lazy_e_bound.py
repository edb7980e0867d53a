"""How often could a row skip the E reduction?  (CPU only, not product code.)

The MSV row (MSV_HMM.cpp:100-110) needs E = max_k M[k] only through J = max(J + loop, E + tEJ) and
C = max(C + loop, E + tEC).  Float rounding is monotone, so UB_t = max(UB_{t-1}, Bt) + max_k e[r_t][k]
bounds E_t from above; when fl(UB_t + tEJ) <= fl(J + loop) the row's J (and C, tEC == tEJ) equal
J + loop exactly and E is not needed.  This replays the float32 recurrence on random sequences and reports
the fraction of rows where the test passes, per sequence and for a wave of 4 sequences (16-lane groups:
all 4 must pass, rows aligned by index).
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import hmm_fasta_viterbi_amd as msv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--profile", default="1400.hmm")
ap.add_argument("--sequences", type=int, default=40)
args = ap.parse_args()
f32 = np.float32
prof = msv.Profile_HMM(os.path.join(os.path.dirname(__file__), "..", "data", "profile_HMMs", args.profile))
es, b, c, j = prof.msv_scores()
es = np.asarray(es, f32).reshape(20, -1)[:, 1:]  # [residue][state 1..M] (node 0 is the dummy)
emax = es.max(axis=1)
rng = np.random.default_rng(0)
per_seq = []
for _ in range(args.sequences):
    L = int(rng.integers(300, 501))
    seq = rng.integers(0, 20, L)
    loop, move = (f32(x) for x in msv.sequence_transitions(L))
    M = np.full(es.shape[1], -np.inf, f32)
    J, N, B, UB = f32(-np.inf), f32(0), move, f32(-np.inf)
    skips = np.zeros(L, bool)
    for t in range(L):
        r = seq[t]
        Bt = f32(B + f32(b))
        prev = np.concatenate([[f32(-np.inf)], M[:-1]])
        M = (np.maximum(prev, Bt) + es[r]).astype(f32)
        E = M.max()
        ub = f32(max(UB, Bt) + emax[r])
        skips[t] = f32(ub + f32(j)) <= f32(J + loop)
        UB = ub if skips[t] else E
        J = max(f32(J + loop), f32(E + f32(j)))
        N = f32(N + loop)
        B = f32(max(N, J) + move)
    per_seq.append(skips)
one = float(np.mean([s.mean() for s in per_seq]))
waves = []
for w in range(0, len(per_seq) - 3, 4):
    n = min(len(s) for s in per_seq[w:w + 4])
    waves.append(np.logical_and.reduce([s[:n] for s in per_seq[w:w + 4]]).mean())
print({"profile": args.profile, "sequences": args.sequences, "skip_fraction_per_sequence": round(one, 4),
       "skip_fraction_wave_of_4": round(float(np.mean(waves)), 4)})
