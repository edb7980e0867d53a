"""How often the Viterbi kernel's lazy-F correction runs (vit_kernel.hip), simulated in float32 numpy with the
kernel's lane layout (64 lanes x S states, each lane's D chain started from -inf, then passes
D_q = max(D_q, D_{q-1} + tDD_q) while some lane's incoming D beats its first D): passes per row, and the last
state each pass changes (what the early exit of the first pass relies on).  Random sequences, L U[300,500].

    python tools/lazy_f_stats.py [profile number] [seed] [sequences]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle_lib import OracleProfile
from hmm_fasta_viterbi_amd.synthetic import random_batch
prof = sys.argv[1] if len(sys.argv) > 1 else "1400"
o = OracleProfile(prof)
msc = o.emission_scores().astype(np.float32)     # [20][M]
_, tsc = o.vit_tables(0)                           # [M][7]: m->m m->i m->d i->m i->i d->m d->d
b, c, j = o.constants()
M = o.model_length; K = M - 1
S = -(-K // 64); S += S & 1
NI = np.float32(-np.inf)
k = np.arange(64)[:, None] * S + np.arange(S)[None, :] + 1   # state of (lane, slot)
valid = k <= K
def tin(col):   # transition from node k-1 into k
    t = np.full(k.shape, NI, np.float32); m = valid & (k >= 2); t[m] = tsc[k[m] - 1, col]; return t
def tout(col):
    t = np.full(k.shape, NI, np.float32); m = valid & (k < K); t[m] = tsc[k[m], col]; return t
tMM, tIM, tDM, tMD, tDD = tin(0), tin(3), tin(5), tin(2), tin(6)
tMI, tII = tout(1), tout(4)
E_tab = np.where(valid[None], msc[:, np.minimum(k, K)], NI).astype(np.float32)  # [20][64][S]
def shift(x):  # lane l-1's last slot into lane l; lane 0 -inf
    r = np.empty(64, np.float32); r[0] = NI; r[1:] = x[:-1, -1]; return r
codes, offsets = random_batch(int(sys.argv[2]) if len(sys.argv) > 2 else 5, int(sys.argv[3]) if len(sys.argv) > 3 else 20, 300, 500)
tot_rows = tot_iter = rows_with = 0; hist = {}
lastslot = []
for s in range(len(offsets) - 1):
    seq = codes[int(offsets[s]):int(offsets[s + 1])]; L = len(seq)
    loop = np.float32(np.log(np.float32(L) / np.float32(L + 3))); move = np.float32(np.log(np.float32(3) / np.float32(L + 3)))
    Mv = np.full((64, S), NI, np.float32); Iv = Mv.copy(); Dv = Mv.copy()
    N = np.float32(0); B = move; J = NI
    for r in seq:
        Bt = np.float32(B + np.float32(b))
        pm = np.concatenate([shift(Mv)[:, None], Mv[:, :-1]], 1); pi = np.concatenate([shift(Iv)[:, None], Iv[:, :-1]], 1)
        pd = np.concatenate([shift(Dv)[:, None], Dv[:, :-1]], 1)
        Mn = np.maximum(np.maximum(np.maximum(pm + tMM, pi + tIM), pd + tDM), Bt) + E_tab[r]
        In = np.maximum(Mv + tMI, Iv + tII)
        Dn = np.empty_like(Mv)
        mprev = np.concatenate([shift(Mn)[:, None], Mn[:, :-1]], 1)
        Dn[:, 0] = mprev[:, 0] + tMD[:, 0]
        for q in range(1, S): Dn[:, q] = np.maximum(mprev[:, q] + tMD[:, q], Dn[:, q - 1] + tDD[:, q])
        it = 0
        cand = shift(Dn) + tDD[:, 0]
        while np.any(cand > Dn[:, 0]):
            it += 1; old = Dn.copy()
            Dn[:, 0] = np.maximum(Dn[:, 0], cand)
            for q in range(1, S): Dn[:, q] = np.maximum(Dn[:, q], Dn[:, q - 1] + tDD[:, q])
            ch = np.nonzero(np.any(Dn != old, axis=0))[0]
            lastslot.append(int(ch.max()) if len(ch) else -1)
            cand = shift(Dn) + tDD[:, 0]
        tot_rows += 1; tot_iter += it; rows_with += it > 0; hist[it] = hist.get(it, 0) + 1
        Mv, Iv, Dv = Mn, In, Dn
        E = Mn.max(); J = max(np.float32(J + loop), np.float32(E + np.float32(j))); N = np.float32(N + loop)
        B = np.float32(max(N, J) + move)
print(prof, "S", S, "rows", tot_rows, "lazy-F passes per row", round(tot_iter / tot_rows, 3), "rows with any", round(rows_with / tot_rows, 3), "hist", sorted(hist.items())[:10])
ls = np.array(lastslot); print("last changed slot per pass: median", np.median(ls), "p90", np.percentile(ls, 90), "max", ls.max(), "frac <=3", np.mean(ls <= 3), "<=7", np.mean(ls <= 7))
