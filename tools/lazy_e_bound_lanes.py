"""Round 6: the lazy-E bound of DESIGN 7 item 1, per LANE instead of per sequence.  Each lane of a G-lane
group bounds its own states' M by U_t = emax_lane[r_t] + max(U_{t-1}, M_left(t-1), Bt), where M_left is the
exact M of the left lane's last state that the row already shifts in.  Rounding is monotone, so U_t >= the
lane's exact E_t.  A wave of 4 sequences skips its E max on a row only if every lane passes.
Usage: python tools/lazy_e_bound_lanes.py [profile] [G]"""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
import hmm_fasta_viterbi_amd as msv
from hmm_fasta_viterbi_amd.synthetic import random_batch
F = np.float32
prof = sys.argv[1] if len(sys.argv) > 1 else '1400.hmm'
G = int(sys.argv[2]) if len(sys.argv) > 2 else 16
h = msv.Profile_HMM('/root/repo/data/profile_HMMs/' + prof)
es, tBM, tEC, tEJ = h.msv_scores()          # es [20, Mcols]
Mcols = es.shape[1]; K = Mcols - 1            # states 1..K
S = -(-K // G)
pad = G * S - K
E20 = np.full((20, G * S), -np.inf, F); E20[:, :K] = es[:, 1:]
emax = E20.reshape(20, G, S).max(axis=2)      # [20, G]
codes, offs = random_batch(2, 4 * 400, 300, 500)
nseq = len(offs) - 1
waves = nseq // 4
rows_total = trig_rows = ev_rows = 0
for w in range(waves):
    seqs = [codes[offs[4*w+g]:offs[4*w+g+1]] for g in range(4)]
    Ls = [len(s) for s in seqs]; Lmax = max(Ls)
    st = []
    for s in seqs:
        L = len(s); loop, move = (F(x) for x in msv.sequence_transitions(L))
        st.append(dict(M=np.full(G*S, -np.inf, F), J=F(-np.inf), N=F(0), B=move, loop=loop, move=move,
                       U=np.full(G, -np.inf, F), s=s, L=L))
    for i in range(Lmax):
        trig = False; ev = False
        for d in st:
            if i >= d['L']: continue
            r = d['s'][i]
            Bt = F(d['B'] + F(tBM))
            prevM = d['M']
            sh = np.concatenate([[F(-np.inf)], prevM[:-1]]).astype(F)
            M = (E20[r] + np.maximum(sh, Bt)).astype(F)
            # bound
            lastprev = prevM.reshape(G, S)[:, -1]
            left = np.concatenate([[F(-np.inf)], lastprev[:-1]]).astype(F)
            U = (emax[r] + np.maximum(np.maximum(d['U'], left), Bt)).astype(F)
            Elane = M.reshape(G, S).max(axis=1)
            assert np.all(U >= Elane)
            T = F(d['J'] + d['loop'])
            d['need'] = np.any(U + F(tEJ) > T)
            d['Mnew'], d['Unew'], d['Elane'] = M, U, Elane
            trig |= d['need']
            E = Elane.max()
            ev |= bool(E + F(tEJ) > T)
        rows_total += 1; trig_rows += trig; ev_rows += ev
        for d in st:
            if i >= d['L']: continue
            d['M'] = d['Mnew']
            d['U'] = d['Elane'] if trig else d['Unew']
            E = d['Elane'].max()
            d['J'] = max(F(d['J'] + d['loop']), F(E + F(tEJ)))
            d['N'] = F(d['N'] + d['loop'])
            d['B'] = F(max(d['N'], d['J']) + d['move'])
print(prof, 'G', G, 'S', S, 'rows', rows_total, 'triggered frac', trig_rows / rows_total, 'event frac', ev_rows / rows_total,
      'emax mean', float(emax.mean()), 'tBM', tBM)
