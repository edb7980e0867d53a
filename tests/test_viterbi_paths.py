"""The Viterbi stage's restatements (oracle/msv_oracle.c, and the library's own CPU DP msv_vit_cpu_score, which the
GPU equals bit for bit) against an INDEPENDENT FORMULATION of the model: every state path through HMMER3's
multihit local model with the MSV path's specials, enumerated explicitly on tiny models and sequences, scored
left to right in float32, and the best one taken -- no dynamic programming, no matrices.

This pins what the DP cannot pin against itself: which node's transition each step reads (m->m of node k takes
M_k to M_k+1, i->m of node k takes I_k to M_k+1, d->m / d->d likewise, m->i and i->i stay on node k), that there is
no I at node LENG, that D states are silent and cannot exit, that E is entered from M only, and the order of the
specials (N loops, B = max(N, J) + move, J / C loops, C(L) + move; MSV_HMM.cpp:100-112).  Bitwise, because fl() is
monotone: the DP's value is the max over paths of each path's left-to-right fl-sum.

VERDICT r05 (weak 1) notes the stage's transition terms have no external pin; HMMER/pyhmmer remain absent, so
this is still "parity unpinned" against HMMER itself -- but an off-by-one node index, a transition of the wrong
kind or a wrong special would fail here, whereas the MSV reduction and the calibration tests could miss it."""
import numpy as np
import pytest

import hmm_fasta_viterbi_amd as msv
from hmm_fasta_viterbi_amd import _native
from oracle_lib import bits, vit_score_tables

F = np.float32
NINF = F(-np.inf)
MM, MI, MD, IM, II, DM, DD = range(7)


def random_model(rng, leng, informative_inserts):
    """Tables as the library takes them: msc / isc [20][LENG+1] (column 0 unused), tsc [LENG+1][7] log-probabilities
    per node (m->{m,i,d}, i->{m,i}, d->{m,d} each summing to 1)."""
    M = leng + 1
    msc = rng.normal(0.0, 1.5, (20, M)).astype(F)
    msc[:, 0] = NINF
    isc = rng.normal(0.0, 0.7, (20, M)).astype(F) if informative_inserts else None
    tsc = np.zeros((M, 7), F)
    for k in range(M):
        m = rng.dirichlet([2.0, 1.0, 1.0])
        i = rng.dirichlet([1.0, 1.0])
        d = rng.dirichlet([1.0, 1.0])
        tsc[k] = np.log(np.array([m[0], m[1], m[2], i[0], i[1], d[0], d[1]], F)).astype(F)
    tBM = F(np.log(F(2.0) / F(M * (M + 1))))  # MSV_HMM.cpp:51's entry, M = LENG + 1
    half = F(np.log(F(0.5)))
    return msc, isc, tsc, (tBM, half, half)


def best_path(msc, isc, tsc, consts, codes):
    """Max over every state path of its float32 left-to-right score (-inf when no path exists)."""
    tBM, tEC, tEJ = (F(x) for x in consts)
    leng = msc.shape[1] - 1
    L = len(codes)
    loop, move = (F(x) for x in msv.sequence_transitions(L))
    best = [NINF]

    def em(k, pos):   # match emission of residue `pos` (1-based) at node k
        return F(msc[codes[pos - 1], k])

    def ei(k, pos):
        return F(0.0) if isc is None else F(isc[codes[pos - 1], k])

    def m_state(pos, k, s):          # s: the score entering M_k (transition added); M_k emits residue pos
        s = F(s + em(k, pos))
        e_state(pos, s)              # local exit M_k -> E (no cost)
        if k < leng:                 # transitions out of node k exist for k = 1 .. LENG-1 only
            if pos < L:
                m_state(pos + 1, k + 1, F(s + tsc[k, MM]))
                i_state(pos + 1, k, F(s + tsc[k, MI]))
            d_state(pos, k + 1, F(s + tsc[k, MD]))   # silent

    def i_state(pos, k, s):          # I_k (k <= LENG-1) emits residue pos
        s = F(s + ei(k, pos))
        if pos < L:
            i_state(pos + 1, k, F(s + tsc[k, II]))
            m_state(pos + 1, k + 1, F(s + tsc[k, IM]))  # k + 1 <= LENG always

    def d_state(pos, k, s):          # D_k at row pos, silent; no exit from D
        if k < leng:
            d_state(pos, k + 1, F(s + tsc[k, DD]))
            if pos < L:
                m_state(pos + 1, k + 1, F(s + tsc[k, DM]))

    def enter(pos, b):               # B at row pos -> M_k emits residue pos + 1
        if pos < L:
            bt = F(b + tBM)
            for k in range(1, leng + 1):
                m_state(pos + 1, k, bt)

    def e_state(pos, s):             # E at row pos
        c = F(s + tEC)               # E -> C, C loops over the rest, then C(L) + move
        for _ in range(L - pos):
            c = F(c + loop)
        best[0] = max(best[0], F(c + move))
        j = F(s + tEJ)               # E -> J, J loops m times, then B -> another pass through the model
        for m in range(0, L - pos):
            enter(pos + m, F(j + move))
            j = F(j + loop)

    n = F(0.0)                       # N(0) = 0; N loops, then B = N + move
    for pos in range(0, L):
        enter(pos, F(n + move))
        n = F(n + loop)
    return best[0]


def lib_cpu(msc, isc, tsc, consts, codes):
    import ctypes as C
    out = C.c_float()
    c = np.ascontiguousarray(codes, np.uint8)
    st = _native.lib().msv_vit_cpu_score(msc.ctypes.data, None if isc is None else isc.ctypes.data, tsc.ctypes.data,
                                         msc.shape[1], *[float(x) for x in consts],
                                         c.ctypes.data if c.size else None, len(c), C.byref(out))
    assert st == 0
    return F(out.value)


@pytest.mark.parametrize("leng", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("inserts", [False, True])
def test_dp_equals_the_best_explicit_path(leng, inserts):
    rng = np.random.Generator(np.random.PCG64(1000 * leng + inserts))
    for trial in range(6):
        msc, isc, tsc, consts = random_model(rng, leng, inserts)
        if trial == 5:  # distinct exits: C and J no longer coincide
            consts = (consts[0], F(consts[1] - F(0.75)), consts[2])
        seqs = [rng.integers(0, 20, L, dtype=np.uint8) for L in (0, 1, 2, 3, 4, 4, 5)]
        offsets = np.zeros(len(seqs) + 1, np.uint64)
        np.cumsum([len(s) for s in seqs], out=offsets[1:])
        oracle = vit_score_tables(msc, isc, tsc, consts, np.concatenate(seqs), offsets)
        for q, codes in enumerate(seqs):
            want = best_path(msc, isc, tsc, consts, codes)
            assert bits(oracle[q]) == bits(want), (leng, inserts, trial, q, oracle[q], want)
            assert bits(lib_cpu(msc, isc, tsc, consts, codes)) == bits(want), (leng, inserts, trial, q)


def test_every_transition_kind_reaches_the_best_path():
    """The enumeration is not vacuous: on these models the best paths use inserts, deletes and J re-entries, so
    each transition kind is exercised by at least one compared score."""
    rng = np.random.Generator(np.random.PCG64(7))
    used = set()
    for trial in range(40):
        msc, isc, tsc, consts = random_model(rng, 3, True)
        for L in (3, 4, 5):
            codes = rng.integers(0, 20, L, dtype=np.uint8)
            ref = best_path(msc, isc, tsc, consts, codes)
            for kind in range(7):  # a kind is used by the optimum iff forbidding it changes the best score
                t2 = tsc.copy()
                t2[:, kind] = NINF
                if bits(best_path(msc, isc, t2, consts, codes)) != bits(ref):
                    used.add(kind)
    # d->d: a model whose best path for "a b" must run M1 -> D2 -> D3 -> M4 (M1 and M4 alone score well)
    msc, isc, tsc, consts = random_model(np.random.Generator(np.random.PCG64(8)), 5, False)
    msc[:, 1:] = F(-5.0)
    msc[0, 1] = msc[1, 4] = F(5.0)
    codes = np.array([0, 1], np.uint8)
    ref = best_path(msc, isc, tsc, consts, codes)
    t2 = tsc.copy()
    t2[:, DD] = NINF
    if bits(best_path(msc, isc, t2, consts, codes)) != bits(ref):
        used.add(DD)
    assert bits(vit_score_tables(msc, isc, tsc, consts, codes, np.array([0, 2], np.uint64))[0]) == bits(ref)
    assert used == set(range(7)), sorted(used)


@pytest.mark.gpu
def test_gpu_equals_the_best_explicit_path():
    """The device kernels on the same tiny models (msv_vit_profile_create over the tables: the picks for the
    smallest S, padding states -inf) against the explicit-path optimum, bitwise."""
    import ctypes as C
    L_ = _native.lib()
    rng = np.random.Generator(np.random.PCG64(99))
    for leng in (1, 2, 3, 4, 5):
        for inserts in (False, True):
            msc, isc, tsc, consts = random_model(rng, leng, inserts)
            p = C.c_void_p()
            assert L_.msv_vit_profile_create(0, msc.ctypes.data, None if isc is None else isc.ctypes.data,
                                             tsc.ctypes.data, leng + 1, *[float(x) for x in consts], C.byref(p)) == 0
            try:
                seqs = [rng.integers(0, 20, L, dtype=np.uint8) for L in (0, 1, 2, 3, 4, 5, 5, 5)]
                offsets = np.zeros(len(seqs) + 1, np.uint64)
                np.cumsum([len(s) for s in seqs], out=offsets[1:])
                codes = np.concatenate(seqs)
                out = np.zeros(len(seqs), np.float32)
                assert L_.msv_vit_score_batch(p, codes.ctypes.data, offsets.ctypes.data, len(seqs), out.ctypes.data,
                                              None) == 0
                want = np.array([best_path(msc, isc, tsc, consts, s) for s in seqs], np.float32)
                assert np.array_equal(bits(out), bits(want)), (leng, inserts, out, want)
            finally:
                L_.msv_vit_profile_destroy(p)
