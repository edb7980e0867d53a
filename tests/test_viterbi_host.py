"""Viterbi stage on the CPU: the oracle's serial restatement (oracle/msv_oracle.c,
oracle_vit_run_codes) and the library's own CPU DP (msv_vit_cpu_score) pinned against

  * an independent pure-Python restatement of HMMER3's generic local Viterbi (p7_GViterbi's recurrence,
    float32 arithmetic, full (L+1) x (K+1) matrices) on small cases -- bitwise;
  * the reference's OWN golden MSV scores: with m->m = 1 and every other transition impossible, the
    Viterbi recurrence IS the MSV recurrence (MSV_HMM.cpp:100-111), so the stage must reproduce
    tests/golden/example_scores.tsv (the reference build's output) bit for bit;
  * the calibration HMMER3 stored in the reference's profiles (STATS LOCAL VITERBI) -- statistically.

There is no reference implementation of the stage and HMMER/pyhmmer are absent: beyond the MSV reduction,
parity is "unpinned" (DESIGN.md 4.6)."""
import ctypes as C
import os

import numpy as np
import pytest

import hmm_fasta_viterbi_amd as msv
from hmm_fasta_viterbi_amd import _native
from hmm_fasta_viterbi_amd.synthetic import background_batch, gapped_homolog_batch, homolog_batch, random_batch
from oracle_lib import PROFILES, ROOT, OracleProfile, bits, profile_path, read_golden_tsv, vit_score_tables

F = np.float32
NINF = F(-np.inf)


def py_viterbi(msc, isc, tsc, consts, codes):
    """HMMER3 generic Viterbi written from the published recurrence, float32 scalar ops, full matrices
    (an implementation independent of both C restatements: different loop structure and storage)."""
    tBM, tEC, tEJ = (F(x) for x in consts)
    M = msc.shape[1]
    K = M - 1
    L = len(codes)
    loop, move = (F(x) for x in msv.sequence_transitions(L))  # glibc logf, MSV_HMM.cpp:59-64
    MM, MI, MD, IM, II, DM, DD = range(7)

    def t(k, x):
        return NINF if k == 0 else F(tsc[k, x])

    Mx = [[NINF] * (K + 1) for _ in range(L + 1)]
    Ix = [[NINF] * (K + 1) for _ in range(L + 1)]
    Dx = [[NINF] * (K + 1) for _ in range(L + 1)]
    N, B, J, Cs = F(0), move, NINF, NINF
    for i in range(1, L + 1):
        r = int(codes[i - 1])
        E = NINF
        for k in range(1, K + 1):
            sc = max(F(Mx[i - 1][k - 1] + t(k - 1, MM)), F(Ix[i - 1][k - 1] + t(k - 1, IM)),
                     F(Dx[i - 1][k - 1] + t(k - 1, DM)), F(B + tBM))
            Mx[i][k] = F(sc + F(msc[r, k]))
            Ix[i][k] = (F(max(F(Mx[i - 1][k] + t(k, MI)), F(Ix[i - 1][k] + t(k, II))) + F(isc[r, k]))
                        if k < K else NINF)
            Dx[i][k] = max(F(Mx[i][k - 1] + t(k - 1, MD)), F(Dx[i][k - 1] + t(k - 1, DD)))
            E = max(E, Mx[i][k])
        E = max(E, Dx[i][K])
        J = max(F(J + loop), F(E + tEJ))
        Cs = max(F(Cs + loop), F(E + tEC))
        N = F(N + loop)
        B = max(F(N + move), F(J + move))
    return F(Cs + move)


def lib_tables(prof, insert_mode=0):
    h = msv.Profile_HMM(profile_path(prof))
    M = h.model_length
    msc = np.zeros((20, M), F)
    isc = np.zeros((20, M), F)
    tsc = np.zeros((M, 7), F)
    b, c, j = C.c_float(), C.c_float(), C.c_float()
    assert _native.lib().msv_hmm_viterbi_scores(h._h, insert_mode, msc.ctypes.data, isc.ctypes.data,
                                                tsc.ctypes.data, C.byref(b), C.byref(c), C.byref(j)) == 0
    return msc, isc, tsc, (b.value, c.value, j.value), h


def lib_cpu_scores(msc, isc, tsc, consts, codes, offsets):
    out = np.zeros(len(offsets) - 1, F)
    for s in range(len(offsets) - 1):
        seg = np.ascontiguousarray(codes[int(offsets[s]):int(offsets[s + 1])])
        r = C.c_float()
        assert _native.lib().msv_vit_cpu_score(msc.ctypes.data, None if isc is None else isc.ctypes.data,
                                               tsc.ctypes.data, msc.shape[1], *consts,
                                               seg.ctypes.data if seg.size else None, seg.size, C.byref(r)) == 0
        out[s] = r.value
    return out


@pytest.mark.parametrize("insert_mode", [0, 1])
def test_library_tables_equal_oracle_tables(insert_mode):
    """msv_hmm_viterbi_scores (the product's table builder) = the oracle's tables, bitwise, 24 profiles."""
    for prof in PROFILES:
        msc, isc, tsc, consts, _ = lib_tables(prof, insert_mode)
        o = OracleProfile(prof)
        oi, ot = o.vit_tables(insert_mode)
        assert np.array_equal(bits(msc), bits(o.emission_scores())), prof
        assert np.array_equal(bits(isc), bits(oi)), prof
        assert np.array_equal(bits(tsc), bits(ot)), prof
        assert [bits(x) for x in consts] == [bits(x) for x in o.constants()]


@pytest.mark.parametrize("prof,insert_mode", [("100.hmm", 0), ("100.hmm", 1), ("200.hmm", 0), ("1301.hmm", 0)])
def test_oracle_equals_independent_python_restatement(prof, insert_mode):
    """Small cases through the pure-Python recurrence: random, ungapped and gapped homologs, edge lengths."""
    o = OracleProfile(prof)
    msc = o.emission_scores()
    isc, tsc = o.vit_tables(insert_mode)
    me, _, _ = o.arrays()
    consts = o.constants()
    batches = [random_batch(5, 6, 0, 12), homolog_batch(me, 6, 3, 20, 40), gapped_homolog_batch(me, 7, 3, 25, 45)]
    for codes, offsets in batches:
        want = o.vit_score_batch(codes, offsets, insert_mode)
        for s in range(len(offsets) - 1):
            got = py_viterbi(msc, isc, tsc, consts, codes[int(offsets[s]):int(offsets[s + 1])])
            assert bits(got) == bits(want[s]), (prof, s, got, want[s])


@pytest.mark.parametrize("prof", ["100.hmm", "400.hmm", "1400.hmm", "2405.hmm"])
def test_library_cpu_equals_oracle(prof):
    """The library's CPU DP (Viterbi_HMM.run_on_sequence) is bitwise the oracle's, both insert modes."""
    o = OracleProfile(prof)
    me, _, _ = o.arrays()
    codes, offsets = random_batch(11, 12, 0, 300)
    gc, go = gapped_homolog_batch(me, 12, 8, 150, 400)
    for insert_mode in (0, 1):
        msc, isc, tsc, consts, _ = lib_tables(prof, insert_mode)
        for c, off in ((codes, offsets), (gc, go)):
            want = o.vit_score_batch(c, off, insert_mode)
            got = lib_cpu_scores(msc, isc if insert_mode else None, tsc, consts, c, off)
            assert np.array_equal(bits(got), bits(want)), (prof, insert_mode)


def msv_reduction_tables(o: OracleProfile):
    """Transitions under which Viterbi IS MSV: m->m probability 1 (score 0), every other transition
    impossible (-inf), no insert scores."""
    M = o.model_length
    tsc = np.full((M, 7), -np.inf, F)
    tsc[:, 0] = 0.0
    return o.emission_scores(), tsc, o.constants()


def test_msv_reduction_reproduces_reference_golden():
    """Pinned against the reference's own output: the Viterbi DP with MSV's transitions returns the
    reference build's MSV scores (tests/golden/example_scores.tsv, all 24 profiles x fasta_like_example)
    bit for bit -- through the oracle restatement and through the library's CPU DP."""
    fa = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "fasta_like_example.fsa"))
    rows = read_golden_tsv("example_scores.tsv")
    for prof in PROFILES:
        want = np.array([w for p, i, L, w in rows if p == prof], np.float32)
        o = OracleProfile(prof)
        msc, tsc, consts = msv_reduction_tables(o)
        got = vit_score_tables(msc, None, tsc, consts, fa.codes, fa.offsets)
        assert np.array_equal(bits(got), bits(want)), prof
        got_lib = lib_cpu_scores(msc, None, tsc, consts, fa.codes, fa.offsets)
        assert np.array_equal(bits(got_lib), bits(want)), prof


def test_empty_sequence_and_bad_residue_cpu():
    msc, isc, tsc, consts, h = lib_tables("100.hmm")
    assert lib_cpu_scores(msc, None, tsc, consts, np.zeros(0, np.uint8), np.zeros(2, np.uint64))[0] == -np.inf
    r = C.c_float()
    bad = np.array([3, 20, 1], np.uint8)
    assert _native.lib().msv_vit_cpu_score(msc.ctypes.data, None, tsc.ctypes.data, msc.shape[1], *consts,
                                           bad.ctypes.data, 3, C.byref(r)) == _native.MSV_ERR_BAD_RESIDUE


def test_viterbi_pvalues_against_the_profiles_own_calibration():
    """Statistical pin (CPU, oracle scores): HMMER3 fits STATS LOCAL VITERBI mu to the Viterbi bit scores of
    iid background sequences of length 200; our P-values of such sequences are ~uniform and the refitted
    mu (lambda fixed) lands near the file's.  HMMER calibrates with its 16-bit ViterbiFilter, whose
    N/C/J loops cost -3 nats per sequence in place of L log(L/(L+3)) and whose entry is occupancy-weighted
    rather than the MSV path's uniform tr_B_Mk, so the bound is 1 bit (measured: profiles/r04_vit_calibration.jsonl);
    a nats/bits, sign or null-model error misses by many bits.  The GPU test repeats this on all 24
    profiles at 20k sequences."""
    for prof, seed in (("100.hmm", 21), ("400.hmm", 22)):
        codes, offsets = background_batch(seed, 1500, 200)
        o = OracleProfile(prof)
        sc = o.vit_score_batch(codes, offsets, 0, threads=8)
        h = msv.Profile_HMM(profile_path(prof))
        mu, lam = h.stats_local_viterbi_mu, h.stats_local_viterbi_lambda
        pv = np.zeros(len(sc), np.float64)
        assert _native.lib().msv_pvalues(sc.ctypes.data, offsets.ctypes.data, len(sc), mu, lam, pv.ctypes.data) == 0
        b = mu - np.log(-np.log1p(-pv)) / lam
        mu_fit = -np.log(np.mean(np.exp(-lam * b))) / lam
        assert abs(mu_fit - mu) < 1.0, (prof, mu, mu_fit)
        for t in (0.5, 0.1):
            assert t / 2.5 < float(np.mean(pv < t)) < t * 2.5, (prof, t, float(np.mean(pv < t)))
