"""Model lengths outside the reference's 24 profiles (LENG 100..2405): tiny models (LENG 1..99, which every plan
pads to its lane layout with -inf states) and the first length past the compiled family (4097 states).

The reference scores any LENG (MSV_HMM.cpp:74-113 loops j = 1..LENG), so a tiny model must score exactly like
its CPU DP; this library's kernel family stops at 4096 states, and a longer model must be refused
with MSV_ERR_UNSUPPORTED_MODEL, not scored wrongly.  The .hmm files are seeded synthetic HMMER3 text
(hmm_fasta_viterbi_amd.synthetic.write_hmm); the checker is the oracle (the reference's own parser and CPU DP
compiled in oracle/_ref, and the C restatement of the Viterbi stage)."""
import numpy as np
import pytest

import hmm_fasta_viterbi_amd as msv
from hmm_fasta_viterbi_amd._native import MSVError
from hmm_fasta_viterbi_amd.synthetic import homolog_batch, random_batch, write_hmm
from oracle_lib import OracleProfile, bits

TINY = (1, 2, 3, 5, 8, 16, 17, 33, 64, 65, 99)


def _arrays_equal(a, b):
    return a.shape == b.shape and np.array_equal(bits(a), bits(b))


def test_tiny_models_parse_like_the_reference(tmp_path):
    """CPU: the library's .hmm reader on 1..99-node files equals the reference parser (Profile_HMM.cpp:8-122)."""
    for leng in TINY:
        path = str(tmp_path / f"tiny{leng}.hmm")
        write_hmm(path, leng, 500 + leng)
        h, o = msv.Profile_HMM(path), OracleProfile(path)
        assert h.model_length == o.model_length == leng + 1
        me, ie, tr = o.arrays()
        assert _arrays_equal(h.match_emissions, me) and _arrays_equal(h.insert_emissions, ie)
        assert _arrays_equal(h.transitions, tr)
        es, tBM, tEC, tEJ = h.msv_scores()
        assert _arrays_equal(es, o.emission_scores())
        assert bits(np.array([tBM, tEC, tEJ], np.float32)).tolist() == bits(np.array(o.constants(), np.float32)).tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("leng", TINY)
def test_tiny_models_every_plan(tmp_path, leng):
    """MSV at batch sizes that take each plan the model has (one sequence, a few hundred, thousands), random and
    homolog sequences (J overtakes N), lengths 0..120; and the Viterbi stage on the same batch.  Bitwise."""
    path = str(tmp_path / f"tiny{leng}.hmm")
    write_hmm(path, leng, 500 + leng)
    h = msv.Profile_HMM(path)
    o = OracleProfile(path)
    e = msv.MSV_HMM(h)
    v = msv.Viterbi_HMM(h)
    try:
        plans = set()
        for n in (1, 300, 6000):
            rc, ro = random_batch(900 + leng + n, n, 0, 120)
            if n > 1:
                hc, ho = homolog_batch(h.match_emissions, 7 + leng, n // 10, 1, 120)
                codes = np.concatenate([rc, hc])
                offsets = np.concatenate([ro, ro[-1] + ho[1:]]).astype(np.uint64)
            else:
                codes, offsets = rc, ro
            want = o.score_batch(codes, offsets)
            got = e.score_batch(codes=codes, offsets=offsets)
            assert _arrays_equal(got, want), (leng, n, e.variant_for(len(offsets) - 1))
            plans.add(e.variant_for(len(offsets) - 1))
            if n == 300:
                vw = o.vit_score_batch(codes, offsets)
                vg = v.score_batch(codes=codes, offsets=offsets)
                assert _arrays_equal(vg, vw), (leng, v.describe()["variant"])
        print(f"LENG {leng}: MSV plans {sorted(plans)}, Viterbi {v.describe()['variant']}")
    finally:
        e.close()
        v.close()


@pytest.mark.gpu
def test_model_past_the_kernel_family_is_refused(tmp_path):
    """4,096 states is the largest model the compiled family covers (test_synthetic_4096_auto_variant scores
    it); 4,097 is refused with MSV_ERR_UNSUPPORTED_MODEL by both stages, at profile creation."""
    path = str(tmp_path / "syn4097.hmm")
    write_hmm(path, 4097, 4097)
    h = msv.Profile_HMM(path)
    assert h.model_length == 4098
    for make in (msv.MSV_HMM, msv.Viterbi_HMM):
        with pytest.raises(MSVError) as err:
            make(h)
        assert err.value.status == 6, (make.__name__, err.value)  # MSV_ERR_UNSUPPORTED_MODEL
