"""The oracle (oracle/msv_oracle.c, a plain-C restatement of MSV_HMM::run_on_sequence,
algorithms/MSV_HMM.cpp:74-113) pinned against the golden scores produced by the REFERENCE's own
CPU path (oracle/make_golden.py over oracle/_ref).  CPU only.  Tolerance: bitwise."""
import json
import os

import numpy as np
import pytest

from oracle_lib import (GOLD, PROFILES, OracleProfile, REF_SO, bits, make_batch, profile_path, read_golden_tsv)


@pytest.fixture(scope="module")
def fasta_parsed():
    with open(os.path.join(GOLD, "fasta_parsed.json")) as f:
        return json.load(f)


def test_example_scores_all_profiles_bitwise(fasta_parsed):
    """Appendix-B table: 24 profiles x fasta_like_example.fsa (test_MSV.cpp:14-36 inputs)."""
    seqs = fasta_parsed["fasta_like_example.fsa"]
    rows = read_golden_tsv("example_scores.tsv")
    assert len(rows) == 24 * 4
    profs = {}
    for prof, i, L, want in rows:
        p = profs.setdefault(prof, OracleProfile(prof))
        assert len(seqs[i]) - 1 == L
        got = np.float32(p.score_string(seqs[i]))
        assert bits(got) == bits(want), (prof, i, got, want)


def test_random_fasta_scores_bitwise(fasta_parsed):
    seqs = fasta_parsed["random_FASTA.fsa"]
    rows = read_golden_tsv("random_fasta_scores.tsv")
    assert len(rows) == 24 * 3
    for prof in ("100.hmm", "1400.hmm", "2405.hmm"):
        p = OracleProfile(prof)
        for prof_, i, L, want in rows:
            if prof_ == prof:
                assert bits(p.score_string(seqs[i])) == bits(want)


@pytest.mark.parametrize("prof", ["100", "1400", "2405"])
def test_seeded_batches_bitwise(prof):
    z = np.load(os.path.join(GOLD, f"seeded_{prof}.npz"))
    got = OracleProfile(prof).score_batch(z["codes"], z["offsets"])
    assert np.array_equal(bits(got), bits(z["scores"]))
    # edge lengths present: 0 -> -inf, 1, 2, 3500
    lens = np.diff(z["offsets"])
    assert lens[0] == 0 and np.isneginf(got[0])
    assert 3500 in lens


def test_seeded_all_profiles_bitwise():
    z = np.load(os.path.join(GOLD, "seeded_all_profiles.npz"))
    for prof in PROFILES:
        k = prof.split(".")[0]
        got = OracleProfile(prof).score_batch(z[f"codes_{k}"], z[f"offsets_{k}"])
        assert np.array_equal(bits(got), bits(z[f"scores_{k}"])), prof


def test_known_constants():
    """tr_B_Mk = logf(2 / (M (M+1))) with M = LENG + 1 (MSV_HMM.cpp:51)."""
    want = {"100": -8.54694653, "1400": -13.7974491, "2405": -14.8787098}
    for prof, v in want.items():
        p = OracleProfile(prof)
        b, c, j = p.constants()
        assert abs(b - v) < 1e-6
        assert np.float32(c) == np.float32(j) == np.float32(np.log(np.float32(0.5)))
        es = p.emission_scores()
        assert np.all(np.isneginf(es[:, 0]))  # dummy M0 column
        assert np.all(np.isfinite(es[:, 1:]))


def test_edge_scores_100():
    """L=1 -> -7.96733618 and L=2 -> -7.00991678 on 100.hmm for its edge inputs."""
    z = np.load(os.path.join(GOLD, "seeded_100.npz"))
    got = OracleProfile("100").score_batch(z["codes"][:3], np.array([0, 0, 1, 3], np.uint64))
    assert np.isneginf(got[0])
    assert np.array_equal(bits(got[1:]), bits(z["scores"][1:3]))


def test_parsed_profiles_match_reference_parser():
    with open(os.path.join(GOLD, "parsed_profiles.json")) as f:
        dig = json.load(f)
    import hashlib
    for prof in PROFILES:
        p = OracleProfile(prof)
        m, i, t = p.arrays()
        d = dig[prof]
        assert p.model_length == d["model_length"]
        assert p.name() == d["name"]
        assert [float(np.float32(x)).hex() for x in p.stats()] == d["stats_hex"]
        assert hashlib.sha256(m.tobytes()).hexdigest() == d["match_sha256"], prof
        assert hashlib.sha256(i.tobytes()).hexdigest() == d["insert_sha256"], prof
        assert hashlib.sha256(t.tobytes()).hexdigest() == d["transitions_sha256"], prof


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="reference build only exists in the build container")
def test_oracle_vs_reference_build_fresh_batch():
    """Cross-check on inputs the fixtures do not contain, against the reference compiled here."""
    import ctypes as C
    ref = C.CDLL(REF_SO)
    ref.ref_score_codes.restype = C.c_double
    ref.ref_score_codes.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_long, C.c_int, C.c_void_p]
    rng = np.random.default_rng(99)
    for prof in ("200", "1301", "2050"):
        codes, offsets = make_batch(4242, rng.integers(0, 300, size=40))
        want = np.zeros(40, np.float32)
        assert ref.ref_score_codes(profile_path(prof).encode(), codes.ctypes.data, offsets.ctypes.data, 40, 4,
                                   want.ctypes.data) >= 0
        got = OracleProfile(prof).score_batch(codes, offsets)
        assert np.array_equal(bits(got), bits(want))
