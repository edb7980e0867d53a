"""Host side of the product (libmsv_hip.so, no GPU needed): parsers and MSV precompute against the
reference's own parser outputs (tests/golden/*, oracle/make_golden.py) and the pinned oracle."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import hmm_fasta_viterbi_amd as msv
from oracle_lib import DATA, GOLD, PROFILES, ROOT, OracleProfile, bits, profile_path


@pytest.fixture(scope="module")
def digests():
    with open(os.path.join(GOLD, "parsed_profiles.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("prof", PROFILES)
def test_profile_parser_matches_reference(prof, digests):
    """Profile_HMM.cpp:48-122 semantics incl. HMMER3.0 headers (1301.hmm) and '*' -> p = 1."""
    h = msv.Profile_HMM(profile_path(prof))
    d = digests[prof]
    assert h.model_length == d["model_length"]
    assert h.name == d["name"]
    st = [h.stats_local_msv_mu, h.stats_local_msv_lambda, h.stats_local_viterbi_mu, h.stats_local_viterbi_lambda,
          h.stats_local_forward_theta, h.stats_local_forward_lambda]
    assert [float(np.float32(x)).hex() for x in st] == d["stats_hex"]
    assert hashlib.sha256(h.match_emissions.astype(np.float32).tobytes()).hexdigest() == d["match_sha256"]
    assert hashlib.sha256(h.insert_emissions.astype(np.float32).tobytes()).hexdigest() == d["insert_sha256"]
    assert hashlib.sha256(h.transitions.astype(np.float32).tobytes()).hexdigest() == d["transitions_sha256"]


def test_profile_known_answers_100():
    """test_hmm_parsing.cpp:19-37 restated (5 ULP)."""
    h = msv.Profile_HMM(profile_path("100"))
    p = lambda x: np.exp(-np.float32(x), dtype=np.float32)
    assert h.model_length == 101 and h.name == "Pfam-B_229"
    assert abs(h.stats_local_msv_mu - np.float32(-9.5678)) <= 5 * np.finfo(np.float32).eps * 19.2
    np.testing.assert_array_max_ulp(h.insert_emissions[0, 0], p(2.68618), 5)
    np.testing.assert_array_max_ulp(h.transitions[0, 6], p(0.0), 5)
    np.testing.assert_array_max_ulp(h.match_emissions[1, 0], p(2.66211), 5)
    np.testing.assert_array_max_ulp(h.match_emissions[100, 19], p(4.01014), 5)
    np.testing.assert_array_max_ulp(h.transitions[1, 1], p(4.09464), 5)
    assert np.all(h.match_emissions[0] == 0)  # dummy node 0


def test_profile_full_arrays_100_and_1301():
    for prof in ("100", "1301"):
        z = np.load(os.path.join(GOLD, f"parsed_{prof}.npz"))
        h = msv.Profile_HMM(profile_path(prof))
        assert np.array_equal(bits(h.match_emissions), bits(z["match"]))
        assert np.array_equal(bits(h.insert_emissions), bits(z["insert"]))
        assert np.array_equal(bits(h.transitions), bits(z["transitions"]))


def test_profile_missing_file_fails_loudly():
    with pytest.raises(msv.MSVError) as e:
        msv.Profile_HMM(os.path.join(DATA, "profile_HMMs", "nope.hmm"))
    assert e.value.name == "MSV_ERR_IO"


@pytest.mark.parametrize("name", ["fasta_like_example.fsa", "random_FASTA.fsa", "edge_cases.fsa"])
def test_fasta_reader_matches_reference(name):
    """FASTA_protein_sequences.cpp:9-44: '#' sentinel, joined lines, whole-record rejection,
    empty records kept, '#' inside a record kept (rejected only when scored)."""
    with open(os.path.join(GOLD, "fasta_parsed.json")) as f:
        want = json.load(f)[name]
    path = os.path.join(GOLD if name == "edge_cases.fsa" else os.path.join(DATA, "FASTA_files"), name)
    fa = msv.FASTA_protein_sequences(path)
    assert fa.sequences == want
    assert len(fa.offsets) == len(want) + 1
    if name == "edge_cases.fsa":
        assert fa.rejected == 5
        assert fa.headers[0] == "ok plain"


def test_fasta_missing_and_malformed(tmp_path):
    with pytest.raises(msv.MSVError):
        msv.FASTA_protein_sequences(str(tmp_path / "none.fsa"))
    bad = tmp_path / "bad.fsa"
    bad.write_text("ACDE\n>x\nAC\n")
    with pytest.raises(msv.MSVError) as e:
        msv.FASTA_protein_sequences(str(bad))
    assert e.value.name == "MSV_ERR_PARSE"


def test_random_fasta_generator_format(tmp_path):
    """Files in the format of FASTA_files/random_FASTA_generator.py:7-16 (70-column lines)."""
    from hmm_fasta_viterbi_amd.synthetic import write_fasta, random_batch
    codes, offsets = random_batch(7, 50, 1, 300)
    path = tmp_path / "r.fsa"
    write_fasta(str(path), codes, offsets)
    fa = msv.FASTA_protein_sequences(str(path))
    assert np.array_equal(fa.codes, codes) and np.array_equal(fa.offsets, offsets)
    assert fa.headers[3] == " random 3"


def test_encode_and_pack():
    assert list(msv.encode("ACDY")) == [0, 1, 2, 19]
    with pytest.raises(IndexError):
        msv.encode("ACX")
    codes, offs = msv.pack_sequences(["#AC", "#", "#Y"])
    assert list(codes) == [0, 1, 19] and list(offs) == [0, 2, 2, 3]


def test_msv_precompute_matches_oracle():
    """MSV_HMM.cpp:35-57 (host libm) bitwise equal to the oracle restatement, every profile."""
    for prof in PROFILES:
        es, b, c, j = msv.Profile_HMM(profile_path(prof)).msv_scores()
        o = OracleProfile(prof)
        assert np.array_equal(bits(es), bits(o.emission_scores())), prof
        assert bits([b, c, j]).tolist() == bits(o.constants()).tolist()


def test_synthetic_profile_writer_parses_like_oracle(tmp_path):
    """synthetic.write_hmm (models beyond the reference's 2405 states): the product parser and the
    oracle parser agree on every array and on the MSV precompute."""
    from hmm_fasta_viterbi_amd.synthetic import write_hmm
    path = str(tmp_path / "syn3000.hmm")
    write_hmm(path, 3000, 3)
    h, o = msv.Profile_HMM(path), OracleProfile(path)
    assert h.model_length == o.model_length == 3001
    for got, want in zip((h.match_emissions, h.insert_emissions, h.transitions), o.arrays()):
        assert np.array_equal(bits(got), bits(want))
    es, b, c, j = h.msv_scores()
    assert np.array_equal(bits(es), bits(o.emission_scores()))
    assert bits([b, c, j]).tolist() == bits(o.constants()).tolist()


def test_sequence_transitions_match_oracle():
    import ctypes as C
    from oracle_lib import oracle
    L = oracle()
    for n in [0, 1, 2, 3, 17, 399, 400, 2000, 35000, 131071]:
        a, b = C.c_float(), C.c_float()
        L.oracle_seq_transitions(n, C.byref(a), C.byref(b))
        got = msv.sequence_transitions(n)
        assert bits(got).tolist() == bits([a.value, b.value]).tolist()
    loop, move = msv.sequence_transitions(0)
    assert np.isneginf(loop) and move == 0.0


def test_cpp_parser_driver():
    """C++ restatement of test_hmm_parsing.cpp / test_fasta_parsing.cpp against the C++ API."""
    exe = os.path.join(ROOT, "hmm_fasta_viterbi_amd", "lib", "test_parsers")
    r = subprocess.run([exe, ROOT], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def _pvalue_f64(score, L, mu, lam):
    """float64 restatement of HMMER3's MSV-stage P-value with HMMER's float steps (msv.h)."""
    if L == 0:
        return 1.0
    p1 = np.float32(np.float32(L) / np.float32(L + 1))
    nullsc = np.float32(float(L) * np.log(np.float64(p1)) + np.log(1.0 - np.float64(p1)))
    bits = np.float32(np.float32(np.float32(score) - nullsc) / np.float32(0.69314718055994529))
    y = np.float64(lam) * (np.float64(bits) - np.float64(mu))
    ey = -np.exp(-y)
    return float(-ey if abs(ey) < 5e-9 else 1.0 - np.exp(ey))


def test_msv_pvalues_host_formula():
    """SURVEY 8(f)-4 (parity unpinned: no reference implementation): the C-ABI host P-values follow
    the HMMER3 MSV-stage formula on golden reference scores, incl. L=0 (-inf) and the tails."""
    import ctypes as C
    z = np.load(os.path.join(GOLD, "seeded_1400.npz"))
    scores, offsets = z["scores"].astype(np.float32), z["offsets"].astype(np.uint64)
    h = msv.Profile_HMM(profile_path("1400.hmm"))
    mu, lam = h.stats_local_msv_mu, h.stats_local_msv_lambda
    n = len(offsets) - 1
    out = np.zeros(n, np.float64)
    from hmm_fasta_viterbi_amd import _native
    assert _native.lib().msv_pvalues(scores.ctypes.data, offsets.ctypes.data, n, mu, lam, out.ctypes.data) == 0
    want = np.array([_pvalue_f64(scores[i], int(offsets[i + 1] - offsets[i]), mu, lam) for i in range(n)])
    np.testing.assert_allclose(out, want, rtol=1e-13, atol=0)
    assert np.all((out >= 0) & (out <= 1))
    lengths = np.diff(offsets)
    assert np.all(out[lengths == 0] == 1.0)
    # a very high score lands in the small-tail branch, a very low one gives P -> 1
    hi = np.zeros(1, np.float64)
    lo = np.zeros(1, np.float64)
    off = np.array([0, 400], np.uint64)
    _native.lib().msv_pvalues(np.array([200.0], np.float32).ctypes.data, off.ctypes.data, 1, mu, lam, hi.ctypes.data)
    _native.lib().msv_pvalues(np.array([-200.0], np.float32).ctypes.data, off.ctypes.data, 1, mu, lam, lo.ctypes.data)
    assert 0 < hi[0] < 1e-30 and lo[0] == 1.0
    assert hi[0] == _pvalue_f64(200.0, 400, mu, lam)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_bounds_c_abi_matches_distributed(world):
    """msv_shard_bounds (C-ABI, used by msv_score_batch_multi) == distributed.shard_bounds (torch
    path): contiguous, residue-balanced, covering, incl. empty sequences and n < world."""
    from hmm_fasta_viterbi_amd.distributed import shard_bounds as py_bounds
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    for seed, n in ((1, 0), (2, 1), (3, 5), (4, 1000)):
        _, offsets = random_batch(seed, n, 0, 600)
        b = msv.shard_bounds(offsets, world)
        assert b[0] == 0 and b[-1] == n and np.all(np.diff(b.astype(np.int64)) >= 0)
        assert [int(x) for x in b] == [py_bounds(offsets, world, 0)[0]] + [py_bounds(offsets, world, r)[1]
                                                                          for r in range(world)]


def _py_fasta(text: bytes):
    """Line-loop restatement of FASTA_protein_sequences.cpp:9-44 (as the C++ reader documents)."""
    lut = {c: i for i, c in enumerate(b"ACDEFGHIKLMNPQRSTVWY")}
    lut[ord("#")] = 255
    codes, offsets, headers, rejected = bytearray(), [0], [], 0
    cur, bad, open_ = bytearray(), False, False
    lines = text.split(b"\n")
    if text.endswith(b"\n"):
        lines = lines[:-1]
    for line in lines:
        if line[:1] == b">":
            if open_:
                if bad:
                    rejected += 1
                else:
                    codes += cur
                    offsets.append(len(codes))
                    headers.append(hdr)
            hdr, cur, bad, open_ = line[1:].decode("latin-1"), bytearray(), False, True
        elif open_ and not bad:
            for ch in line:
                if ch not in lut:
                    bad = True
                    break
                cur.append(lut[ch])
    if open_:
        if bad:
            rejected += 1
        else:
            codes += cur
            offsets.append(len(codes))
            headers.append(hdr)
    return np.frombuffer(bytes(codes), np.uint8), np.array(offsets, np.uint64), headers, rejected


def test_fasta_reader_parallel_chunks_match_line_semantics(tmp_path):
    """A ~20 MB file (parsed in several chunks on several threads) with rejected records (lowercase,
    X, CR), '#' inside records, empty records and blank lines: identical to the line-loop semantics."""
    rng = np.random.default_rng(9)
    letters = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    parts = []
    for i in range(50_000):
        L = int(rng.integers(0, 700))
        seq = letters[rng.integers(0, 20, L)].tobytes()
        kind = rng.integers(0, 40)
        if kind == 0:
            seq = seq[: L // 2] + b"x" + seq[L // 2:]
        elif kind == 1:
            seq = seq + b"X"
        elif kind == 2:
            seq = seq.replace(b"A", b"#", 1)
        lines = [seq[k:k + 60] for k in range(0, len(seq), 60)] or [b""]
        eol = b"\r\n" if kind == 3 else b"\n"
        parts.append(b">rec %d desc\n" % i + eol.join(lines) + eol)
        if kind == 4:
            parts.append(b"\n")
    text = b"".join(parts)
    path = tmp_path / "big.fsa"
    path.write_bytes(text)
    assert len(text) > 16 << 20
    fa = msv.FASTA_protein_sequences(str(path))
    codes, offsets, headers, rejected = _py_fasta(text)
    assert fa.rejected == rejected and rejected > 1000
    assert np.array_equal(fa.offsets, offsets)
    assert np.array_equal(fa.codes, codes)
    assert fa.headers == headers


def test_native_random_fasta_generator_format(tmp_path):
    """lib/random_fasta (seeded mt19937_64) writes the reference generator's format
    (random_FASTA_generator.py:1-16): same line structure as data/FASTA_files/random_FASTA.fsa by
    default, seeded and reproducible, length range honoured."""
    exe = os.path.join(ROOT, "hmm_fasta_viterbi_amd", "lib", "random_fasta")
    a, b, c = (str(tmp_path / x) for x in ("a.fsa", "b.fsa", "c.fsa"))
    subprocess.run([exe, a], check=True)
    subprocess.run([exe, b], check=True)
    ref = open(os.path.join(DATA, "FASTA_files", "random_FASTA.fsa")).read().splitlines()
    got = open(a).read().splitlines()
    assert [len(x) for x in got] == [len(x) for x in ref]
    assert [x for x in got if x.startswith(">")] == [x for x in ref if x.startswith(">")]
    assert open(a).read() == open(b).read()
    subprocess.run([exe, c, "500", "0", "900", "7"], check=True)
    fa = msv.FASTA_protein_sequences(c)
    lens = np.diff(fa.offsets.astype(np.int64))
    assert len(fa) == 500 and fa.rejected == 0 and lens.min() >= 0 and lens.max() <= 900


def test_msv_pvalues_gumbel_against_scipy():
    """The Gumbel survival step of the P-values, pinned against an independent implementation
    (scipy.stats.gumbel_r.sf with loc = mu, scale = 1/lambda, HMMER's esl_gumbel_surv in closed
    form), on the bit scores the null1 step gives (HMMER3's p7_bg_NullOne restated; no reference
    implementation exists, so that step stays unpinned)."""
    import scipy.stats as ss
    from hmm_fasta_viterbi_amd import _native
    rng = np.random.default_rng(7)
    n = 4000
    lengths = rng.integers(1, 3000, n).astype(np.uint64)
    offsets = np.zeros(n + 1, np.uint64)
    np.cumsum(lengths, out=offsets[1:])
    scores = rng.uniform(-40.0, 25.0, n).astype(np.float32)
    for prof in ("100.hmm", "1400.hmm", "2405.hmm"):
        h = msv.Profile_HMM(profile_path(prof))
        mu, lam = h.stats_local_msv_mu, h.stats_local_msv_lambda
        out = np.zeros(n, np.float64)
        assert _native.lib().msv_pvalues(scores.ctypes.data, offsets.ctypes.data, n, mu, lam, out.ctypes.data) == 0
        L = lengths.astype(np.float64)
        p1 = (lengths.astype(np.float32) / (lengths + 1).astype(np.float32)).astype(np.float32)
        nullsc = (L * np.log(p1.astype(np.float64)) + np.log(1.0 - p1.astype(np.float64))).astype(np.float32)
        bits = ((scores - nullsc).astype(np.float32) / np.float32(0.69314718055994529)).astype(np.float32)
        want = ss.gumbel_r.sf(bits.astype(np.float64), loc=np.float64(mu), scale=1.0 / np.float64(lam))
        # scipy's sf = -expm1(-exp(-y)); the library's 1 - exp(-exp(-y)) loses relative precision only
        # where P is tiny, which the small-tail branch (P = exp(-y) when exp(-y) < 5e-9) covers
        np.testing.assert_allclose(out, want, rtol=1e-7, atol=1e-15)


def test_msv_pvalues_against_the_profiles_own_calibration():
    """The whole P-value pipeline (MSV score -> null1 -> bits -> Gumbel with the file's STATS LOCAL MSV)
    checked statistically against the calibration HMMER3 stored in the reference's own .hmm fixtures:
    HMMER fits mu to the MSV bit scores of iid background sequences of length 200 (p7_MSVMu), so our
    P-values of such sequences must be ~uniform, and a Gumbel mu refitted to our bit scores (lambda
    fixed, ML) must land on the file's mu.  The reference's float MSV scores ~0.0-0.5 bits above the
    calibration (HMMER calibrates with its 8-bit MSV filter), so the bounds allow 0.75 bits and a factor
    2.5 in the tail; a nats/bits, sign or null-model error moves these by orders of magnitude.  Scores
    here are the oracle's (CPU, bit-identical to the GPU kernel); the GPU test repeats it at 20k."""
    from hmm_fasta_viterbi_amd.synthetic import background_batch
    for prof, seed in (("100.hmm", 11), ("400.hmm", 12)):
        codes, offsets = background_batch(seed, 1500, 200)
        sc = OracleProfile(prof).score_batch(codes, offsets)
        e_h = msv.Profile_HMM(profile_path(prof))
        mu, lam = e_h.stats_local_msv_mu, e_h.stats_local_msv_lambda
        pv = np.zeros(len(sc), np.float64)
        from hmm_fasta_viterbi_amd import _native
        assert _native.lib().msv_pvalues(sc.ctypes.data, offsets.ctypes.data, len(sc), mu, lam, pv.ctypes.data) == 0
        bits = mu - np.log(-np.log1p(-pv)) / lam  # invert the Gumbel survival: the bit scores used
        mu_fit = -np.log(np.mean(np.exp(-lam * bits))) / lam
        assert abs(mu_fit - mu) < 0.75, (prof, mu, mu_fit)
        for t in (0.5, 0.1):
            assert t / 2.5 < float(np.mean(pv < t)) < t * 2.5, (prof, t, float(np.mean(pv < t)))
