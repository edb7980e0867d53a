"""GPU parity: the fused gfx950 MSV kernel (through the C-ABI) against the golden scores of the
reference's CPU path and the pinned oracle.  Tolerance: BITWISE (the north_star allows 1e-4; the
kernel uses only IEEE add/max in the reference's order, so equality is expected and required).
Size-independent properties cover BASELINE.json's full sizes."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import hmm_fasta_viterbi_amd as msv
from hmm_fasta_viterbi_amd.synthetic import concat_batches, homolog_batch, random_batch
from oracle_lib import GOLD, PROFILES, ROOT, OracleProfile, bits, profile_path, read_golden_tsv

_engines = {}


def engine(prof: str) -> msv.MSV_HMM:
    if prof not in _engines:
        _engines[prof] = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof)))
    return _engines[prof]


def test_device_visible():
    assert msv.device_count() >= 1


@pytest.mark.parametrize("prof", PROFILES)
def test_example_fasta_every_profile(prof):
    """test_MSV.cpp:14-36 inputs: every profile x fasta_like_example.fsa, via run_on_sequence,
    parallel_run_on_sequence(seq), parallel_run_on_sequence(seq, True) and the batch API."""
    fa = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "fasta_like_example.fsa"))
    want = np.array([w for p, i, L, w in read_golden_tsv("example_scores.tsv") if p == prof], np.float32)
    e = engine(prof)
    got_batch = e.score_batch(fa.sequences)
    assert np.array_equal(bits(got_batch), bits(want))
    for i, s in enumerate(fa.sequences):
        for got in (e.run_on_sequence(s), e.parallel_run_on_sequence(s), e.parallel_run_on_sequence(s, True)):
            assert bits(got) == bits(want[i]), (prof, i, got, want[i])


def test_random_fasta_3500():
    fa = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "random_FASTA.fsa"))
    rows = read_golden_tsv("random_fasta_scores.tsv")
    for prof in PROFILES:
        want = np.array([w for p, i, L, w in rows if p == prof], np.float32)
        assert np.array_equal(bits(engine(prof).score_batch(fa.sequences)), bits(want)), prof


@pytest.mark.parametrize("prof", ["100", "1400", "2405"])
def test_seeded_golden_edge_lengths(prof):
    """Lengths 0,1,2,3,...,257,1000,3500 + random, golden from the reference build."""
    z = np.load(os.path.join(GOLD, f"seeded_{prof}.npz"))
    got = engine(prof + ".hmm").score_batch(codes=z["codes"], offsets=z["offsets"])
    assert np.array_equal(bits(got), bits(z["scores"]))


def test_seeded_golden_every_profile():
    z = np.load(os.path.join(GOLD, "seeded_all_profiles.npz"))
    for prof in PROFILES:
        k = prof.split(".")[0]
        got = engine(prof).score_batch(codes=z[f"codes_{k}"], offsets=z[f"offsets_{k}"])
        assert np.array_equal(bits(got), bits(z[f"scores_{k}"])), prof


@pytest.mark.parametrize("prof,n,lmin,lmax,seed", [
    ("100", 3000, 300, 500, 1),      # cfg2 shape (sample)
    ("1400", 400, 300, 500, 2),      # cfg3 shape (sample)
    ("2405", 60, 1500, 2500, 4),     # cfg5 shape (sample)
    ("700", 500, 1, 900, 11),
    ("1901", 200, 1, 1200, 12),
    ("2050", 150, 1, 1500, 13),
])
def test_against_oracle_seeded(prof, n, lmin, lmax, seed):
    codes, offsets = random_batch(seed, n, lmin, lmax)
    want = OracleProfile(prof).score_batch(codes, offsets)
    got = engine(prof + ".hmm").score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))


def test_empty_and_degenerate_batches():
    e = engine("1400.hmm")
    # all empty -> -inf, no residue bytes at all
    got = e.score_batch(codes=np.zeros(0, np.uint8), offsets=np.zeros(6, np.uint64))
    assert np.all(np.isneginf(got))
    # empty batch
    assert e.score_batch(codes=np.zeros(0, np.uint8), offsets=np.zeros(1, np.uint64)).size == 0
    # homopolymers and a single very long sequence mixed with empties
    o = OracleProfile("1400")
    for r in range(20):
        codes = np.full(700, r, np.uint8)
        offs = np.array([0, 0, 700, 700], np.uint64)
        assert np.array_equal(bits(e.score_batch(codes=codes, offsets=offs)), bits(o.score_batch(codes, offs)))


def test_bad_residue_raises_like_reference():
    e = engine("100.hmm")
    with pytest.raises(IndexError):
        e.run_on_sequence("#ACDXEF")
    with pytest.raises(IndexError):
        e.score_batch(codes=np.array([0, 1, 20, 3], np.uint8), offsets=np.array([0, 4], np.uint64))
    with pytest.raises(IndexError):  # '#' inside a record (kept by the FASTA reader)
        e.run_on_sequence("#AC#DE")
    # the profile stays usable after an error
    assert np.isfinite(e.run_on_sequence("#ACDEF"))


def test_bad_residue_every_large_table_layout():
    """Codes >= 20 must reach the +inf poison row in every layout of a table larger than LDS: the
    split layouts (LDS rows 0..19 only, poison row in the global B table; G = 32 and 64) and the
    G = 64 LDS/L2 row-class layout."""
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("2405.hmm")))
    good_c, good_o = random_batch(31, 40, 1, 300)
    bad = good_c.copy()
    bad[int(good_o[17]) + 3] = 20
    want = OracleProfile("2405").score_batch(good_c, good_o)
    names = [v for v in msv.MSV_HMM.variants()
             if not v.startswith("exp") and _variant_shape(v)[0] * _variant_shape(v)[1] >= 2405
             and _variant_shape(v)[0] >= 32]
    assert any("_a" in v and v.startswith("msv_g32") for v in names)
    for name in names:
        e.set_variant(name)
        with pytest.raises(IndexError):
            e.score_batch(codes=bad, offsets=good_o)
        assert np.array_equal(bits(e.score_batch(codes=good_c, offsets=good_o)), bits(want)), name
    e.close()


def test_order_entry_outside_batch_is_reported():
    """A caller's dequeue order with an index >= n is reported (MSV_ERR_INVALID_ARGUMENT) and never
    dereferenced; a valid order on the same profile afterwards scores exactly."""
    import torch
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("400.hmm")))
    codes, offsets = random_batch(41, 3000, 1, 300)
    want = OracleProfile("400").score_batch(codes, offsets)
    dev = torch.device("cuda:0")
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.zeros(3000, dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    bad = torch.arange(3000, dtype=torch.int32, device=dev)
    bad[1234] = 3000 + 77
    torch.cuda.synchronize()
    e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), 3000, s.data_ptr(), bad.data_ptr(), st.cuda_stream)
    with pytest.raises(msv.MSVError) as ex:
        e.check(st.cuda_stream)
    assert ex.value.name == "MSV_ERR_INVALID_ARGUMENT"
    good = torch.arange(3000, dtype=torch.int32, device=dev).flip(0)
    e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), 3000, s.data_ptr(), good.data_ptr(), st.cuda_stream)
    e.check(st.cuda_stream)
    assert np.array_equal(bits(s.cpu().numpy()), bits(want))
    e.close()


def test_long_sequence_grows_table():
    e = engine("100.hmm")
    codes, offsets = random_batch(77, 2, 140000, 150000)
    want = OracleProfile("100").score_batch(codes, offsets)
    assert np.array_equal(bits(e.score_batch(codes=codes, offsets=offsets)), bits(want))


def test_device_api_with_torch_tensors_and_order():
    torch = pytest.importorskip("torch")
    e = engine("1400.hmm")
    codes, offsets = random_batch(5, 3000, 1, 800)
    dev = torch.device("cuda:0")
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.empty(3000, dtype=torch.float32, device=dev)
    order = torch.empty(3000, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    e.order_longest_first(o.data_ptr(), 3000, order.data_ptr(), stream)
    e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), 3000, s.data_ptr(), order.data_ptr(), stream)
    e.check(stream)
    got = s.cpu().numpy()
    want = e.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))
    # the order is a permutation sorted by length, descending
    perm = order.cpu().numpy().astype(np.int64)
    assert np.array_equal(np.sort(perm), np.arange(3000))
    lens = np.diff(offsets.astype(np.int64))[perm]
    assert np.all(lens[:-1] >= lens[1:])
    sample = np.arange(0, 3000, 37)
    want_o = OracleProfile("1400").score_batch(*subset(codes, offsets, sample))
    assert np.array_equal(bits(got[sample]), bits(want_o))


def subset(codes, offsets, idx):
    parts = [codes[int(offsets[i]):int(offsets[i + 1])] for i in idx]
    offs = np.zeros(len(idx) + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts])
    return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), offs


def test_full_size_cfg3_properties():
    """BASELINE cfg3 at full size (1400.hmm x 100k, len U[300,500]): determinism, permutation
    invariance, and a seeded sample against the oracle."""
    e = engine("1400.hmm")
    codes, offsets = random_batch(2, 100_000, 300, 500)
    a = e.score_batch(codes=codes, offsets=offsets)
    b = e.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(a), bits(b))
    assert np.all(np.isfinite(a))
    perm = np.random.default_rng(0).permutation(100_000)[:5000]
    pc, po = subset(codes, offsets, perm)
    assert np.array_equal(bits(e.score_batch(codes=pc, offsets=po)), bits(a[perm]))
    sample = perm[:60]
    assert np.array_equal(bits(a[sample]), bits(OracleProfile("1400").score_batch(*subset(codes, offsets, sample))))


def test_full_size_cfg5_sample():
    """BASELINE cfg5 shape (2405.hmm, len U[1500,2500]) at 20k sequences + oracle sample."""
    e = engine("2405.hmm")
    codes, offsets = random_batch(4, 20_000, 1500, 2500)
    a = e.score_batch(codes=codes, offsets=offsets)
    sample = np.arange(0, 20_000, 1000)
    assert np.array_equal(bits(a[sample]), bits(OracleProfile("2405").score_batch(*subset(codes, offsets, sample))))


def test_cpp_parity_driver():
    """tests/cpp/test_msv.cpp: the C++ MSV_HMM surface, every profile, bitwise vs golden."""
    exe = os.path.join(ROOT, "hmm_fasta_viterbi_amd", "lib", "test_msv")
    r = subprocess.run([exe, ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_describe_variant_for_1400():
    d = engine("1400.hmm").describe()
    assert d["model_length"] == 1401
    assert d["lanes_per_group"] * d["states_per_lane"] >= 1400



def _variant_shape(name):
    parts = name.split("_")
    return int(parts[1][1:]), int(parts[2][1:])


def test_every_variant_matches_oracle(tmp_path):
    """Every shipped kernel instantiation (G, S, waves, PF, D), forced with set_variant, on the
    largest profile it covers (so BIG variants run a real BIG table), against the oracle.  Model
    lengths past the reference's largest profile (2405) use seeded synthetic HMMER3 files."""
    from hmm_fasta_viterbi_amd.synthetic import write_hmm
    paths = [profile_path(p) for p in PROFILES]
    for leng in (2600, 3000, 3500, 4096):
        paths.append(str(tmp_path / f"syn{leng}.hmm"))
        write_hmm(paths[-1], leng, leng)
    lengs = {p: msv.Profile_HMM(p).model_length - 1 for p in paths}
    codes0, offsets0 = random_batch(21, 48, 0, 400)
    by_prof = {}
    for name in msv.MSV_HMM.variants():
        if name.startswith("exp"):
            continue
        g, s = _variant_shape(name)
        fits = [p for p in paths if lengs[p] <= g * s]
        if fits:
            by_prof.setdefault(max(fits, key=lambda p: lengs[p]), []).append(name)
    assert sum(len(v) for v in by_prof.values()) >= 40
    for prof, names in by_prof.items():
        # random sequences (J stays below N) interleaved with sequences emitted by the profile
        # (J overtakes N: the kernel's group reduction of J for B runs on those rows)
        hc, ho = homolog_batch(msv.Profile_HMM(prof).match_emissions, 22, 24, 0, 400)
        codes, offsets = concat_batches((codes0, offsets0), (hc, ho))
        want = OracleProfile(prof).score_batch(codes, offsets)
        e = msv.MSV_HMM(msv.Profile_HMM(prof))
        for name in names:
            e.set_variant(name)
            got = e.score_batch(codes=codes, offsets=offsets)
            assert np.array_equal(bits(got), bits(want)), (prof, name)
        e.close()


def test_synthetic_4096_auto_variant(tmp_path):
    """The largest supported model (4096 states) under the automatic variant choice, at the cfg5
    sequence-length range."""
    from hmm_fasta_viterbi_amd.synthetic import write_hmm
    path = str(tmp_path / "syn4096.hmm")
    write_hmm(path, 4096, 1)
    codes, offsets = random_batch(5, 40, 1500, 2500)
    e = msv.MSV_HMM(msv.Profile_HMM(path))
    assert e.describe()["lanes_per_group"] == 64
    assert np.array_equal(bits(e.score_batch(codes=codes, offsets=offsets)),
                          bits(OracleProfile(path).score_batch(codes, offsets)))


def test_score_grid_example_all_profiles():
    """every profile x fasta_like_example.fsa in one grid call, bitwise equal to the
    reference's CPU scores (the benchmark_MSV.cpp loop shape)."""
    fa = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "fasta_like_example.fsa"))
    rows = read_golden_tsv("example_scores.tsv")
    engines = [engine(p) for p in PROFILES]
    grid = msv.score_grid(engines, fa.sequences)
    assert grid.shape == (len(PROFILES), len(fa.sequences))
    for k, prof in enumerate(PROFILES):
        want = np.array([w for p, i, L, w in rows if p == prof], np.float32)
        assert np.array_equal(bits(grid[k]), bits(want)), prof


def test_score_grid_random_fasta_and_seeded():
    fa = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "random_FASTA.fsa"))
    rows = read_golden_tsv("random_fasta_scores.tsv")
    engines = [engine(p) for p in PROFILES]
    grid = msv.score_grid(engines, fa.sequences)
    for k, prof in enumerate(PROFILES):
        want = np.array([w for p, i, L, w in rows if p == prof], np.float32)
        assert np.array_equal(bits(grid[k]), bits(want)), prof
    codes, offsets = random_batch(31, 300, 0, 900)
    sub = ["100.hmm", "1400.hmm", "2405.hmm", "100.hmm"]  # a repeated profile serialises on its stream
    grid = msv.score_grid([engine(p) for p in sub], codes=codes, offsets=offsets)
    for k, prof in enumerate(sub):
        assert np.array_equal(bits(grid[k]), bits(engine(prof).score_batch(codes=codes, offsets=offsets))), prof


def test_score_grid_fused_launch_matches_per_profile():
    """A grid of few sequences runs as ONE launch over all profiles, in chunks of 32 profiles.  Here 32 x 50
    workgroups per launch exceed the smallest profile's cooperative limit (coop_max_n), so the
    launch takes the round-2 latency layout of the largest model (msv_grid_kernel, grid_fused): 40 entries
    (all 24 profiles, 16 of them twice) x 50 random + homolog sequences equal every profile's own launch
    bitwise, and the oracle."""
    rc, ro = random_batch(150, 40, 0, 900)
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path("1400.hmm")).match_emissions, 151, 10, 1, 600)
    codes, offsets = concat_batches((rc, ro), (hc, ho))
    names = list(PROFILES) + list(PROFILES[:16])
    engines = [engine(p) for p in names]
    grid = msv.score_grid(engines, codes=codes, offsets=offsets)
    assert grid.shape == (40, 50)
    for k, prof in enumerate(names):
        assert np.array_equal(bits(grid[k]), bits(engine(prof).score_batch(codes=codes, offsets=offsets))), prof
    for prof in ("100.hmm", "1400.hmm", "2405.hmm"):
        want = OracleProfile(prof).score_batch(codes, offsets)
        assert np.array_equal(bits(grid[names.index(prof)]), bits(want)), prof


@pytest.mark.parametrize("coop_limit", [None, 0])
def test_score_grid_small_grid_cooperative_or_latency_fused(coop_limit):
    """benchmark_MSV's shape (every profile x 3 sequences, 72 workgroups per launch) runs the fused
    cooperative grid (msv_coop_grid_kernel); with one profile's cooperative limit set to 0
    (msv_debug_set_coop_max_n) the same grid takes the latency-layout fused launch (msv_grid_kernel) for
    profiles of <= 2480 states.  Either way every score equals the profile's own launch and the golden."""
    import ctypes as C
    from hmm_fasta_viterbi_amd import _native
    fa = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "random_FASTA.fsa"))
    rows = read_golden_tsv("random_fasta_scores.tsv")
    names = [p for p in PROFILES if int(p.split(".")[0]) <= 2480]
    engines = [msv.MSV_HMM(msv.Profile_HMM(profile_path(p))) for p in names]
    if coop_limit is not None:
        _native.lib().msv_debug_set_coop_max_n.argtypes = [C.c_void_p, C.c_uint64]
        _native.lib().msv_debug_set_coop_max_n(engines[3]._p, coop_limit)
    grid = msv.score_grid(engines, fa.sequences)
    for k, prof in enumerate(names):
        want = np.array([w for p, i, L, w in rows if p == prof], np.float32)
        assert np.array_equal(bits(grid[k]), bits(want)), (prof, coop_limit)


@pytest.mark.parametrize("leng", [2600, 3500])
def test_score_grid_fused_big_layout(tmp_path, leng):
    """The fused grid launch in the latency layout of a model too large for LDS (split 64-lane layout at
    2600 states, BIG row-class layout at 3500), shared by small profiles: equal to per-profile launches."""
    from hmm_fasta_viterbi_amd.synthetic import write_hmm
    path = str(tmp_path / f"syn{leng}.hmm")
    write_hmm(path, leng, leng)
    big = msv.MSV_HMM(msv.Profile_HMM(path))
    engines = [big, engine("100.hmm"), engine("1400.hmm"), engine("2405.hmm")]
    codes, offsets = random_batch(190 + leng, 30, 0, 800)
    grid = msv.score_grid(engines, codes=codes, offsets=offsets)
    for k, e in enumerate(engines):
        assert np.array_equal(bits(grid[k]), bits(e.score_batch(codes=codes, offsets=offsets))), k
    assert np.array_equal(bits(grid[0]), bits(OracleProfile(path).score_batch(codes, offsets)))
    big.close()


def test_score_grid_pinned_buffers():
    """Page-locked residues (read in place) and a page-locked destination (written by the kernels),
    fused (few sequences) and per-profile (many) grid launches: equal to the pageable call."""
    names = ["100.hmm", "700.hmm", "1400.hmm", "2405.hmm"]
    engines = [engine(p) for p in names]
    for n in (40, 3000):
        codes, offsets = random_batch(160 + n, n, 0, 700)
        want = msv.score_grid(engines, codes=codes, offsets=offsets)
        pc = msv.pinned_empty(codes.size, np.uint8)
        pc[:] = codes
        out = msv.pinned_empty((len(names), n), np.float32)
        got = msv.score_grid(engines, codes=pc, offsets=offsets, out=out)
        assert got is out
        assert np.array_equal(bits(out), bits(want)), n


def test_score_grid_bad_residue_reported_then_cleared():
    """A bad residue in a grid call raises (read from the call's +inf scores, then the profiles' latched
    words are read back and cleared), and the next grid call on good input succeeds bitwise."""
    codes, offsets = random_batch(33, 200, 1, 400)
    sub = [engine(p) for p in ("200.hmm", "1400.hmm", "2405.hmm")]
    want = msv.score_grid(sub, codes=codes, offsets=offsets)
    bad = codes.copy()
    bad[int(offsets[17]) + 1] = 200
    with pytest.raises(IndexError):
        msv.score_grid(sub, codes=bad, offsets=offsets)
    assert np.array_equal(bits(msv.score_grid(sub, codes=codes, offsets=offsets)), bits(want))
    for e in sub:
        e.check()


def test_score_grid_device_torch_stream():
    import torch
    codes, offsets = random_batch(32, 2000, 1, 700)
    sub = [engine(p) for p in ("300.hmm", "1901.hmm", "2207.hmm")]
    for e in sub:
        e.reserve_length(700)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    out = torch.full((len(sub), len(offsets) - 1), float("nan"), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    msv.score_grid_device(sub, r.data_ptr(), r.numel(), o.data_ptr(), len(offsets) - 1, out.data_ptr(),
                          None, st.cuda_stream)
    st.synchronize()
    for e in sub:
        e.check(st.cuda_stream)
    got = out.cpu().numpy()
    for k, e in enumerate(sub):
        assert np.array_equal(bits(got[k]), bits(e.score_batch(codes=codes, offsets=offsets)))


def test_pvalues_match_every_profiles_calibration():
    """Statistical pin of the P-value pipeline on all 24 profiles: 20k iid background sequences of length
    200 (what HMMER3's p7_MSVMu scores to fit STATS LOCAL MSV mu) scored on the GPU give P-values that
    are ~uniform, and a Gumbel mu refitted to our bit scores (lambda fixed) lands within 0.75 bits of the
    file's mu (measured -0.07 .. +0.50: the reference's float MSV scores slightly above HMMER's 8-bit
    calibration filter; profiles/r02_pvalue_calibration.jsonl).  A unit, sign or null-model error would
    miss by orders of magnitude."""
    from hmm_fasta_viterbi_amd.synthetic import background_batch
    codes, offsets = background_batch(2024, 20_000, 200)
    for prof in PROFILES:
        e = engine(prof)
        pv = e.pvalues(e.score_batch(codes=codes, offsets=offsets), offsets)
        mu, lam = e.msv_mu, e.msv_lambda
        b = mu - np.log(-np.log1p(-pv)) / lam
        mu_fit = -np.log(np.mean(np.exp(-lam * b))) / lam
        assert abs(mu_fit - mu) < 0.75, (prof, mu, mu_fit)
        for t in (0.5, 0.1, 0.01):
            assert t / 2.5 < float(np.mean(pv < t)) < t * 2.5, (prof, t, float(np.mean(pv < t)))


@pytest.mark.parametrize("length,n", [(400, 10_000), (2000, 2_500)])
def test_pvalues_calibrated_at_the_bench_lengths(length, n):
    """the MSV filter where it is used -- iid background sequences of the bench's
    lengths (cfg3 ~400, cfg5 ~2000), not only HMMER's L = 200 sample -- still give ~uniform P-values and a
    refitted mu within 0.75 bits on all 24 profiles: the per-length N/C/J loops and null1 carry the
    calibration across lengths (profiles/r05_filter_length_composition.jsonl).  The bench's survivor
    fraction (7% cfg3, 11% cfg5 at F1 = 0.02) comes from its uniform-letter composition, not from length
    (tests/test_filter_composition.py)."""
    from hmm_fasta_viterbi_amd.synthetic import background_batch
    codes, offsets = background_batch(2024 + length, n, length)
    for prof in PROFILES:
        e = engine(prof)
        pv = e.pvalues(e.score_batch(codes=codes, offsets=offsets), offsets)
        mu, lam = e.msv_mu, e.msv_lambda
        b = mu - np.log(-np.log1p(-pv)) / lam
        mu_fit = -np.log(np.mean(np.exp(-lam * b))) / lam
        assert abs(mu_fit - mu) < 0.75, (prof, length, mu, mu_fit)
        for t in (0.5, 0.1, 0.01):
            assert t / 2.5 < float(np.mean(pv < t)) < t * 2.5, (prof, length, t, float(np.mean(pv < t)))


def test_pvalues_device_matches_host():
    """the device P-value kernel equals the host formula (float64 libm vs device
    libm: 1e-13 relative), on GPU scores of a seeded batch, and msv_filter's pass mask uses it."""
    import torch
    e = engine("1400.hmm")
    codes, offsets = random_batch(41, 3000, 0, 600)
    sc, pv, passed = e.msv_filter(codes=codes, offsets=offsets)
    assert passed.dtype == bool and np.array_equal(passed, pv <= 0.02)
    dev = torch.device("cuda:0")
    d_sc = torch.from_numpy(sc).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    d_pv = torch.zeros(len(sc), dtype=torch.float64, device=dev)
    st = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    e.pvalues_device(d_sc.data_ptr(), d_off.data_ptr(), len(sc), d_pv.data_ptr(), st.cuda_stream)
    st.synchronize()
    np.testing.assert_allclose(d_pv.cpu().numpy(), pv, rtol=1e-13, atol=0)


@pytest.mark.parametrize("n", [1, 1000, 16384, 16385, 200_000])
def test_order_longest_first_sizes(n):
    """Both order paths (one-launch small sort up to 16384, two-launch sort above: count + scan by the
    last block, then place) give a permutation in non-increasing length order (lengths >= 4095 share
    the first bin)."""
    import torch
    e = engine("100.hmm")
    _, offsets = random_batch(50 + n % 7, n, 0, 5000)
    dev = torch.device("cuda:0")
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    order = torch.full((n,), -1, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    e.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
    st.synchronize()
    perm = order.cpu().numpy().astype(np.int64)
    assert np.array_equal(np.sort(perm), np.arange(n))
    lens = np.minimum(np.diff(offsets.astype(np.int64))[perm], 4095)
    assert np.all(lens[:-1] >= lens[1:])


def test_order_back_to_back_sorts_reuse_scratch():
    """Sorts queued back to back on one stream with no sync between them: each must find the
    histogram and the last-block ticket that the previous sort left zeroed (no memset between)."""
    import torch
    e = engine("100.hmm")
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    cases = []
    rng = np.random.default_rng(90)
    for n in [200_000, 16_385, 70_001, 200_000, 1_000_003, 33_333]:
        lens = rng.integers(0, 5000, n, dtype=np.uint64)  # the sort reads offsets only
        offsets = np.concatenate([np.zeros(1, np.uint64), np.cumsum(lens, dtype=np.uint64)])
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        order = torch.full((n,), -1, dtype=torch.int32, device=dev)
        cases.append((offsets, o, order))
    torch.cuda.synchronize()
    for _, o, order in cases:
        e.order_longest_first(o.data_ptr(), len(order), order.data_ptr(), st.cuda_stream)
    st.synchronize()
    for offsets, _, order in cases:
        n = len(order)
        perm = order.cpu().numpy().astype(np.int64)
        assert np.array_equal(np.sort(perm), np.arange(n))
        lens = np.minimum(np.diff(offsets.astype(np.int64))[perm], 4095)
        assert np.all(lens[:-1] >= lens[1:])


def test_back_to_back_launches_self_reset_counter():
    """The dequeue counter is reset by the last wave of each launch (no memset between launches):
    many launches of different sizes and grids on one stream, then a variant switch."""
    import torch
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("700.hmm")))
    e.reserve_length(900)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    batches = [random_batch(60 + k, n, 0, 900) for k, n in enumerate((5, 70_000, 1, 3000, 70_000, 17))]
    outs = []
    for codes, offsets in batches:
        r = torch.from_numpy(codes).to(dev)
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        s = torch.empty(len(offsets) - 1, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), len(offsets) - 1, s.data_ptr(), None,
                             st.cuda_stream)
        outs.append((r, o, s))
    e.check(st.cuda_stream)
    for (codes, offsets), (_, _, s) in zip(batches, outs):
        want = OracleProfile("700").score_batch(*subset(codes, offsets, np.arange(0, len(offsets) - 1, 97)))
        got = s.cpu().numpy()[np.arange(0, len(offsets) - 1, 97)]
        assert np.array_equal(bits(got), bits(want))
    e.set_variant("msv_g16_s48_w12_p2_d1")
    codes, offsets = batches[1]
    got = e.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(outs[1][2].cpu().numpy()))
    e.close()


def test_score_batch_multi_shards_match_single():
    """msv_score_batch_multi: shards scored concurrently by one host thread per profile (here
    several profiles on the available device(s)), bitwise equal to one launch, input order kept."""
    prof = msv.Profile_HMM(profile_path("1400.hmm"))
    ndev = msv.device_count()
    engines = [msv.MSV_HMM(prof, device=k % ndev) for k in range(3)]
    codes, offsets = random_batch(71, 20_000, 0, 800)
    want = engine("1400.hmm").score_batch(codes=codes, offsets=offsets)
    got = msv.score_batch_multi(engines, codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))
    few = msv.score_batch_multi(engines, codes=codes[:int(offsets[2])], offsets=offsets[:3])  # n < shards
    assert np.array_equal(bits(few), bits(want[:2]))
    for e in engines:
        e.close()


def test_long_sequence_grows_length_table():
    """A 200k-residue sequence (beyond the default 131072-entry {tr_loop, tr_move} table): the host
    API grows the table (msv_profile_reserve_length) and the score matches the oracle."""
    codes, offsets = random_batch(81, 3, 1, 50)
    long = np.random.default_rng(5).integers(0, 20, 200_000, dtype=np.uint8)
    codes = np.concatenate([codes, long])
    offsets = np.append(offsets, offsets[-1] + np.uint64(len(long))).astype(np.uint64)
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("100.hmm")))
    got = e.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(OracleProfile("100").score_batch(codes, offsets)))
    e.close()


def test_device_api_latches_errors_and_keeps_other_scores():
    """Device path: a sequence longer than the reserved table -> MSV_ERR_SEQUENCE_TOO_LONG from
    check() (its slot NaN); a code >= 20 -> IndexError (its slot +inf); every other score exact."""
    import torch
    from hmm_fasta_viterbi_amd._native import MSVError
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("300.hmm")))
    codes, offsets = random_batch(82, 50, 1, 300)
    want = OracleProfile("300").score_batch(codes, offsets)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)

    def run(c, o):
        r = torch.from_numpy(c).to(dev)
        oo = torch.from_numpy(o.view(np.int64)).to(dev)
        s = torch.empty(len(o) - 1, dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        e.score_batch_device(r.data_ptr(), r.numel(), oo.data_ptr(), len(o) - 1, s.data_ptr(), None, st.cuda_stream)
        st.synchronize()
        return s

    bad = codes.copy()
    bad[int(offsets[7]) + 3] = 21
    s = run(bad, offsets)
    with pytest.raises(IndexError):
        e.check(st.cuda_stream)
    got = s.cpu().numpy()
    assert np.isposinf(got[7])
    keep = np.arange(50) != 7
    assert np.array_equal(bits(got[keep]), bits(want[keep]))
    e.check(st.cuda_stream)  # cleared

    n_tab = 131072
    long = np.zeros(n_tab + 5, np.uint8)
    c2 = np.concatenate([codes, long])
    o2 = np.append(offsets, offsets[-1] + np.uint64(len(long))).astype(np.uint64)
    s = run(c2, o2)
    with pytest.raises(MSVError):
        e.check(st.cuda_stream)
    got = s.cpu().numpy()
    assert np.isnan(got[50])
    assert np.array_equal(bits(got[:50]), bits(want))
    e.close()


def _fasta_cases(tmp_path):
    """FASTA texts for device-vs-host ingest parity: the reference's files, the golden edge cases,
    a ~20 MB mixed file, one record on a single 300k-residue line, long headers across tiles, a
    header at EOF without newline, blank lines before the first header, CRLF, empty file."""
    rng = np.random.default_rng(17)
    letters = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    out = [os.path.join(ROOT, "data", "FASTA_files", f) for f in ("fasta_like_example.fsa", "random_FASTA.fsa")]
    out.append(os.path.join(GOLD, "edge_cases.fsa"))
    parts = []
    for i in range(40_000):
        L = int(rng.integers(0, 900))
        seq = letters[rng.integers(0, 20, L)].tobytes()
        kind = int(rng.integers(0, 30))
        if kind == 0:
            seq = seq[: L // 2] + b"z" + seq[L // 2:]
        elif kind == 1:
            seq = seq.replace(b"C", b"#", 1)
        eol = b"\r\n" if kind == 2 else b"\n"
        width = int(rng.integers(1, 120))
        lines = [seq[k:k + width] for k in range(0, len(seq), width)] or [b""]
        hdr = b"h%d " % i + (b"x" * int(rng.integers(0, 5000)) if kind == 3 else b"")
        parts.append(b">" + hdr + eol + eol.join(lines) + eol + (b"\n\n" if kind == 4 else b""))
    blobs = {
        "mixed.fsa": b"".join(parts),
        "oneline.fsa": b">big one\n" + letters[rng.integers(0, 20, 300_000)].tobytes() + b"\n>tail",
        "preblank.fsa": b"\n\n\n>a\nACD\n\n>b\n\nEF\n",
        "crlf_end.fsa": b">a\r\nACDE\r\n>b\r\nKLM",
        "headers_only.fsa": b">a\n>b\n>c",
        "empty.fsa": b"",
    }
    for name, blob in blobs.items():
        path = tmp_path / name
        path.write_bytes(blob)
        out.append(str(path))
    return out


def test_fasta_device_matches_host_reader(tmp_path):
    """the GPU FASTA parse (tile scans) yields exactly the host reader's records:
    codes, offsets, rejected count and headers (from the returned spans)."""
    for path in _fasta_cases(tmp_path):
        host = msv.FASTA_protein_sequences(path)
        dev = msv.FASTA_device(path)
        codes, offsets, spans = dev.download()
        assert dev.count == len(host.offsets) - 1 and dev.rejected == host.rejected, path
        assert np.array_equal(offsets, host.offsets), path
        assert np.array_equal(codes, host.codes), path
        text = open(path, "rb").read()
        hdrs = [text[int(a):int(a) + int(b)].decode("latin-1") for a, b in spans]
        assert hdrs == host.headers, path
        dev.close()


def test_fasta_device_parse_errors_like_host(tmp_path):
    bad = tmp_path / "bad.fsa"
    bad.write_bytes(b"\nACDE\n>a\nAC\n")
    from hmm_fasta_viterbi_amd._native import MSVError
    with pytest.raises(MSVError):
        msv.FASTA_protein_sequences(str(bad))
    with pytest.raises(MSVError):
        msv.FASTA_device(str(bad))
    with pytest.raises(MSVError):
        msv.FASTA_device(str(tmp_path / "missing.fsa"))


def test_fasta_device_to_scores_end_to_end(tmp_path):
    """File bytes -> GPU parse -> GPU scores, with no host parse: equal to the host path's scores."""
    import torch
    codes, offsets = random_batch(91, 30_000, 0, 700)
    path = tmp_path / "batch.fsa"
    from hmm_fasta_viterbi_amd.synthetic import write_fasta
    write_fasta(str(path), codes, offsets)
    e = engine("1400.hmm")
    e.reserve_length(700)
    dev = msv.FASTA_device(str(path))
    s = torch.empty(dev.count, dtype=torch.float32, device="cuda:0")
    st = torch.cuda.Stream(torch.device("cuda:0"))
    torch.cuda.synchronize()
    e.score_batch_device(dev.codes_ptr, dev.residues, dev.offsets_ptr, dev.count, s.data_ptr(), None, st.cuda_stream)
    e.check(st.cuda_stream)
    assert np.array_equal(bits(s.cpu().numpy()), bits(e.score_batch(codes=codes, offsets=offsets)))
    dev.close()


def test_score_fasta_device_with_rejections_and_bad_residue(tmp_path):
    """msv_score_fasta_device on a GPU-parsed file: rejected records dropped exactly like the host
    reader, scores equal the host path's, a '#' inside a kept record raises like the reference."""
    rng = np.random.default_rng(23)
    letters = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    parts = []
    for i in range(5000):
        seq = letters[rng.integers(0, 20, int(rng.integers(0, 600)))].tobytes()
        if i % 17 == 0:
            seq += b"b"  # rejected record
        parts.append(b">s%d\n" % i + seq + b"\n")
    path = tmp_path / "r.fsa"
    path.write_bytes(b"".join(parts))
    host = msv.FASTA_protein_sequences(str(path))
    dev = msv.FASTA_device(str(path))
    e = engine("700.hmm")
    assert dev.count == len(host) and dev.rejected == host.rejected > 0
    assert dev.max_length == int(np.diff(host.offsets.astype(np.int64)).max())
    assert np.array_equal(bits(e.score_fasta_device(dev)), bits(e.score_batch(codes=host.codes, offsets=host.offsets)))
    bad = tmp_path / "hash.fsa"
    bad.write_bytes(b">a\nACD#EF\n>b\nKLM\n")
    with pytest.raises(IndexError):
        e.score_fasta_device(msv.FASTA_device(str(bad)))


@pytest.mark.parametrize("prof", ["100", "700", "1400", "1901", "2405"])
def test_latency_plan_small_batches_match_main_plan(prof):
    """Batches of <= 2048 sequences run the latency plan (one sequence per 64-lane wave); it must
    give the main plan's bits (forced with set_variant) and the oracle's."""
    codes, offsets = random_batch(101, 700, 0, 900)
    auto = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
    got = auto.score_batch(codes=codes, offsets=offsets)
    forced = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
    forced.set_variant(forced.describe()["variant"])
    assert np.array_equal(bits(got), bits(forced.score_batch(codes=codes, offsets=offsets)))
    sample = np.arange(0, 700, 23)
    assert np.array_equal(bits(got[sample]), bits(OracleProfile(prof).score_batch(*subset(codes, offsets, sample))))
    auto.close()
    forced.close()


@pytest.mark.parametrize("prof", ["600", "900", "1001", "1400", "1509"])
def test_mid_plan_batches_match_main_plan(prof):
    """Batches between the latency plan's limit and one round of the main grid run the 32-lane mid
    plan (large G = 16 profiles); random and homolog sequences (J >= N rows), empty ones included,
    give the main plan's bits and the oracle's."""
    auto = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
    d = auto.describe()
    assert d["mid_variant"].startswith("msv_g32_") and d["latency_max_n"] < d["mid_max_n"]
    n = (d["latency_max_n"] + d["mid_max_n"]) // 2
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path(prof + ".hmm")).match_emissions, 131, 200, 1, 600)
    codes, offsets = concat_batches(random_batch(130, n - 200, 0, 800), (hc, ho))
    got = auto.score_batch(codes=codes, offsets=offsets)
    forced = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
    forced.set_variant(d["variant"])
    assert np.array_equal(bits(got), bits(forced.score_batch(codes=codes, offsets=offsets)))
    sample = np.concatenate([np.arange(0, n, n // 40), np.arange(n - 200, n, 10)])
    assert np.array_equal(bits(got[sample]), bits(OracleProfile(prof).score_batch(*subset(codes, offsets, sample))))
    auto.close()
    forced.close()


def test_narrow_plan_full_batches_match():
    """100.hmm: batches that fill the SIMDs run 4-lane groups (16 sequences per wave), smaller ones the
    16-lane plan; both sizes equal a forced 16-lane launch bitwise, and an oracle sample."""
    auto = msv.MSV_HMM(msv.Profile_HMM(profile_path("100.hmm")))
    d = auto.describe()
    forced = msv.MSV_HMM(msv.Profile_HMM(profile_path("100.hmm")))
    forced.set_variant(d["mid_variant"])
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path("100.hmm")).match_emissions, 141, 300, 1, 600)
    for n in (d["mid_max_n"] - 300, d["mid_max_n"] + 20_000):
        codes, offsets = concat_batches(random_batch(140 + n, n, 0, 900), (hc, ho))
        assert auto.variant_for(n + 300) == (d["mid_variant"] if n + 300 <= d["mid_max_n"] else d["variant"])
        got = auto.score_batch(codes=codes, offsets=offsets)
        assert np.array_equal(bits(got), bits(forced.score_batch(codes=codes, offsets=offsets))), n
        sample = np.concatenate([np.arange(0, n, n // 50), np.arange(n, n + 300, 7)])
        assert np.array_equal(bits(got[sample]), bits(OracleProfile("100").score_batch(*subset(codes, offsets, sample))))
    auto.close()
    forced.close()


@pytest.mark.parametrize("prof", ["200", "400", "500"])
def test_whole_row_ring_plan_matches(prof):
    """200-500-state profiles: full batches run a whole-row-ring variant, smaller ones the PF-2 variant;
    both sizes equal a forced PF-2 launch bitwise, and an oracle sample."""
    auto = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
    d = auto.describe()
    assert d["variant"] != d["mid_variant"] and d["mid_max_n"] > 0
    forced = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
    forced.set_variant(d["mid_variant"])
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path(prof + ".hmm")).match_emissions, 171, 200, 1, 600)
    for n in (d["mid_max_n"] - 200, d["mid_max_n"] + 10_000):
        codes, offsets = concat_batches(random_batch(170 + n, n, 0, 900), (hc, ho))
        got = auto.score_batch(codes=codes, offsets=offsets)
        assert np.array_equal(bits(got), bits(forced.score_batch(codes=codes, offsets=offsets))), n
        sample = np.concatenate([np.arange(0, n, n // 40), np.arange(n, n + 200, 9)])
        assert np.array_equal(bits(got[sample]), bits(OracleProfile(prof).score_batch(*subset(codes, offsets, sample))))
    auto.close()
    forced.close()


def test_score_batch_multi_concurrent_length_table_growth():
    """Each shard holds a sequence longer than the default length table, so every host thread of
    msv_score_batch_multi grows its profile's table at once (shared host cache under a lock)."""
    prof = msv.Profile_HMM(profile_path("100.hmm"))
    ndev = msv.device_count()
    engines = [msv.MSV_HMM(prof, device=k % ndev) for k in range(4)]
    rng = np.random.default_rng(13)
    lens = [140_000 + 1000 * k for k in range(4)]
    codes = rng.integers(0, 20, sum(lens), dtype=np.uint8)
    offsets = np.zeros(5, np.uint64)
    offsets[1:] = np.cumsum(lens)
    got = msv.score_batch_multi(engines, codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(OracleProfile("100").score_batch(codes, offsets)))
    for e in engines:
        e.close()


def _homolog_j_rows(codes, offsets, scores):
    """How many sequences end with J >= N (so B took J at least on the last row)."""
    L = np.diff(offsets).astype(np.float64)
    ok = L > 0
    move = np.log(3.0 / (L[ok] + 3.0))
    return int(((scores[ok] - move) >= L[ok] * np.log(L[ok] / (L[ok] + 3.0)) + 1e-3).sum())


@pytest.mark.parametrize("prof", ["100", "500", "1400", "1901", "2405"])
def test_homolog_sequences_match_oracle(prof):
    """Sequences emitted by the profile itself (high scores: J >= N on many rows, so B depends on
    the group-wide J), mixed with random ones in the same waves, under the automatic variant and
    the latency plan's batch sizes, bitwise against the oracle."""
    e = engine(prof)
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path(prof)).match_emissions, 5, 300, 1, 700)
    rc, ro = random_batch(6, 300, 1, 700)
    codes, offsets = concat_batches((hc, ho), (rc, ro))
    want = OracleProfile(prof).score_batch(codes, offsets)
    assert _homolog_j_rows(hc, ho, want[:300]) > 150, "homolog batch no longer exercises J >= N"
    got = e.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))
    small = e.score_batch(codes=hc[: int(ho[8])], offsets=ho[:9])  # latency-plan sized batch
    assert np.array_equal(bits(small), bits(want[:8]))


def _numpy_msv(es, tBMk, tEC, tEJ, codes, offsets):
    """float32 restatement of MSV_HMM::run_on_sequence (MSV_HMM.cpp:74-113) with free tr_E_C /
    tr_E_J (the reference fixes both to logf(0.5f)); every add is one IEEE float32 op in the
    reference's order, max is exact, so results are bit-comparable."""
    f = np.float32
    out = np.zeros(len(offsets) - 1, np.float32)
    for s in range(len(offsets) - 1):
        seq = codes[int(offsets[s]):int(offsets[s + 1])]
        L = len(seq)
        loop, move = msv.sequence_transitions(L)
        loop, move = f(loop), f(move)
        M = np.full(es.shape[1], -np.inf, np.float32)
        J = C = f(-np.inf)
        N, B = f(0.0), move
        for r in seq:
            Bt = f(B + f(tBMk))
            newM = np.full_like(M, -np.inf)
            newM[1:] = es[r, 1:] + np.maximum(M[:-1], Bt)
            M = newM
            E = M[1:].max()
            J = max(f(J + loop), f(E + f(tEJ)))
            C = max(f(C + loop), f(E + f(tEC)))
            N = f(N + loop)
            B = f(max(N, J) + move)
        out[s] = f(C + move) if L else -np.inf
    return out


def test_distinct_tr_E_C_and_tr_E_J():
    """The C-ABI accepts tr_E_C != tr_E_J (no reference profile has that): the kernel then keeps
    separate C partials instead of reading C from J."""
    import ctypes as C
    from hmm_fasta_viterbi_amd import _native
    L = _native.lib()
    h = msv.Profile_HMM(profile_path("100"))
    es, tBMk, _, _ = h.msv_scores()
    es = np.ascontiguousarray(es, np.float32)
    hc, ho = homolog_batch(h.match_emissions, 9, 12, 1, 60)
    rc, ro = random_batch(10, 12, 0, 60)
    codes, offsets = concat_batches((hc, ho), (rc, ro))
    for tEC, tEJ in ((-0.3, -1.2), (-2.0, -0.1)):
        want = _numpy_msv(es, tBMk, tEC, tEJ, codes, offsets)
        p = C.c_void_p()
        assert L.msv_profile_create(0, es.ctypes.data, es.shape[1], tBMk, tEC, tEJ, C.byref(p)) == 0
        try:
            got = np.zeros(len(offsets) - 1, np.float32)
            assert L.msv_score_batch(p, codes.ctypes.data, offsets.ctypes.data, len(got), got.ctypes.data, None) == 0
        finally:
            L.msv_profile_destroy(p)
        assert np.array_equal(bits(got), bits(want)), (tEC, tEJ)
    # and the numpy restatement itself agrees with the oracle at the reference's constants
    _, _, tEC0, tEJ0 = h.msv_scores()
    assert np.array_equal(bits(_numpy_msv(es, tBMk, tEC0, tEJ0, codes, offsets)),
                          bits(OracleProfile("100").score_batch(codes, offsets)))


@pytest.mark.parametrize("prof", ["100", "400", "1001", "1400", "1901", "2405"])
def test_coop_plan_edges_and_homologs(prof):
    """The cooperative plan (msv_coop.hip: one sequence per workgroup, its row over 4 waves with halo
    states and a speculated B) takes batches of up to one workgroup per CU.  Lengths around its
    16-row blocks (0, 1, 15, 16, 17, 31, 32, 33, ...) and up to 3500, homologs (J >= N rows: the
    rolled-back blocks and exact rows), bitwise against the oracle; a bad residue raises.  1901 and
    2405.hmm take the split form (each lane's last states read from a global table per row)."""
    e = engine(prof)
    info = e.describe()
    assert info["coop_variant"].startswith("msv_coop") and info["coop_max_n"] >= 64
    assert ("_a" in info["coop_variant"]) == (int(prof) > 1464)
    assert e.variant_for(1) == info["coop_variant"] and e.variant_for(info["coop_max_n"] + 1) != info["coop_variant"]
    rng = np.random.default_rng(int(prof))
    lens = [0, 1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 63, 100, 255, 256, 257, 1000, 3500]
    parts = [rng.integers(0, 20, L, dtype=np.uint8) for L in lens]
    ec = np.concatenate(parts)
    eo = np.zeros(len(lens) + 1, np.uint64)
    eo[1:] = np.cumsum(lens)
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path(prof)).match_emissions, 7, 40, 16, 900)
    codes, offsets = concat_batches((ec, eo), (hc, ho))
    want = OracleProfile(prof).score_batch(codes, offsets)
    got = e.score_batch(codes=codes, offsets=offsets)
    assert len(lens) + 40 <= info["coop_max_n"]
    assert np.array_equal(bits(got), bits(want))
    for k in range(len(lens) + 40):  # one sequence per call: the reference's benchmark shape
        if k % 7 == 0:
            one = e.score_batch(codes=codes[int(offsets[k]):int(offsets[k + 1])],
                                offsets=np.array([0, offsets[k + 1] - offsets[k]], np.uint64))
            assert bits(one)[0] == bits(want)[k], k
    bad = codes.copy()
    bad[int(offsets[len(lens) - 1]) + 1234] = 20
    with pytest.raises(IndexError):
        e.score_batch(codes=bad, offsets=offsets)
    assert np.array_equal(bits(e.score_batch(codes=codes, offsets=offsets)), bits(want))


def test_coop_plan_several_sequences_per_workgroup():
    """At its largest batch (two rounds of the grid on 1400.hmm) each workgroup scores sequences in turn."""
    e = engine("1400.hmm")
    info = e.describe()
    n = info["coop_max_n"]
    assert n > info["coop_blocks"] and e.variant_for(n) == info["coop_variant"]
    codes, offsets = random_batch(91, n, 0, 300)
    want = OracleProfile("1400").score_batch(codes, offsets, threads=min(16, len(os.sched_getaffinity(0))))
    assert np.array_equal(bits(e.score_batch(codes=codes, offsets=offsets)), bits(want))


def test_coop_plan_reference_benchmark_shape():
    """benchmark_MSV_1400 (benchmark_MSV_1400.cpp:8-13): 1400.hmm x random_FASTA.fsa, one
    parallel_run_on_sequence per sequence, each bitwise equal to the golden score."""
    e = engine("1400.hmm")
    gold = {(p, i): sc for p, i, _, sc in read_golden_tsv("random_fasta_scores.tsv")}
    seqs = msv.FASTA_protein_sequences(os.path.join(ROOT, "data", "FASTA_files", "random_FASTA.fsa")).sequences
    assert e.variant_for(1).startswith("msv_coop") and len(seqs) == 3
    for k, s in enumerate(seqs):
        got = e.parallel_run_on_sequence(s)
        assert bits([got])[0] == bits([gold[("1400.hmm", k)]])[0]


def test_coop_plan_device_order_async_and_shards():
    """The cooperative plan under the other entry points: a caller's dequeue order on device buffers (a
    valid permutation scores exactly, an entry >= n is reported as MSV_ERR_INVALID_ARGUMENT), the
    asynchronous host path (no sort for one sequence per workgroup), and residue-balanced shards of a
    small batch through msv_score_batch_multi -- all bitwise against the oracle."""
    import torch
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1001.hmm")))
    n = 120
    assert e.variant_for(n).startswith("msv_coop")
    codes, offsets = random_batch(93, n, 0, 700)
    want = OracleProfile("1001").score_batch(codes, offsets)
    dev = torch.device("cuda:0")
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.zeros(n, dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    perm = torch.from_numpy(np.random.default_rng(5).permutation(n).astype(np.int32)).to(dev)
    torch.cuda.synchronize()
    e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), perm.data_ptr(), st.cuda_stream)
    e.check(st.cuda_stream)
    assert np.array_equal(bits(s.cpu().numpy()), bits(want))
    bad = perm.clone()
    bad[17] = n + 3
    e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), bad.data_ptr(), st.cuda_stream)
    with pytest.raises(msv.MSVError) as ex:
        e.check(st.cuda_stream)
    assert ex.value.name == "MSV_ERR_INVALID_ARGUMENT"
    out = np.zeros(n, np.float32)
    t = e.score_batch_async(codes, offsets, out)
    assert np.array_equal(bits(e.wait(t)), bits(want))
    engines = [msv.MSV_HMM(msv.Profile_HMM(profile_path("1001.hmm")), device=0) for _ in range(3)]
    assert np.array_equal(bits(msv.score_batch_multi(engines, codes=codes, offsets=offsets)), bits(want))
    for x in engines:
        x.close()
    e.close()


@pytest.mark.parametrize("prof", PROFILES)
def test_every_plan_of_every_profile(prof):
    """Every kernel plan a profile installs (cooperative, latency, mid, throughput -- msv_profile_describe),
    each at the largest batch that takes it and the main plan beyond them, as HBM-resident launches with
    the longest-first order: the plan named by variant_for(n) runs, and its scores equal the oracle on a
    sample of each batch that includes the longest and shortest sequences (lengths U[0,700])."""
    import torch
    e = engine(prof)
    info = e.describe()
    sizes = {1}
    for key in ("coop_max_n", "latency_max_n", "mid_max_n"):
        if info[key]:
            sizes.add(int(info[key]))
    sizes.add(max(sizes) + 2000)
    o = OracleProfile(prof)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    names = {info["coop_variant"], info["latency_variant"], info["mid_variant"], info["variant"]} - {""}
    ran = set()
    for k, n in enumerate(sorted(sizes)):
        codes, offsets = random_batch(7000 + 31 * k + int(prof.split(".")[0]), n, 0, 700)
        ran.add(e.variant_for(n))
        r = torch.from_numpy(codes).to(dev)
        off = torch.from_numpy(offsets.view(np.int64)).to(dev)
        s = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
        order = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        e.order_longest_first(off.data_ptr(), n, order.data_ptr(), st.cuda_stream)
        e.score_batch_device(r.data_ptr(), r.numel(), off.data_ptr(), n, s.data_ptr(), order.data_ptr(), st.cuda_stream)
        e.check(st.cuda_stream)
        got = s.cpu().numpy()
        lens = np.diff(offsets.astype(np.int64))
        rng = np.random.default_rng(n)
        idx = np.unique(np.concatenate([[int(np.argmax(lens)), int(np.argmin(lens)), 0, n - 1],
                                        rng.choice(n, min(n, 150), replace=False)]))
        parts = [codes[int(offsets[i]):int(offsets[i + 1])] for i in idx]
        so = np.zeros(len(idx) + 1, np.uint64)
        so[1:] = np.cumsum([len(p) for p in parts])
        sc = np.concatenate(parts) if so[-1] else np.zeros(0, np.uint8)
        want = o.score_batch(sc, so, threads=min(16, len(os.sched_getaffinity(0))))
        assert np.array_equal(bits(got[idx]), bits(want)), (prof, n, e.variant_for(n))
    assert ran <= names and info["variant"] in ran, (prof, ran, names)
    assert not info["coop_max_n"] or info["coop_variant"] in ran
