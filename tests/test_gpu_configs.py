"""BASELINE.json's configs at full size on the GPU, the host-buffer pipeline, and the per-launch
counter slots.  Bitwise against the oracle (tests/oracle_lib.py) on samples, and through
size-independent properties (three scorings agree, determinism, permutation invariance) on the
whole batch.

  cfg4: 1400.hmm x 1,000,000 sequences, len U[300,500], seed 3 -- one launch, the host pipeline,
        8 residue-balanced shards through msv_score_batch_multi (the one device listed 8 times) and
        distributed.shard slices must all give the same bits, and EVERY score equals the oracle's
        (~5.6e11 cells on the host's threads).
  cfg2: 100.hmm x 10,000 sequences, len U[300,500] -- EVERY score bitwise against the oracle, for the
        config's seed (1) and for bench.py's rank-0 batch (seed 1000).
  cfg3: 1400.hmm x 100,000 sequences, len U[300,500] -- bench.py's rank-0 batch (seed 2000), EVERY
        score bitwise against the oracle (~56 G cells on the host's threads).
  cfg5: 2405.hmm x 100,000 sequences, len U[1500,2500], seed 4 -- the host path equals one launch,
        permutation invariance, and EVERY score equals the oracle's (~4.8e11 cells).
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import hmm_fasta_viterbi_amd as msv
from hmm_fasta_viterbi_amd import distributed
from hmm_fasta_viterbi_amd.synthetic import concat_batches, homolog_batch, random_batch
from oracle_lib import OracleProfile, bits, profile_path

ORACLE_THREADS = min(16, len(os.sched_getaffinity(0)))


def subset(codes, offsets, idx):
    parts = [codes[int(offsets[i]):int(offsets[i + 1])] for i in idx]
    offs = np.zeros(len(idx) + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts])
    return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), offs


def sample_with_extremes(offsets, k, seed):
    """k sequence indices: the longest, the shortest, the first and last, and a seeded spread."""
    lens = np.diff(offsets.astype(np.int64))
    n = len(lens)
    pick = {int(np.argmax(lens)), int(np.argmin(lens)), 0, n - 1}
    rng = np.random.default_rng(seed)
    pick.update(int(i) for i in rng.choice(n, k, replace=False))
    return np.array(sorted(pick), np.int64)


def device_scores(engine, codes, offsets, order=True):
    """One launch over the whole batch resident in HBM (torch tensors, caller stream)."""
    import torch
    dev = torch.device("cuda", engine.device)
    n = len(offsets) - 1
    r = torch.from_numpy(codes).to(dev)
    o = torch.from_numpy(offsets.view(np.int64)).to(dev)
    s = torch.full((n,), float("nan"), dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    engine.reserve_length(int(np.diff(offsets.astype(np.int64)).max()))
    ordp = None
    if order:
        ordt = torch.empty(n, dtype=torch.int32, device=dev)
        engine.order_longest_first(o.data_ptr(), n, ordt.data_ptr(), st.cuda_stream)
        ordp = ordt.data_ptr()
    engine.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), ordp, st.cuda_stream)
    engine.check(st.cuda_stream)
    return s.cpu().numpy()


@pytest.mark.timeout(900)
def test_cfg4_full_size_every_score():
    """cfg4 (1400.hmm x 1M, one set): one launch, the host pipeline, 8 shards through msv_score_batch_multi and
    the torch.distributed slices all bitwise equal, and every score equal to the oracle's."""
    prof = msv.Profile_HMM(profile_path("1400.hmm"))
    e = msv.MSV_HMM(prof)
    codes, offsets = random_batch(3, 1_000_000, 300, 500)
    assert int(offsets[-1]) < (1 << 32)
    one = device_scores(e, codes, offsets)                      # (a) one launch
    assert np.all(np.isfinite(one))
    host = e.score_batch(codes=codes, offsets=offsets)           # the host-buffer pipeline (pieces)
    assert np.array_equal(bits(host), bits(one))
    engines = [msv.MSV_HMM(prof, device=0) for _ in range(8)]    # (b) 8 shards, msv_score_batch_multi
    multi = msv.score_batch_multi(engines, codes=codes, offsets=offsets)
    assert np.array_equal(bits(multi), bits(one))
    bounds = msv.shard_bounds(offsets, 8)                        # (c) the torch.distributed split
    sliced = np.empty_like(one)
    for r in range(8):
        c, o, first, last = distributed.shard(codes, offsets, 8, r)
        assert (first, last) == (int(bounds[r]), int(bounds[r + 1]))
        sliced[first:last] = e.score_batch(codes=c, offsets=o)
    assert np.array_equal(bits(sliced), bits(one))
    # residue balance of the shards (BASELINE cfg4's 8-GPU split)
    res = np.diff(offsets[bounds.astype(np.int64)].astype(np.int64))
    assert res.max() - res.min() <= 2 * 500
    want = OracleProfile("1400").score_batch(codes, offsets, threads=ORACLE_THREADS)  # every score
    assert np.array_equal(bits(one), bits(want))
    for x in engines:
        x.close()
    e.close()


@pytest.mark.parametrize("seed", [1, 1000])
def test_cfg2_full_size_every_score(seed):
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("100.hmm")))
    codes, offsets = random_batch(seed, 10_000, 300, 500)
    got = device_scores(e, codes, offsets)
    want = OracleProfile("100").score_batch(codes, offsets, threads=ORACLE_THREADS)
    assert np.array_equal(bits(got), bits(want))
    assert np.array_equal(bits(e.score_batch(codes=codes, offsets=offsets)), bits(want))  # host pipeline
    e.close()


def test_cfg3_full_size_every_score():
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400.hmm")))
    codes, offsets = random_batch(2000, 100_000, 300, 500)  # bench.py --config cfg3, rank 0
    got = device_scores(e, codes, offsets)
    want = OracleProfile("1400").score_batch(codes, offsets, threads=ORACLE_THREADS)
    assert np.array_equal(bits(got), bits(want))
    e.close()


@pytest.mark.timeout(900)
def test_cfg5_full_size_every_score():
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("2405.hmm")))
    codes, offsets = random_batch(4, 100_000, 1500, 2500)
    a = e.score_batch(codes=codes, offsets=offsets)
    b = device_scores(e, codes, offsets)
    assert np.array_equal(bits(a), bits(b))
    assert np.all(np.isfinite(a))
    perm = np.random.default_rng(1).permutation(100_000)[:5000]
    pc, po = subset(codes, offsets, perm)
    assert np.array_equal(bits(e.score_batch(codes=pc, offsets=po)), bits(a[perm]))
    want = OracleProfile("2405").score_batch(codes, offsets, threads=ORACLE_THREADS)  # every score
    assert np.array_equal(bits(a), bits(want))
    e.close()


def test_host_pipeline_piece_edges():
    """msv_score_batch over >= 4 Mi residues runs as pieces on two compute streams + a copy stream:
    empty records, a long record and homologs placed around the piece cuts; pinned (torch
    pin_memory) and pageable sources; equal to one device launch."""
    import torch
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("700.hmm")))
    rc, ro = random_batch(201, 12_000, 0, 900)
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path("700.hmm")).match_emissions, 202, 400, 1, 900)
    long = np.random.default_rng(3).integers(0, 20, 150_000, dtype=np.uint8)
    lc, lo = long, np.array([0, long.size], np.uint64)
    empty = (np.zeros(0, np.uint8), np.zeros(2001, np.uint64))
    codes, offsets = concat_batches((rc, ro), empty, (lc, lo), (hc, ho), (rc, ro), empty)
    assert int(offsets[-1]) >= 4 << 20
    want = device_scores(e, codes, offsets)
    got = e.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))
    pc = torch.from_numpy(codes).pin_memory()
    po = torch.from_numpy(offsets.view(np.int64)).pin_memory()
    got = e.score_batch(codes=pc.numpy(), offsets=po.numpy().view(np.uint64))
    assert np.array_equal(bits(got), bits(want))
    idx = sample_with_extremes(offsets, 60, 7)
    assert np.array_equal(bits(want[idx]), bits(OracleProfile("700").score_batch(*subset(codes, offsets, idx),
                                                                                  threads=ORACLE_THREADS)))
    # an offsets array that does not start at 0 (a slice of a larger batch)
    sub = e.score_batch(codes=codes, offsets=offsets[5000:])
    assert np.array_equal(bits(sub), bits(want[5000:]))
    e.close()


def test_pinned_small_model_large_batch_copied():
    """Page-locked residues of a small model's large batch (< 300 states, >= 16 MiB: msv_device.cpp
    kInPlaceMinStates) are copied through the piece pipeline instead of read in place: bitwise equal to a
    device launch, with pageable and page-locked score destinations, and to the oracle on a sample."""
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("200.hmm")))
    codes, offsets = random_batch(98, 50_000, 300, 500)
    assert int(offsets[-1]) >= 16 << 20
    want = device_scores(e, codes, offsets)
    pc = msv.pinned_empty(codes.size, np.uint8)
    pc[:] = codes
    out = msv.pinned_empty(len(want), np.float32)
    assert np.array_equal(bits(e.score_batch(codes=pc, offsets=offsets)), bits(want))
    assert np.array_equal(bits(e.score_batch(codes=pc, offsets=offsets, out=out)), bits(want))
    shards = [msv.MSV_HMM(msv.Profile_HMM(profile_path("200.hmm")), device=0) for _ in range(2)]
    assert np.array_equal(bits(msv.score_batch_multi(shards, codes=pc, offsets=offsets)), bits(want))  # same policy
    for x in shards:
        x.close()
    idx = sample_with_extremes(offsets, 200, 99)
    assert np.array_equal(bits(want[idx]), bits(OracleProfile("200").score_batch(*subset(codes, offsets, idx))))
    e.close()


def test_small_host_calls_staged():
    """Pageable host calls of at most 1 MiB of residues (msv_device.cpp kSmallCall) send the residues in
    the offsets' H2D and take the scores through pinned staging: bitwise equal to a device launch on
    both sides of the limit (1 MiB and 1 MiB + 1 residues), one-sequence calls of every length class,
    an all-empty batch, and a bad residue (raises; the next call is clean)."""
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400.hmm")))
    o = OracleProfile("1400")
    rng = np.random.default_rng(97)
    for total in (1 << 20, (1 << 20) + 1):
        lens = np.full(total // 500, 500, np.int64)
        lens[-1] += total - int(lens.sum())
        codes = rng.integers(0, 20, total).astype(np.uint8)
        offsets = np.zeros(len(lens) + 1, np.uint64)
        offsets[1:] = np.cumsum(lens)
        assert np.array_equal(bits(e.score_batch(codes=codes, offsets=offsets)), bits(device_scores(e, codes, offsets)))
    for L in (0, 1, 7, 16, 17, 3500, 20_000):
        c = rng.integers(0, 20, L).astype(np.uint8)
        off = np.array([0, L], np.uint64)
        assert bits(e.score_batch(codes=c, offsets=off))[0] == bits(o.score_batch(c, off))[0], L
    assert np.all(np.isneginf(e.score_batch(codes=np.zeros(0, np.uint8), offsets=np.zeros(4, np.uint64))))
    c = rng.integers(0, 20, 900).astype(np.uint8)
    off = np.array([0, 300, 900], np.uint64)
    bad = c.copy()
    bad[450] = 20
    with pytest.raises(IndexError):
        e.score_batch(codes=bad, offsets=off)
    assert np.array_equal(bits(e.score_batch(codes=c, offsets=off)), bits(o.score_batch(c, off)))
    e.close()


def test_one_profile_on_two_streams_without_sync():
    """launches of one profile on different streams with no synchronisation between them
    (a device call on a torch stream, then the host API on the library's stream, then two more
    device calls on two other streams) each take their own dequeue counter slot."""
    import torch
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400.hmm")))
    dev = torch.device("cuda:0")
    batches = [random_batch(300 + k, n, 0, 700) for k, n in enumerate((70_000, 20_000, 50_000, 9_000))]
    e.reserve_length(700)
    ref = [e.score_batch(codes=c, offsets=o) for c, o in batches]
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    tens = []
    for c, o in batches:
        tens.append((torch.from_numpy(c).to(dev), torch.from_numpy(o.view(np.int64)).to(dev),
                     torch.full((len(o) - 1,), float("nan"), dtype=torch.float32, device=dev)))
    torch.cuda.synchronize()
    for rep in range(3):
        r, o, s = tens[0]
        e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), s.numel(), s.data_ptr(), None,
                             streams[0].cuda_stream)
        host = e.score_batch(codes=batches[1][0], offsets=batches[1][1])  # library stream, no sync first
        for k in (2, 3):
            r, o, s = tens[k]
            e.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), s.numel(), s.data_ptr(), None,
                                 streams[k - 1].cuda_stream)
        torch.cuda.synchronize()
        e.check()
        assert np.array_equal(bits(host), bits(ref[1])), rep
        for k in (0, 2, 3):
            assert np.array_equal(bits(tens[k][2].cpu().numpy()), bits(ref[k])), (rep, k)
        # rep 1: stream 0 bound (its slot events are recorded lazily, only when another stream takes
        # the slot); rep 2: unbound again (the pending events are flushed first)
        e.bind_stream(streams[0].cuda_stream if rep == 0 else None)
    e.close()


def test_score_batch_multi_same_handle_twice():
    """the same profile handle listed more than once scores its shards one after another
    on one host thread (no race on its staging buffers)."""
    prof = msv.Profile_HMM(profile_path("1400.hmm"))
    a, b = msv.MSV_HMM(prof), msv.MSV_HMM(prof)
    codes, offsets = random_batch(72, 30_000, 0, 800)
    want = a.score_batch(codes=codes, offsets=offsets)
    for handles in ([a, a], [a, b, a, b, a], [b, b, b, b]):
        got = msv.score_batch_multi(handles, codes=codes, offsets=offsets)
        assert np.array_equal(bits(got), bits(want)), len(handles)
    a.close()
    b.close()


def test_describe_reports_every_plan():
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400.hmm")))
    d = e.describe()
    assert d["latency_variant"].startswith("msv_g64_") and d["latency_max_n"] >= 4096
    assert d["latency_blocks"] > 0 and d["variant"] != d["latency_variant"]
    # mid-size batches of a large G = 16 profile: the 32-lane plan, above the latency plan's range
    assert d["mid_variant"].startswith("msv_g32_") and d["mid_blocks"] > 0
    assert d["latency_max_n"] < d["mid_max_n"] < d["blocks"] * 64
    # batches of at most one workgroup per CU: the cooperative plan (msv_coop.hip), then the latency plan
    assert d["coop_variant"] == "msv_coop_w4_s6" and d["coop_max_n"] == 2 * d["coop_blocks"] >= 512
    assert e.variant_for(1) == d["coop_variant"] == e.variant_for(d["coop_max_n"])
    assert e.variant_for(d["coop_max_n"] + 1) == d["latency_variant"] == e.variant_for(d["latency_max_n"])
    assert e.variant_for(d["latency_max_n"] + 1) == d["mid_variant"] == e.variant_for(d["mid_max_n"])
    assert e.variant_for(d["mid_max_n"] + 1) == d["variant"] == e.variant_for(10**7)
    # 100.hmm: 4-lane groups for full batches, the 16-lane plan below 3.5 of its waves per SIMD
    small_e = msv.MSV_HMM(msv.Profile_HMM(profile_path("100.hmm")))
    small = small_e.describe()
    assert small["latency_variant"] == "" and small["latency_max_n"] == 0
    assert small["variant"].startswith("msv_g4_") and small["mid_variant"].startswith("msv_g16_")
    assert small_e.variant_for(10_000) == small["mid_variant"] and small_e.variant_for(100_000) == small["variant"]
    small_e.close()
    # 200.hmm: a whole-row-ring variant for full batches, the PF-2 one below 10,752 sequences
    two_e = msv.MSV_HMM(msv.Profile_HMM(profile_path("200.hmm")))
    two = two_e.describe()
    assert two["variant"] == "msv_g16_s16_w16_p4_d1" and two["mid_variant"] == "msv_g16_s16_w8_p2_d1"
    assert two_e.variant_for(10_000) == two["mid_variant"] and two_e.variant_for(20_000) == two["variant"]
    two_e.close()
    g32 = msv.MSV_HMM(msv.Profile_HMM(profile_path("1901.hmm"))).describe()  # main plan already 32 lanes
    assert g32["lanes_per_group"] == 32 and g32["mid_variant"] == ""
    assert g32["coop_variant"] == "msv_coop_w4_s8_a6"  # 1901 states: the split cooperative table
    e.close()


def test_async_stream_of_batches():
    """msv_score_batch_async / msv_profile_wait: three calls in flight (the copies of the later ones
    under the kernel of the first), results equal to the synchronous path; a bad residue is reported
    by the wait of ITS call only; a fourth outstanding call is refused."""
    import torch
    from hmm_fasta_viterbi_amd._native import MSVError
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400.hmm")))
    batches = [random_batch(400 + k, n, 0, 700) for k, n in enumerate((30_000, 1, 5_000, 60_000, 0, 12_345))]
    want = [e.score_batch(codes=c, offsets=o) for c, o in batches]
    pinned = [(torch.from_numpy(c).pin_memory().numpy(), o) for c, o in batches]
    tickets = []
    got = []
    for k, (c, o) in enumerate(pinned):
        tickets.append(e.score_batch_async(c, o))
        if k >= 2:
            got.append(e.wait(tickets[k - 2]))
    got.append(e.wait(tickets[-2]))
    got.append(e.wait(tickets[-1]))
    for k, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(bits(g), bits(w)), k
    # errors stay with their call
    bad_c = batches[0][0].copy()
    bad_c[int(batches[0][1][9]) + 1] = 25
    t_bad = e.score_batch_async(bad_c, batches[0][1])
    t_ok = e.score_batch_async(batches[2][0], batches[2][1])
    t_ok2 = e.score_batch_async(batches[5][0], batches[5][1])
    with pytest.raises(MSVError):
        e.score_batch_async(batches[3][0], batches[3][1])  # three already outstanding
    with pytest.raises(IndexError):
        e.wait(t_bad)
    assert np.array_equal(bits(e.wait(t_ok)), bits(want[2]))
    assert np.array_equal(bits(e.wait(t_ok2)), bits(want[5]))
    with pytest.raises(MSVError):
        e.wait(t_ok)  # already waited for
    e.close()


def test_pinned_destinations_written_by_kernel():
    """Page-locked score destinations are written by the kernels themselves (no D2H): the one-call
    pipeline and the async stream of batches return the staged paths' scores bitwise; a bad residue
    in a direct async call is found from its +inf score, reported by that call's wait only, and
    leaves no latched bit behind for the next (staged) call on the same slot."""
    import torch
    from hmm_fasta_viterbi_amd._native import MSVError
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400.hmm")))
    batches = [random_batch(500 + k, n, 0, 700) for k, n in enumerate((40_000, 3, 15_000, 25_000))]
    want = [e.score_batch(codes=c, offsets=o) for c, o in batches]
    pin = lambda n: torch.full((n,), float("nan"), dtype=torch.float32).pin_memory().numpy()
    big_c, big_o = random_batch(510, 30_000, 100, 400)  # >= 4 Mi residues: the piece pipeline
    assert int(big_o[-1]) >= 4 << 20
    big_want = e.score_batch(codes=big_c, offsets=big_o)
    got = e.score_batch(codes=big_c, offsets=big_o, out=pin(len(big_o) - 1))
    assert np.array_equal(bits(got), bits(big_want))
    outs = [pin(len(o) - 1) for _, o in batches]
    tickets, got = [], []
    for k, ((c, o), out) in enumerate(zip(batches, outs)):
        tickets.append(e.score_batch_async(c, o, out=out))
        if k >= 1:
            got.append(e.wait(tickets[k - 1]))
    got.append(e.wait(tickets[-1]))
    for k, (g, w) in enumerate(zip(got, want)):
        assert np.array_equal(bits(g), bits(w)), k
    bad_c = batches[0][0].copy()
    bad_c[int(batches[0][1][7]) + 2] = 31
    for slot_pair in range(2):  # both staging slots take a direct bad call, then a staged good one
        if slot_pair:  # shift the slot parity by one call
            assert np.array_equal(bits(e.wait(e.score_batch_async(*batches[1]))), bits(want[1]))
        t_bad = e.score_batch_async(bad_c, batches[0][1], out=pin(len(batches[0][1]) - 1))
        t_ok = e.score_batch_async(batches[2][0], batches[2][1], out=pin(len(batches[2][1]) - 1))
        with pytest.raises(IndexError):
            e.wait(t_bad)
        assert np.array_equal(bits(e.wait(t_ok)), bits(want[2])), slot_pair
        t1 = e.score_batch_async(batches[3][0], batches[3][1])  # pageable: staged D2H + error word
        t2 = e.score_batch_async(batches[2][0], batches[2][1])
        assert np.array_equal(bits(e.wait(t1)), bits(want[3]))
        assert np.array_equal(bits(e.wait(t2)), bits(want[2]))
    with pytest.raises(MSVError):
        e.wait(t2)
    e.close()


@pytest.mark.parametrize("prof", ["700", "1600", "1901"])
def test_zero_copy_twin_variants(prof):
    """Page-locked residues of a full batch run the variant's zero-copy twin (residue blocks instead of
    one row of prefetch, msv_kernel.hip zc_fn): random + homolog sequences equal a device launch of the
    ordinary variant bitwise, and the oracle on a sample."""
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
    assert e.describe()["states_per_lane"] > 40
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path(prof + ".hmm")).match_emissions, 531, 300, 1, 700)
    codes, offsets = concat_batches(random_batch(530, 24_000, 0, 800), (hc, ho))
    want = device_scores(e, codes, offsets)
    pc = msv.pinned_empty(codes.size, np.uint8)
    pc[:] = codes
    got = e.score_batch(codes=pc, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))
    n = len(offsets) - 1
    sample = np.concatenate([np.arange(0, n - 300, 997), np.arange(n - 300, n, 11)])
    assert np.array_equal(bits(got[sample]), bits(OracleProfile(prof).score_batch(*subset(codes, offsets, sample))))
    e.close()


def _wide_edge_batch(prof, seed):
    """Lengths around the 16-row blocks and 64-row superblocks of the wide twins (0-5, 15-17, ..., 127-129),
    random ones, and homologs (J >= N rows), shuffled so sequences begin at every phase of the row loop."""
    edges = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 47, 48, 49, 63, 64, 65, 79, 80, 81, 127, 128, 129, 200]
    rng = np.random.default_rng(seed)
    lens = np.array(edges * 3 + list(rng.integers(0, 400, 150)), np.int64)
    codes = rng.integers(0, 20, int(lens.sum())).astype(np.uint8)
    offsets = np.zeros(len(lens) + 1, np.uint64)
    offsets[1:] = np.cumsum(lens)
    hc, ho = homolog_batch(msv.Profile_HMM(profile_path(prof + ".hmm")).match_emissions, seed + 1, 40, 1, 300)
    codes, offsets = concat_batches((codes, offsets), (hc, ho))
    perm = rng.permutation(len(offsets) - 1)
    return subset(codes, offsets, perm)


def test_zero_copy_wide_blocks_every_short_row_variant():
    """The zero-copy twins of residue-block variants (rows of <= 40 states, G >= 16) read 64-row
    superblocks as unaligned dwords (msv_kernel_body.inc WIDE): every such variant, forced, on residues in
    a page-locked buffer of exactly the batch's size (the last sequence ends at the allocation's end),
    equals the oracle bitwise -- lengths around every block/superblock edge, homologs, all begin phases
    -- and so does the 16-byte-block form (msv_debug_set_zero_copy 2)."""
    import ctypes as C
    from hmm_fasta_viterbi_amd import _native

    def _variant_shape(name):  # msv_g<G>_s<S>_...
        parts = name.split("_")
        return int(parts[1][1:]), int(parts[2][1:])
    L = _native.lib()
    L.msv_debug_set_zero_copy.argtypes = [C.c_void_p, C.c_int]
    names = [n for n in msv.MSV_HMM.variants() if not n.startswith("exp")]
    short = [n for n in names if _variant_shape(n)[0] >= 16 and _variant_shape(n)[1] <= 40
             and "_a" not in n and "_d1" in n]
    assert len(short) >= 20
    by_prof = {}
    lengs = {p: msv.Profile_HMM(profile_path(p + ".hmm")).model_length - 1
             for p in ("100", "200", "300", "400", "500", "600", "700", "800", "900", "1001", "1100", "1200")}
    for name in short:
        g, s = _variant_shape(name)
        fits = [p for p in lengs if lengs[p] <= g * s]
        if fits:  # (16 x 4 covers no real profile: the smallest has 100 states)
            by_prof.setdefault(max(fits, key=lambda p: lengs[p]), []).append(name)
    assert sum(len(v) for v in by_prof.values()) >= 20
    for k, (prof, vs) in enumerate(sorted(by_prof.items())):
        codes, offsets = _wide_edge_batch(prof, 900 + k)
        want = OracleProfile(prof).score_batch(codes, offsets)
        pc = msv.pinned_empty(codes.size, np.uint8)
        pc[:] = codes
        out = msv.pinned_empty(len(want), np.float32)
        e = msv.MSV_HMM(msv.Profile_HMM(profile_path(prof + ".hmm")))
        for name in vs:
            e.set_variant(name)
            for mode in (1, 2):
                assert L.msv_debug_set_zero_copy(e._p, mode) == 0
                assert np.array_equal(bits(e.score_batch(codes=pc, offsets=offsets)), bits(want)), (prof, name, mode)
                got = e.score_batch(codes=pc, offsets=offsets, out=out)  # page-locked scores too
                assert got is out and np.array_equal(bits(out), bits(want)), (prof, name, mode)
        e.close()


def test_zero_copy_wide_blocks_small_buffers_and_errors():
    """Buffers of 63 bytes (too small for the dword twin: the ordinary variant runs) and of 64 and 65
    bytes (the twin, its clamp at the buffer's first and last bytes), a bad residue inside a superblock
    (raises, and the next call is clean), and cfg2's full batch from page-locked memory against the
    resident launch."""
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("100.hmm")))
    o = OracleProfile("100")
    rng = np.random.default_rng(77)
    for total in (63, 64, 65, 66, 67, 130):
        for lens in ([total], [1, total - 1], [total - 3, 3], [20, 20, total - 40] if total > 40 else [total]):
            codes = rng.integers(0, 20, total).astype(np.uint8)
            offsets = np.zeros(len(lens) + 1, np.uint64)
            offsets[1:] = np.cumsum(lens)
            pc = msv.pinned_empty(total, np.uint8)
            pc[:] = codes
            assert np.array_equal(bits(e.score_batch(codes=pc, offsets=offsets)), bits(o.score_batch(codes, offsets)))
    codes, offsets = random_batch(1, 10_000, 300, 500)  # cfg2 (BASELINE configs[1]), seed 1
    want = device_scores(e, codes, offsets)
    pc = msv.pinned_empty(codes.size, np.uint8)
    pc[:] = codes
    out = msv.pinned_empty(len(want), np.float32)
    assert np.array_equal(bits(e.score_batch(codes=pc, offsets=offsets, out=out)), bits(want))
    pc[int(offsets[4321]) + 37] = 25  # bad residue, inside the sequence's first superblock but one
    with pytest.raises(IndexError):
        e.score_batch(codes=pc, offsets=offsets, out=out)
    pc[int(offsets[4321]) + 37] = codes[int(offsets[4321]) + 37]
    assert np.array_equal(bits(e.score_batch(codes=pc, offsets=offsets, out=out)), bits(want))
    e.close()


def test_zero_copy_pinned_residues():
    """Page-locked residues are read by the kernel in place (no H2D): bitwise equal to the copy
    pipeline (zero-copy switched off) and to a device launch -- for a > 4 Mi-residue batch (one launch
    instead of pieces), an offsets array not starting at 0, a view starting inside the pinned
    allocation, a pinned buffer rewritten between calls, and a bad residue (raises)."""
    import ctypes as C
    import torch
    from hmm_fasta_viterbi_amd import _native
    L = _native.lib()
    L.msv_debug_set_zero_copy.argtypes = [C.c_void_p, C.c_int]
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400.hmm")))
    codes, offsets = random_batch(520, 30_000, 0, 600)
    assert int(offsets[-1]) >= 4 << 20
    want = device_scores(e, codes, offsets)
    pinned = torch.from_numpy(codes).pin_memory().numpy()
    got = e.score_batch(codes=pinned, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))
    assert L.msv_debug_set_zero_copy(e._p, 0) == 0  # the copy pipeline on the same pinned source
    assert np.array_equal(bits(e.score_batch(codes=pinned, offsets=offsets)), bits(want))
    assert L.msv_debug_set_zero_copy(e._p, 1) == 0
    sub = e.score_batch(codes=pinned, offsets=offsets[7000:])  # offsets[0] != 0
    assert np.array_equal(bits(sub), bits(want[7000:]))
    base = int(offsets[123])  # a view whose first byte is inside the pinned allocation
    view = e.score_batch(codes=pinned[base:], offsets=(offsets[123:] - base).astype(np.uint64))
    assert np.array_equal(bits(view), bits(want[123:]))
    c2, o2 = random_batch(521, 30_000, 0, 600)  # rewrite the same pinned buffer
    m = min(len(c2), len(pinned))
    keep = int(np.searchsorted(o2, m, side="right")) - 1
    pinned[:int(o2[keep])] = c2[:int(o2[keep])]
    want2 = e.score_batch(codes=c2, offsets=o2[:keep + 1])  # pageable: copied
    assert np.array_equal(bits(e.score_batch(codes=pinned, offsets=o2[:keep + 1])), bits(want2))
    pinned[int(o2[5]) + 3] = 22
    with pytest.raises(IndexError):
        e.score_batch(codes=pinned, offsets=o2[:keep + 1])
    e.close()


def test_pinned_empty_arrays_zero_copy():
    """msv.pinned_empty (msv_host_alloc): page-locked numpy arrays for residues and scores -- read and
    written by the kernel in place -- give the pageable path's bits; the memory is released with the
    last view (msv_host_free)."""
    import gc
    e = msv.MSV_HMM(msv.Profile_HMM(profile_path("900.hmm")))
    codes, offsets = random_batch(530, 20_000, 1, 700)
    want = e.score_batch(codes=codes, offsets=offsets)
    for _ in range(3):  # allocate / release repeatedly
        pc = msv.pinned_empty(codes.shape, np.uint8)
        pc[:] = codes
        out = msv.pinned_empty(len(want), np.float32)
        got = e.score_batch(codes=pc, offsets=offsets, out=out)
        assert got is out and np.array_equal(bits(out), bits(want))
        view = pc[int(offsets[10]):]
        del pc, out, got
        gc.collect()
        sub = e.score_batch(codes=view, offsets=(offsets[10:] - offsets[10]).astype(np.uint64))
        assert np.array_equal(bits(sub), bits(want[10:]))  # the view alone keeps the allocation alive
        del view
        gc.collect()
    e.close()


def test_rccl_multi_device_context():
    """msv_multi_*: ncclCommInitAll over the given devices, shards scored per device, scores gathered
    into device 0 by ONE grouped ncclSend/ncclRecv (rank 0 through a self send/recv), one D2H.  On a
    one-GPU box this is a 1-rank communicator (the exchange still runs, as a self send/recv); with
    more devices every visible one joins.  A device listed twice is refused (one RCCL rank per
    device: RCCL rejects duplicate GPUs in one communicator)."""
    from hmm_fasta_viterbi_amd._native import MSVError
    prof = msv.Profile_HMM(profile_path("1400.hmm"))
    ndev = msv.device_count()
    engines = [msv.MSV_HMM(prof, device=k) for k in range(ndev)]
    codes, offsets = random_batch(3, 200_000, 300, 500)  # cfg4's generator, 200k of its 1M
    want = engines[0].score_batch(codes=codes, offsets=offsets)
    multi = msv.MultiGPU(engines)
    got = multi.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(bits(got), bits(want))
    small = multi.score_batch(codes=codes[:int(offsets[3])], offsets=offsets[:4])  # fewer sequences than ranks
    assert np.array_equal(bits(small), bits(want[:3]))
    import torch
    pinned = torch.from_numpy(codes).pin_memory().numpy()  # shards read in place by every rank's kernel
    assert np.array_equal(bits(multi.score_batch(codes=pinned, offsets=offsets)), bits(want))
    # the fallback when a rank cannot alias the page-locked source: its shard is copied (msv_debug_multi_no_alias)
    from hmm_fasta_viterbi_amd import _native
    _native.lib().msv_debug_multi_no_alias.argtypes = [C.c_int]
    _native.lib().msv_debug_multi_no_alias(1)
    try:
        assert np.array_equal(bits(multi.score_batch(codes=pinned, offsets=offsets)), bits(want))
    finally:
        _native.lib().msv_debug_multi_no_alias(0)
    empty = multi.score_batch(codes=pinned[:0], offsets=np.zeros(5, np.uint64))  # all-empty, pinned source
    assert np.all(empty == -np.inf)
    idx = sample_with_extremes(offsets, 64, 9)
    assert np.array_equal(bits(got[idx]), bits(OracleProfile("1400").score_batch(*subset(codes, offsets, idx),
                                                                                  threads=ORACLE_THREADS)))
    multi.close()
    with pytest.raises(MSVError):
        msv.MultiGPU([engines[0], engines[0]])
    for e in engines:
        e.close()
