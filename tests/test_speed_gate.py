"""Speed gate (GPU): the automatically picked MSV and Viterbi kernels of every one of the 24 reference profiles
(benchmark_MSV.cpp:32-41 scores every profile) on one fixed device-resident batch, each held to >= 30% of the
GCUPS recorded for it in tests/golden/speed_table.json.

The bitwise suite checks bits, not time: in round 5 a change that pushed the Viterbi M / I / D rows of S = 14-24
into scratch memory (40x slower on 1001.hmm and 1200.hmm, profiles/r05_vit_scratch_regression.jsonl) passed the
whole GPU suite.  This test fails on exactly that build (profiles/r06_speed_gate/).

Timing: kernel only (torch events on the launch's own stream), best of 3 after a warm-up, 2,000,000 residues.

The 5,000-sequence batch runs each profile's latency or mid plan; the throughput plans the bench's own lines run
(cfg3's 100,000 sequences, cfg5's long ones) are gated separately, at the bench's sizes and seeds with its
longest-first order (bench.py CONFIGS, step()), against a tighter floor: they are the headline kernels.

Re-record the table on an MI355X with  SPEED_GATE_RECORD=tests/golden/speed_table.json  (both tests update their
own keys in it; then review the diff)."""
import json
import os

import numpy as np
import pytest

from oracle_lib import ROOT

TABLE = os.path.join(ROOT, "tests", "golden", "speed_table.json")
PROFILES = sorted((f for f in os.listdir(os.path.join(ROOT, "data", "profile_HMMs")) if f.endswith(".hmm")),
                  key=lambda f: int(f.split(".")[0]))
N_SEQ, LMIN, LMAX, SEED = 5000, 300, 500, 61  # ~2.0 M residues, the bench's length distribution
FLOOR = 0.30
BENCH_FLOOR = 0.75
BENCH_CONFIGS = ("cfg2", "cfg3", "cfg5")  # the single-GPU weak-scaling configs (cfg4 is cfg3's kernel, sharded)


def _time_ms(launch, stream, reps=3):
    import torch
    launch()  # warm-up (first launch of a profile: code object load, tables)
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        launch()
        b.record(stream)
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


def _record(path, note_key, note, measured):
    table = json.load(open(path)) if os.path.exists(path) else {}
    table.update({note_key: note, **measured})
    with open(path, "w") as f:
        json.dump(table, f, indent=1)
    print(json.dumps(measured))


@pytest.mark.gpu
def test_every_profile_keeps_its_recorded_speed():
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch

    codes, offsets = random_batch(SEED, N_SEQ, LMIN, LMAX)
    residues = int(offsets[-1])
    dev = torch.device("cuda:0")
    d_res = torch.from_numpy(codes).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    d_sc = torch.empty(N_SEQ, dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    s = st.cuda_stream
    measured = {"msv": {}, "viterbi": {}, "msv_variant": {}, "viterbi_variant": {}}
    for prof in PROFILES:
        hmm = msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof))
        leng = hmm.model_length - 1
        m, v = msv.MSV_HMM(hmm), msv.Viterbi_HMM(hmm)
        try:
            tm = _time_ms(lambda: m.score_batch_device(d_res.data_ptr(), residues, d_off.data_ptr(), N_SEQ,
                                                       d_sc.data_ptr(), None, s), st)
            tv = _time_ms(lambda: v.score_batch_device(d_res.data_ptr(), residues, d_off.data_ptr(), N_SEQ,
                                                       d_sc.data_ptr(), None, None, s), st)
            m.check(s)
            v.check(s)
            key = prof.split(".")[0]
            measured["msv"][key] = round(residues * leng / tm / 1e6, 1)
            measured["viterbi"][key] = round(residues * leng / tv / 1e6, 1)
            measured["msv_variant"][key] = m.variant_for(N_SEQ)
            measured["viterbi_variant"][key] = v.describe()["variant"]
        finally:
            m.close()
            v.close()
    record = os.environ.get("SPEED_GATE_RECORD")
    if record:
        _record(record, "note", "GCUPS (residues x LENG / kernel time) of the auto-picked kernels on "
                                f"random_batch({SEED}, {N_SEQ}, {LMIN}, {LMAX}) = {residues} residues, "
                                "one MI355X, best of 3 (tests/test_speed_gate.py)", measured)
        return
    table = json.load(open(TABLE))
    slow = {}
    for stage in ("msv", "viterbi"):
        for key, want in table[stage].items():
            got = measured[stage][key]
            if got < FLOOR * want:
                slow[f"{stage} {key}.hmm ({measured[stage + '_variant'][key]})"] = (got, want)
    print(json.dumps(measured))
    assert not slow, f"below {FLOOR:.0%} of the recorded GCUPS (got, recorded): {slow}"


@pytest.mark.gpu
def test_bench_configs_keep_their_recorded_speed():
    """The MSV launch of bench.py's step() for cfg2 / cfg3 / cfg5 on rank 0's batch (random_batch(seed * 1000, ...),
    device-resident, order_longest_first then the plan variant_for(n) picks), kernel-only GCUPS >= 75% of the
    recorded value, and the plan is still the recorded one."""
    import sys
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd.synthetic import random_batch
    sys.path.insert(0, ROOT)
    import bench

    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    s = st.cuda_stream
    measured = {"bench_msv": {}, "bench_msv_variant": {}}
    for cfg in BENCH_CONFIGS:
        prof, n, lmin, lmax, seed, scaling = bench.CONFIGS[cfg]
        assert scaling == "weak"
        codes, offsets = random_batch(seed * 1000, n, lmin, lmax)
        residues = int(offsets[-1])
        d_res = torch.from_numpy(codes).to(dev)
        d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
        d_sc = torch.empty(n, dtype=torch.float32, device=dev)
        d_ord = torch.empty(n, dtype=torch.int32, device=dev)
        m = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", prof)))
        try:
            m.reserve_length(lmax)
            m.order_longest_first(d_off.data_ptr(), n, d_ord.data_ptr(), s)
            tm = _time_ms(lambda: m.score_batch_device(d_res.data_ptr(), residues, d_off.data_ptr(), n,
                                                       d_sc.data_ptr(), d_ord.data_ptr(), s), st, reps=5)
            m.check(s)
            measured["bench_msv"][cfg] = round(residues * (m.model_length - 1) / tm / 1e6, 1)
            measured["bench_msv_variant"][cfg] = m.variant_for(n)
        finally:
            m.close()
        del d_res, d_off, d_sc, d_ord
    record = os.environ.get("SPEED_GATE_RECORD")
    if record:
        _record(record, "bench_note", "GCUPS of the MSV launch in bench.py's step() for each config (rank 0's "
                                      "batch, longest-first order, kernel only, best of 5 after ONE warm-up launch "
                                      "-- the bench warms 12, so these read a few % below its kernel rates; "
                                      "tests/test_speed_gate.py)", measured)
        return
    table = json.load(open(TABLE))
    print(json.dumps(measured))
    assert measured["bench_msv_variant"] == table["bench_msv_variant"]
    slow = {cfg: (measured["bench_msv"][cfg], want) for cfg, want in table["bench_msv"].items()
            if measured["bench_msv"][cfg] < BENCH_FLOOR * want}
    assert not slow, f"below {BENCH_FLOOR:.0%} of the recorded GCUPS (got, recorded): {slow}"
