"""bench.py -- MSV scoring throughput on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W [--config cfg3]
    (N > 1, one process per GPU: under torch.distributed.run WORLD_SIZE must equal N; started
    without it, bench.py runs `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a
    child process before touching torch or the GPU and exits with its status)

A step = one pass of the hot path over one batch resident in HBM: the longest-first dequeue
order (device counting sort) + ONE fused MSV kernel launch scoring every sequence of the rank's
shard against the profile.  Sequences are independent, so the batch shards across ranks with no
data-path collective.
  cfg2/cfg3/cfg5 (weak scaling): every rank scores its own seeded batch of the config's size; the
      scores are gathered to rank 0 over RCCL once after timing (reported as gather_ms).
  cfg4 (strong scaling, BASELINE configs[3]): ONE seeded 1M-sequence set, cut into residue-balanced
      contiguous shards (distributed.shard_bounds == msv_shard_bounds); the RCCL gather of the
      scores to every rank is part of every timed step.

Rank 0 prints ONE JSON line with the contract keys plus:
  roofline     -- the dominant kernel against the fp32 VALU issue roofline:
                  3 fp32 ops (add, max, max) per cell, cells = residues x LENG;
                  peak = 256 CU x 128 lanes x 2.4 GHz = 78.64 T ops/s (non-FMA VALU);
                  achieved from the kernel's HIP-event time on the stream it runs on.
  cpu_baseline -- the reference's OWN run_on_sequence (oracle/_ref, "reference") or the oracle
                  restatement ("port") on the host cores, on a bounded leading sample of the same
                  batch, timed in this run; its scores are also compared bitwise with the GPU's.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# The host pipeline (msv_score_batch / msv_score_batch_async) keeps a copy stream and two compute
# streams busy at once next to torch's streams; HIP's default of 4 hardware queues per process then
# makes streams share queues and serialise (cfg3 pipelined host path 9,543 vs 10,597 M res/s with 8).
# Informational figures only; the HBM-resident `value` runs on one stream.  (Set before torch loads
# HIP; the GPU box exports 4.)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

CONFIGS = {
    # name: (profile, sequences, lmin, lmax, seed, scaling)  -- SURVEY 8(d) / BASELINE.md
    # weak: sequences per GPU; strong: sequences of the whole job, sharded over the GPUs
    "cfg2": ("100.hmm", 10_000, 300, 500, 1, "weak"),
    "cfg3": ("1400.hmm", 100_000, 300, 500, 2, "weak"),
    "cfg4": ("1400.hmm", 1_000_000, 300, 500, 3, "strong"),
    "cfg5": ("2405.hmm", 100_000, 1500, 2500, 4, "weak"),
}
METRIC = "M residues/sec (GCUPS) for profile M=1400 vs 100k seqs, 1/2/4/8 GPU"
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12  # 78.64 T fp32 lane-ops/s
HBM_PEAK_GBPS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=12,
                    help="untimed steps; the MI355X clock ramps over the first ~10 launches (3.8 -> 3.0 ms)")
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may run on")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-viterbi", action="store_true", help="skip the informational Viterbi-stage figure")
    ap.add_argument("--no-clock", action="store_true", help="time the steps without the in-kernel clock stamps")
    ap.add_argument("--no-order", action="store_true", help="dequeue in input order (no longest-first sort)")
    ap.add_argument("--no-launch-events", action="store_true",
                    help="diagnostic: time the steps without the MSV launch's start/stop events (kernel_ms null)")
    ap.add_argument("--dry-run", action="store_true",
                    help="check the rank layout (gloo rendezvous, no GPU) and print it from rank 0")
    return ap.parse_args()


def host_cpus() -> dict:
    """nproc (os.cpu_count) and the CPUs this process may run on (sched_getaffinity)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None  # cgroup v2 CPU quota in CPUs ("max" = none)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            quota = None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota}


def cpu_threads(arg: int) -> int:
    """One thread per CPU this process may run on, capped at the cgroup CPU quota when there is one
    (on the GPU box the affinity mask is the whole 256-CPU host while the quota is 16 CPUs; 256
    threads under that quota measured 4.31 M res/s against 4.97 for 16 on cfg3, so the cap is the
    more generous baseline)."""
    if arg > 0:
        return arg
    h = host_cpus()
    n = h["affinity_cpus"]
    if h["cgroup_cpu_quota"]:
        n = min(n, max(1, int(-(-h["cgroup_cpu_quota"] // 1))))
    return max(1, n)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(profile_path, codes, offsets, gpu_scores, target_s, threads):
    """Time the reference CPU path (or the oracle port) on a bounded leading sample."""
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libref_msv.so")
    ora_so = os.path.join(ROOT, "oracle", "_build", "libmsv_oracle.so")
    n_total = len(offsets) - 1

    def run(n):
        offs = np.ascontiguousarray(offsets[: n + 1])
        out = np.zeros(n, np.float32)
        if kind == "reference":
            sec = lib.ref_score_codes(profile_path.encode(), codes.ctypes.data, offs.ctypes.data, n, threads,
                                      out.ctypes.data)
        else:
            t0 = time.perf_counter()
            lib.oracle_profile_score_batch(prof, codes.ctypes.data, offs.ctypes.data, n, out.ctypes.data)
            sec = time.perf_counter() - t0
        return sec, out

    if os.path.exists(ref_so):
        kind = "reference"
        lib = C.CDLL(ref_so)
        lib.ref_score_codes.restype = C.c_double
        lib.ref_score_codes.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_long, C.c_int, C.c_void_p]
    else:
        kind = "port"
        threads = 1
        lib = C.CDLL(ora_so)
        lib.oracle_profile_load.restype = C.c_void_p
        lib.oracle_profile_load.argtypes = [C.c_char_p]
        lib.oracle_profile_score_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        prof = lib.oracle_profile_load(profile_path.encode())
    # calibrate on a small prefix, then size the sample for ~target_s seconds
    n_cal = min(n_total, max(threads * 32, 256))
    sec, _ = run(n_cal)
    per_seq = max(sec, 1e-6) / n_cal
    n = int(min(n_total, max(n_cal, target_s / per_seq)))
    sec, out = run(n)
    residues = int(offsets[n] - offsets[0])
    match = bool(np.array_equal(out.view(np.uint32), gpu_scores[:n].view(np.uint32)))
    single = None
    if kind == "reference" and threads > 1:  # also one thread, on a ~2 s sample
        threads_saved, threads = threads, 1
        n1 = int(min(n_total, max(8, 2.0 / (per_seq * threads_saved))))
        sec1, out1 = run(n1)
        res1 = int(offsets[n1] - offsets[0])
        single = {"value": res1 / sec1 / 1e6, "sequences": n1, "seconds": sec1,
                  "bitwise_equal_to_gpu": bool(np.array_equal(out1.view(np.uint32), gpu_scores[:n1].view(np.uint32)))}
        threads = threads_saved
    return {
        "value": residues / sec / 1e6,
        "unit": "M residues/s",
        "cores": threads,
        **host_cpus(),
        "kind": kind,
        "sample": f"first {n} of {n_total} sequences of this rank's batch ({residues} residues), "
                  f"{sec:.2f} s on {threads} host threads, one MSV_HMM per thread",
        "seconds": sec,
        "bitwise_equal_to_gpu": match,
        "single_thread": single,
        "cpu_model": cpu_model(),
    }


VIT_WARMUP = 20  # untimed Viterbi launches before the timed ones
VIT_OPS_PER_CELL = 14  # fp32 ops per Viterbi DP cell (msv.h): M 3 adds + 3 max + 1 add, I 2 + 1, D 2 + 1, E 1


def viterbi_stage(args, msv_engine, prof_path, dev, stream, d_res, residues, d_off, n, d_scores, d_order, codes,
                  offsets, lmax, leng, hip_event, hip_elapsed_ms, F1=0.02):
    """Information, never `value`: the Viterbi stage on this batch's MSV survivors.  The
    timed steps' device scores -> msv_filter_select_device (P <= F1 against STATS LOCAL MSV, on the GPU,
    survivors listed in the MSV launch's longest-first order)
    -> ONE Viterbi launch over the survivors list (count read on the device), timed with HIP events the
    launch itself updates.  Roofline: 14 fp32 add/max ops per cell (cells = survivor residues x LENG).
    CPU baseline: the oracle's serial Viterbi ("port") on a bounded sample of the survivors, on the host
    threads, whose scores are also compared bitwise with the kernel's."""
    import torch

    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    native = _native.lib()
    native.msv_vit_debug_time_next_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    h = msv.Profile_HMM(prof_path)
    vit = msv.Viterbi_HMM(h, device=dev.index or 0)
    vit.reserve_length(lmax)
    sh = stream.cuda_stream
    d_sel = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    d_vsc = torch.full((max(n, 1),), float("-inf"), dtype=torch.float32, device=dev)
    from hmm_fasta_viterbi_amd._native import check
    check(native.msv_filter_select_device(dev.index or 0, d_scores.data_ptr(), d_off.data_ptr(),
                                          None if d_order is None else d_order.data_ptr(), n, msv_engine.msv_mu,
                                          msv_engine.msv_lambda, F1, None, d_sel.data_ptr(), d_cnt.data_ptr(), sh))

    def launch(ev=None):
        if ev is not None:
            native.msv_vit_debug_time_next_launch(vit._p, ev[0], ev[1])
        vit.score_batch_device(d_res.data_ptr(), residues, d_off.data_ptr(), n, d_vsc.data_ptr(), d_sel.data_ptr(),
                               d_cnt.data_ptr(), sh)

    # warm until the launches are steady: after the MSV phase the first Viterbi launches run slower (cfg3:
    # 1.47 ms falling to 1.35 ms over ten launches behind three warm-ups, profiles/r05_bench_cfg3_vit_warmup.json)
    for _ in range(VIT_WARMUP):
        launch()
    torch.cuda.synchronize(dev)
    steps = max(10, args.steps)
    events = [(hip_event(), hip_event()) for _ in range(steps)]
    t0 = time.perf_counter()
    for ev in events:
        launch(ev)
    torch.cuda.synchronize(dev)
    wall_ms = (time.perf_counter() - t0) / steps * 1e3
    vit.check(sh)
    kall = [hip_elapsed_ms(a, b) for a, b in events]
    kms = float(np.median(kall))
    cnt = int(d_cnt.item())
    sel = np.sort(d_sel[:cnt].cpu().numpy().view(np.uint32))
    vsc = d_vsc[:n].cpu().numpy()
    lens = np.diff(offsets.astype(np.int64))
    surv_res = int(lens[sel].sum())
    cells = surv_res * leng
    achieved = VIT_OPS_PER_CELL * cells / (kms * 1e-3) / 1e12
    info = vit.describe()
    # CPU port baseline on a bounded sample of the survivors (the oracle's serial DP, one profile per run)
    ora = C.CDLL(os.path.join(ROOT, "oracle", "_build", "libmsv_oracle.so"))
    ora.oracle_profile_load.restype = C.c_void_p
    ora.oracle_profile_load.argtypes = [C.c_char_p]
    ora.oracle_profile_vit_prepare.argtypes = [C.c_void_p, C.c_int]
    ora.oracle_profile_vit_score_batch.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t,
                                                   C.c_void_p]
    ora.oracle_profile_free.argtypes = [C.c_void_p]
    op = ora.oracle_profile_load(prof_path.encode())
    ora.oracle_profile_vit_prepare(op, 0)
    threads = cpu_threads(args.cpu_threads)
    sub_off = np.zeros(len(sel) + 1, np.uint64)
    np.cumsum(lens[sel], out=sub_off[1:])
    sub_codes = np.concatenate([codes[int(offsets[s]):int(offsets[s + 1])] for s in sel]) if cnt else codes[:0]
    sub_codes = np.ascontiguousarray(sub_codes)

    def cpu_run(m):
        out = np.zeros(m, np.float32)
        cuts = np.linspace(0, m, threads + 1).astype(np.int64)
        from concurrent.futures import ThreadPoolExecutor

        def part(k):
            lo, hi = int(cuts[k]), int(cuts[k + 1])
            if hi > lo:
                ora.oracle_profile_vit_score_batch(op, 0, sub_codes.ctypes.data, sub_off[lo:].ctypes.data, hi - lo,
                                                   out[lo:].ctypes.data)
        t = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(part, range(threads)))
        return time.perf_counter() - t, out

    cpu = None
    if cnt and not args.no_cpu:
        m0 = min(cnt, 2 * threads)
        sec, _ = cpu_run(m0)
        m = int(min(cnt, max(m0, args.cpu_seconds / 3 / max(sec, 1e-6) * m0)))
        sec, out = cpu_run(m)
        res_m = int(sub_off[m])
        cpu = {"value": round(res_m / sec / 1e6, 4), "unit": "M residues/s", "cores": threads, "kind": "port",
               "sample": f"first {m} of {cnt} survivors ({res_m} residues), {sec:.2f} s on {threads} host threads "
                         "(oracle_vit_run_codes, serial restatement)",
               "bitwise_equal_to_gpu": bool(np.array_equal(out.view(np.uint32), vsc[sel[:m]].view(np.uint32)))}
    ora.oracle_profile_free(op)
    return {
        "F1": F1,
        "survivors": cnt,
        "survivor_fraction": round(cnt / max(n, 1), 5),
        "input_composition": "uniform over the 20 letters (random_FASTA_generator.py's format), not the null "
                             "model's background composition that STATS LOCAL MSV is calibrated on: uniform "
                             "letters over-weight residues rare in the background (W, C, H, M, Y) that carry "
                             "high match scores, so more than F1 pass -- on the CPU oracle at F1 = 0.02, "
                             "1400.hmm passes 0.070 of uniform vs 0.028 of background sequences at L = 400, "
                             "2405.hmm 0.129 vs 0.035 at L = 2000 (profiles/r05_filter_length_composition.jsonl; "
                             "background batches stay calibrated at every length: "
                             "tests/test_gpu_parity.py::test_pvalues_calibrated_at_the_bench_lengths)",
        "survivor_residues": surv_res,
        "kernel_variant": info["variant"],
        "kernel_ms": round(kms, 4),
        "kernel_ms_launches": [round(x, 4) for x in kall],
        "kernel_ms_note": f"median over the timed launches (each timed by HIP events the launch itself updates), after {VIT_WARMUP} untimed ones",
        "ms_per_launch_wall": round(wall_ms, 4),
        "M_residues_s": round(surv_res / (kms * 1e-3) / 1e6, 2),
        "gcups": round(cells / (kms * 1e-3) / 1e9, 2),
        "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": round(VALU_PEAK_TOPS, 2),
                     "unit": "TFLOP/s", "frac": round(achieved / VALU_PEAK_TOPS, 4),
                     "note": f"{VIT_OPS_PER_CELL} fp32 add/max ops per Viterbi cell (M: 3 transition adds, 3 max, "
                             "1 emission add; I: 2 adds, 1 max; D: 2 adds, 1 max; E: 1 max), cells = survivor "
                             "residues x LENG; kernel time from the launch's own HIP events"},
        "scores_finite": bool(np.all(np.isfinite(vsc[sel]))),
        "cpu_baseline": cpu,
        "note": "information, not `value`: the MSV filter's survivors (P <= F1, STATS LOCAL MSV) of the timed "
                "batch, selected on the device, scored by the Viterbi stage in one launch",
    }


def latency_ceiling(engine, dev, sh, n, lmax, longest, kernel_ms, hip_event, hip_elapsed_ms) -> dict:
    """cfg2's measured floor (tools/cfg2_floor.py is the standalone form): a batch that
    fits the grid once ends when its longest sequence's rows end, so the floor is those rows at the fastest
    row time the plan has -- one wave per SIMD (n = 4096 uniform-length sequences: 1,024 waves of the 16-lane
    plan's 4 sequences each) -- and the same batch size with every sequence at the longest length bounds it
    from above at this occupancy.  Both timed here, on this box, with the launches' own HIP events."""
    import torch

    from hmm_fasta_viterbi_amd.synthetic import random_batch

    def timed(codes, offsets, reps=15):
        m = len(offsets) - 1
        r = torch.from_numpy(codes).to(dev)
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        s = torch.empty(m, dtype=torch.float32, device=dev)
        od = torch.empty(m, dtype=torch.int32, device=dev)
        evs = []
        for k in range(reps + 3):
            engine.order_longest_first(o.data_ptr(), m, od.data_ptr(), sh)
            ev = (hip_event(), hip_event()) if k >= 3 else None
            if ev:
                _native.lib().msv_debug_time_next_launch(engine._p, ev[0], ev[1])
                evs.append(ev)
            engine.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), m, s.data_ptr(), od.data_ptr(), sh)
        engine.check(sh)
        torch.cuda.synchronize(dev)
        return float(np.median([hip_elapsed_ms(a, b) for a, b in evs])), engine.variant_for(m)

    from hmm_fasta_viterbi_amd import _native
    one_ms, one_var = timed(*random_batch(77, 4096, lmax, lmax))
    row_ns = one_ms * 1e6 / lmax
    uni_ms, _ = timed(*random_batch(90, n, lmax, lmax))
    floor_ms = longest * row_ns / 1e6
    return {"row_ns_one_wave_per_simd": round(row_ns, 2), "one_wave_variant": one_var, "longest_rows": int(longest),
            "floor_ms": round(floor_ms, 4), "kernel_over_floor": round(kernel_ms / floor_ms, 4),
            "uniform_longest_ms": round(uni_ms, 4), "kernel_over_uniform_longest": round(kernel_ms / uni_ms, 4),
            "note": "floor = the batch's longest sequence at the one-wave-per-SIMD row time (4,096 sequences of "
                    "the longest length, 1,024 waves); uniform_longest = this batch size with every sequence "
                    "that long (the occupancy this batch runs at, no shorter co-resident waves)"}


def per_rank_summary(allr, steps: int, scaling: str) -> dict:
    """Each rank's own figures for an N-rank line: allr = [world, 4] rows of {elapsed s,
    kernel ms, residues, sequences} as all-gathered after the timed window; min / max / max-over-min of the
    step time, kernel time and residues say whether a sub-linear curve is imbalance, the gather or launch skew."""
    allr = np.asarray(allr, np.float64)

    def spread(x):
        x = np.asarray(x, np.float64)
        return {"min": round(float(x.min()), 4), "max": round(float(x.max()), 4),
                "max_over_min": round(float(x.max() / x.min()), 4) if x.min() > 0 else None}
    step_ms = allr[:, 0] / steps * 1e3
    return {
        "ms_per_step": [round(float(v), 4) for v in step_ms],
        "kernel_ms": [round(float(v), 4) for v in allr[:, 1]],
        "residues": [int(v) for v in allr[:, 2]],
        "sequences": [int(v) for v in allr[:, 3]],
        "imbalance": {"ms_per_step": spread(step_ms), "kernel_ms": spread(allr[:, 1]), "residues": spread(allr[:, 2])},
        "step_minus_kernel_ms": [round(float(a - b), 4) for a, b in zip(step_ms, allr[:, 1])],
        "note": "each rank's own timed window (barrier-bracketed); `ms_per_step` and `kernel_ms` above are the "
                "max over ranks; a step's time beyond its kernel (step_minus_kernel_ms) is the order launch"
                + (" and the in-step RCCL all-gather" if scaling == "strong" else ""),
    }


def pmc_traffic(config: str, variant: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc passes (profiles/pmc_<config>.json,
    tools/pmc.sh -> tools/pmc_summary.py), FETCH_SIZE corrected by the factor measured for the
    kernel's read pattern (MI355X_MICROARCH.md §HBM; profiles/r02_fetch_calib.json).  Published only
    when that file measured exactly the kernel this run's timed steps launch (its recorded symbol ==
    the resident instantiation of `variant`) with a calibrated factor; otherwise None, with the reason."""
    from hmm_fasta_viterbi_amd.kernel_names import kernel_symbol
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    want = kernel_symbol(variant)
    if not os.path.exists(path):
        return None, {"file": None, "reason": "no PMC file for this config"}
    with open(path) as f:
        d = json.load(f)
    src = {"file": os.path.relpath(path, ROOT), "pmc_kernel": d.get("kernel"), "timed_kernel": want}
    if not d.get("kernel") or want not in d["kernel"]:
        return None, {**src, "reason": "PMC file measured another kernel than the timed one"}
    if not d.get("fetch_factor_calibrated"):
        return None, {**src, "reason": "FETCH_SIZE factor uncalibrated"}
    return d.get("hbm_bytes_per_launch"), src


def issue_ceiling_tcells():
    """Measured instruction-issue ceiling of the cell update as the kernel issues it
    (profiles/r01_micro_row_sched.jsonl: tools/micro/row_sched.hip, one row of the kernel's exact
    per-chunk ops -- 4 v_max + 4 v_add + 2 v_max3 per 4 cells, in the kernel's interleaved order
    and with its real dependencies -- with no memory and no per-row work, 4 waves/SIMD; best run):
    cells/ns/SIMD x 1024 SIMDs -> T cells/s."""
    path = os.path.join(ROOT, "profiles", "r01_micro_row_sched.jsonl")
    if not os.path.exists(path):
        return None
    best = None
    with open(path) as f:
        for line in f:
            d = json.loads(line)
            if d["sched"].startswith("D_max3_interleaved"):
                best = max(best or 0.0, d["cells_per_ns_per_simd"])
    return None if best is None else best * 1024 / 1000.0


def launcher_command(argv: list[str], gpus: int, port: int) -> list[str]:
    """The child command that runs this bench as `gpus` ranks (one process per GPU) when it was
    started as a plain `python bench.py --gpus N` (no torch.distributed.run around it)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def check_world(gpus: int, env=os.environ) -> str:
    """'launch' -- spawn the ranks; 'run' -- this process is a rank (or the only one).  A rank whose
    WORLD_SIZE differs from --gpus is an error: the line would report a GPU count nobody ran."""
    world = env.get("WORLD_SIZE")
    if world is None:
        return "launch" if gpus > 1 else "run"
    if int(world) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}")
    return "run"


def launch_ranks(argv: list[str], gpus: int) -> int:
    """Run the ranks as ONE child process tree (never exec: this process has not touched the GPU, and
    must not replace itself) and return its exit status; rank 0 prints the JSON line to our stdout."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    return subprocess.run(launcher_command(argv, gpus, port)).returncode


def main(args=None):
    args = args or parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert world == args.gpus, (world, args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MSV_BENCH_BACKEND=gloo + MSV_BENCH_ONE_DEVICE=1 rehearse the multi-rank path on one GPU (all ranks
    # on cuda:0, collectives on host tensors); the driver's N-GPU runs use the defaults (RCCL, one GPU
    # per rank).
    backend = os.environ.get("MSV_BENCH_BACKEND", "nccl")
    if args.dry_run:  # the launcher's plumbing, testable on a CPU-only host
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
        layout = {"dry_run": True, "n_gpus": world, "ranks": dist.get_world_size() if world > 1 else 1,
                  "local_rank": local, "config": args.config}
        if rank == 0:
            print(json.dumps(layout), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return layout
    if os.environ.get("MSV_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    cdev = dev if backend == "nccl" else torch.device("cpu")  # where collective tensors live
    dist_world = dist.get_world_size() if world > 1 else 1
    if dist_world != world:
        raise SystemExit(f"bench.py: process group has {dist_world} ranks, WORLD_SIZE {world}")

    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import distributed
    from hmm_fasta_viterbi_amd.kernel_names import kernel_symbol
    from hmm_fasta_viterbi_amd.synthetic import random_batch

    prof_name, n_cfg, lmin, lmax, seed, scaling = CONFIGS[args.config]
    prof_path = os.path.join(ROOT, "data", "profile_HMMs", prof_name)
    engine = msv.MSV_HMM(msv.Profile_HMM(prof_path), device=local)
    leng = engine.model_length - 1
    info = engine.describe()

    if scaling == "weak":  # every rank its own batch of the config's size
        codes, offsets = random_batch(seed * 1000 + rank, n_cfg, lmin, lmax)
        first, width = 0, n_cfg
    else:  # one job-wide set, residue-balanced contiguous shards (the same cut as msv_shard_bounds)
        all_codes, all_offsets = random_batch(seed, n_cfg, lmin, lmax)
        codes, offsets, first, last = distributed.shard(all_codes, all_offsets, world, rank)
        bounds = [distributed.shard_bounds(all_offsets, world, r) for r in range(world)]
        width = max(b - a for a, b in bounds)  # gather pads every shard to the largest
        del all_codes
    n = len(offsets) - 1
    # the plan this batch size runs (latency / mid / throughput, msv_device.cpp select_plan)
    variant = engine.variant_for(n)
    var_g, var_s = (int(x[1:]) for x in variant.split("_")[1:3])
    residues = int(offsets[-1])
    d_res = torch.from_numpy(codes).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    d_scores = torch.full((max(width, 1),), float("nan"), dtype=torch.float32, device=dev)
    d_order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    gathered = torch.empty(world * max(width, 1), dtype=torch.float32, device=cdev) if scaling == "strong" else None
    # A dedicated stream: torch's default (null) stream has handle 0, which the C-ABI reads as
    # "use the library's own stream"; events must be recorded on the stream the kernel runs on.
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    sh = stream.cuda_stream
    engine.reserve_length(lmax)
    engine.bind_stream(sh)  # the bench's stream outlives every launch of this engine
    from hmm_fasta_viterbi_amd import _native
    native = _native.lib()
    native.msv_debug_time_next_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    hip = C.CDLL("libamdhip64.so.7")  # torch's HIP runtime (already loaded: one runtime per process)
    hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    hip.hipEventDestroy.argtypes = [C.c_void_p]

    def hip_event():
        e = C.c_void_p()
        assert hip.hipEventCreate(C.byref(e)) == 0
        return e.value

    def hip_elapsed_ms(a, b):
        ms = C.c_float()
        assert hip.hipEventElapsedTime(C.byref(ms), a, b) == 0
        return float(ms.value)

    native.msv_debug_set_clock_stamps.argtypes = [C.c_void_p, C.c_void_p]
    native.msv_debug_grid_waves.argtypes = [C.c_void_p]

    def step(ev=None, stamps=None):
        order_ptr = None
        if not args.no_order:
            engine.order_longest_first(d_off.data_ptr(), n, d_order.data_ptr(), sh)
            order_ptr = d_order.data_ptr()
        if ev is not None:  # the MSV launch itself updates these two HIP events (hipExtLaunchKernel)
            native.msv_debug_time_next_launch(engine._p, ev[0], ev[1])
        # stamps: this launch runs the plan's CLOCK twin, every wave writing realtime + shader-clock stamps
        native.msv_debug_set_clock_stamps(engine._p, None if stamps is None else stamps.data_ptr())
        engine.score_batch_device(d_res.data_ptr(), residues, d_off.data_ptr(), n, d_scores.data_ptr(), order_ptr, sh)
        if gathered is not None and world > 1:  # cfg4: the RCCL gather of the scores is part of the step
            with torch.cuda.stream(stream):
                src = d_scores if backend == "nccl" else d_scores.cpu()
                dist.all_gather_into_tensor(gathered, src)

    # Informational end-to-end rates first (their calls also bring the GPU clock up before the timed
    # loop): host buffers -> msv_score_batch (H2D pipelined under the kernels, scores D2H), warm.
    # Pinned = residues in page-locked memory (SURVEY 8(d)'s headline shape); pageable = plain numpy.
    pinned_codes = torch.from_numpy(codes).pin_memory().numpy()

    def host_rate(src, out, settle_s=0.0):
        t = time.perf_counter()  # warm; the first call also settles the GPU clock (ramps from idle)
        while True:
            engine.score_batch(codes=src, offsets=offsets, out=out)
            if time.perf_counter() - t >= settle_s:
                break
        for _ in range(3):
            engine.score_batch(codes=src, offsets=offsets, out=out)
        t = time.perf_counter()
        for _ in range(args.steps):
            engine.score_batch(codes=src, offsets=offsets, out=out)
        return residues * args.steps / (time.perf_counter() - t) / 1e6, out.copy()

    # pinned: residues AND scores in page-locked host memory; pageable: both plain numpy arrays
    host_pinned, pinned_scores = host_rate(pinned_codes, torch.empty(n, dtype=torch.float32).pin_memory().numpy(),
                                           settle_s=0.5)
    host_pageable, pageable_scores = host_rate(codes, np.zeros(n, np.float32))
    # pinned residues are read in place by the kernel (zero-copy); the same call through the copy pipeline:
    _native.lib().msv_debug_set_zero_copy.argtypes = [C.c_void_p, C.c_int]
    _native.lib().msv_debug_set_zero_copy(engine._p, 0)
    host_pinned_copy, copy_scores = host_rate(pinned_codes, torch.empty(n, dtype=torch.float32).pin_memory().numpy())
    _native.lib().msv_debug_set_zero_copy(engine._p, 1)

    # Stream of batches (serving): msv_score_batch_async keeps three calls in flight, so the H2D of the
    # next calls runs back to back under the current call's kernel; scores land in pinned host arrays.
    outs = [torch.empty(n, dtype=torch.float32).pin_memory().numpy() for _ in range(3)]

    def streamed_rate():
        for _ in range(3):
            engine.wait(engine.score_batch_async(pinned_codes, offsets, outs[0]))
        t = time.perf_counter()
        inflight = []
        for k in range(args.steps):
            inflight.append(engine.score_batch_async(pinned_codes, offsets, outs[k % 3]))
            if len(inflight) == 3:
                engine.wait(inflight.pop(0))
        for tk in inflight:
            engine.wait(tk)
        return residues * args.steps / (time.perf_counter() - t) / 1e6

    host_streamed = streamed_rate()
    streamed_scores = outs[(args.steps - 1) % 3].copy()

    # Information, never `value` (run BEFORE the timed steps, so those stay the last K MSV dispatches for
    # tools/rocprof_window.py): K steps as a stream of resident batches alternating over two streams, so
    # each step's blocks take the CUs that the previous step's drain tail frees (what
    # msv_score_batch_async does for host batches).  Every step still sorts and scores its whole batch.
    stream_b = torch.cuda.Stream(dev)
    d_scores_b = torch.full_like(d_scores, float("nan"))
    d_order_b = torch.empty_like(d_order)
    lanes = [(stream, d_scores, d_order), (stream_b, d_scores_b, d_order_b)]

    def step_two_streams(k):
        st, sc, od = lanes[k % 2]
        order_ptr = None
        if not args.no_order:
            engine.order_longest_first(d_off.data_ptr(), n, od.data_ptr(), st.cuda_stream)
            order_ptr = od.data_ptr()
        engine.score_batch_device(d_res.data_ptr(), residues, d_off.data_ptr(), n, sc.data_ptr(), order_ptr,
                                  st.cuda_stream)

    for k in range(2):
        step_two_streams(k)
    torch.cuda.synchronize(dev)
    tb = time.perf_counter()
    for k in range(args.steps):
        step_two_streams(k)
    torch.cuda.synchronize(dev)
    two_stream_rate = residues * args.steps / (time.perf_counter() - tb) / 1e6
    engine.check(sh)
    two_stream_scores = (d_scores[:n].cpu().numpy().copy(), d_scores_b[:n].cpu().numpy().copy())

    for _ in range(args.warmup):
        step()
    engine.check(sh)  # raises on any latched kernel error
    torch.cuda.synchronize(dev)

    # Kernel timing: HIP events that the MSV launch updates with its own start and end (hipExtLaunchKernel on
    # the launch stream), not event records around it -- each record is a marker packet (~4 us in the
    # stream), which would add ~8 us to every step (7% of cfg2's).
    events = [(hip_event(), hip_event()) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(None if args.no_launch_events else events[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    engine.check(sh)
    # The timed launches' own scores, before the CLOCK twin below writes the same buffer again: these are
    # what every equality check and the CPU baseline compare against.
    timed_scores = d_scores[:n].cpu().numpy().copy()
    # Clock under this load: `steps` more steps right after the timed window, the same batch and plan, run
    # by the plan's CLOCK twin (msv_kernel_impl.h clock_fn: the production kernel whose per-wave stamps also
    # record s_memtime -- one tick per shader cycle -- beside s_memrealtime at 100 MHz; a separate
    # instantiation, so the timed kernel's ISA is untouched).  clock = sum of ticks / sum of realtime over
    # the waves of a launch, median over the launches; the twin's own kernel time is reported beside it.
    clock = None
    if not args.no_clock:
        nwaves = int(native.msv_debug_grid_waves(engine._p))
        bufs = [torch.zeros(nwaves * 6, dtype=torch.int64, device=dev) for _ in range(args.steps)]
        cev = [(hip_event(), hip_event()) for _ in range(args.steps)]
        for k in range(args.steps):
            step(cev[k], bufs[k])
        native.msv_debug_set_clock_stamps(engine._p, None)
        torch.cuda.synchronize(dev)
        engine.check(sh)
        per_launch = []
        for b in bufs:
            a = b.cpu().numpy().reshape(nwaves, 6)
            a = a[(a[:, 1] > 0) & (a[:, 5] > 0)]
            rt, ck = (a[:, 1] - a[:, 0]).sum(), (a[:, 5] - a[:, 4]).sum()
            if rt > 0:
                per_launch.append(float(ck) / float(rt) * 0.1)  # GHz
        twin_ms = float(np.mean([hip_elapsed_ms(a, b) for a, b in cev]))
        for a, b in cev:
            hip.hipEventDestroy(a)
            hip.hipEventDestroy(b)
        if per_launch:
            clock = {"median": round(float(np.median(per_launch)), 4), "min": round(float(min(per_launch)), 4),
                     "max": round(float(max(per_launch)), 4), "launches": len(per_launch),
                     "twin_kernel_ms": round(twin_ms, 4)}
    elapsed = t1 - t0
    kernel_ms = float("nan") if args.no_launch_events else float(np.mean([hip_elapsed_ms(a, b) for a, b in events]))
    for a, b in events:
        hip.hipEventDestroy(a)
        hip.hipEventDestroy(b)
    residues_all = residues
    per_rank = None
    if world > 1:
        # every rank's own figures (so an N-rank line explains itself: imbalance vs gather vs launch skew),
        # then the contract's max-over-ranks time and the job's total residues
        mine = torch.tensor([elapsed, kernel_ms, float(residues), float(n)], dtype=torch.float64, device=cdev)
        allr = torch.empty(world * 4, dtype=torch.float64, device=cdev)
        dist.all_gather_into_tensor(allr, mine)
        allr = allr.cpu().numpy().reshape(world, 4)
        elapsed, kernel_ms = float(allr[:, 0].max()), float(allr[:, 1].max())
        residues_all = int(allr[:, 2].sum())
        per_rank = per_rank_summary(allr, args.steps, scaling)

    # weak configs: output collection after timing (RCCL all-gather of every rank's scores)
    gather_ms = None
    if world > 1 and gathered is None:
        torch.cuda.synchronize(dev)
        g0 = time.perf_counter()
        full = torch.empty(world * n, dtype=torch.float32, device=cdev)
        dist.all_gather_into_tensor(full, d_scores[:n].to(cdev))
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) * 1e3

    scores = timed_scores
    twin_scores = d_scores[:n].cpu().numpy()  # the CLOCK twin's launches (after the timed window)
    twin_equal = bool(np.array_equal(twin_scores.view(np.uint32), scores.view(np.uint32)))
    d_scores[:n].copy_(torch.from_numpy(timed_scores))  # the Viterbi stage filters the timed launches' scores
    ok = bool(np.all(np.isfinite(scores)))
    ok = ok and bool(np.array_equal(pinned_scores.view(np.uint32), scores.view(np.uint32)))
    ok = ok and bool(np.array_equal(pageable_scores.view(np.uint32), scores.view(np.uint32)))
    ok = ok and bool(np.array_equal(streamed_scores.view(np.uint32), scores.view(np.uint32)))
    ok = ok and all(bool(np.array_equal(x.view(np.uint32), scores.view(np.uint32))) for x in two_stream_scores)
    ok = ok and bool(np.array_equal(copy_scores.view(np.uint32), scores.view(np.uint32)))
    if gathered is not None and world > 1:  # every shard landed at its rows of the gathered set
        g = gathered.cpu().numpy().reshape(world, -1)
        ok = ok and bool(np.array_equal(g[rank, :n].view(np.uint32), scores.view(np.uint32)))
    value = residues_all * args.steps / elapsed / 1e6  # M residues / s, whole job
    gcups = value * 1e6 * leng / 1e9

    result = None
    if rank == 0:
        cells_per_launch = residues * leng
        achieved = 3.0 * cells_per_launch / (kernel_ms * 1e-3) / 1e12
        alg_bytes = residues + n * (8 + 8 + 4 + 4) + 21 * var_g * var_s * 4
        traffic, traffic_src = pmc_traffic(args.config, variant)
        ceiling = issue_ceiling_tcells()
        per = "per GPU" if scaling == "weak" else f"in one set, {world} residue-balanced shard(s)"
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "M residues/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: seeded uniform residues (random_FASTA_generator.py format), lengths uniform "
                    f"[{lmin},{lmax}]; real Pfam profile {prof_name}",
            "config": {
                "workload": f"{args.config}: {prof_name} (LENG={leng}) x {n_cfg} sequences {per}, "
                            f"len U[{lmin},{lmax}], inputs resident in HBM",
                "profile": prof_name,
                "sequences_rank0": n,
                "residues_rank0": residues,
                "residues_all_ranks": residues_all,
                "parallelism": f"dp{world} (sequence shards, no data-path collective"
                               + ("; RCCL all-gather of the scores in every step)" if scaling == "strong" else ")"),
                "kernel_variant": variant,
                "kernel_symbol": kernel_symbol(variant),
                "rccl_world_size": dist_world if backend == "nccl" else None,
                "collective_backend": backend if world > 1 else None,
                "dequeue_order": "input" if args.no_order else "longest-first",
            },
            "gcups": round(gcups, 2),
            "kernel_ms": round(kernel_ms, 4),
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": round(VALU_PEAK_TOPS, 2),
                "unit": "TFLOP/s",
                "frac": round(achieved / VALU_PEAK_TOPS, 4),
                "clock_GHz": None if clock is None else clock["median"],
                "frac_at_clock": None if clock is None else round(
                    achieved / (256 * 128 * clock["median"] * 1e9 / 1e12), 4),
                "clock": None if clock is None else {
                    **clock, "source": "in-kernel, over `steps` launches right after the timed window (same batch "
                                       "and plan) by the plan's CLOCK twin, whose waves stamp s_memtime (one tick "
                                       "per shader cycle) and s_memrealtime (100 MHz) at start and end; clock = sum "
                                       "of ticks / sum of realtime over the waves, median over the launches; "
                                       "twin_kernel_ms vs kernel_ms shows the twin ran like the timed kernel; "
                                       "frac_at_clock = achieved / (256 CU x 128 lanes x clock)"},
                "traffic": traffic,
                "traffic_source": traffic_src,
                "note": "fp32 add/max ops: 3 per DP cell (cells = residues x LENG); peak = 256 CU x 128 "
                        "lanes/clk x 2.4 GHz non-FMA VALU; HBM is not the bound (see hbm); traffic = "
                        "calibrated FETCH_SIZE + WRITE_SIZE per launch (profiles/pmc_<config>.json)",
            },
            "issue_ceiling": None if ceiling is None else {
                "tcells_per_s": round(ceiling, 3),
                "achieved_tcells_per_s": round(cells_per_launch / (kernel_ms * 1e-3) / 1e12, 3),
                "frac": round(cells_per_launch / (kernel_ms * 1e-3) / 1e12 / ceiling, 4),
                "source": "profiles/r01_micro_row_sched.jsonl (measured: v_max/v_max3 issue at half the "
                          "v_add rate, so 2.5 VALU/cell cannot reach the nominal peak; kernel's interleaved "
                          "chunk order, no per-row work)",
            },
            "hbm": {
                "algorithmic_bytes_per_launch": alg_bytes,
                "achieved_GBps": round(alg_bytes / (kernel_ms * 1e-3) / 1e9, 2),
                "peak_GBps": HBM_PEAK_GBPS,
            },
            "gather_ms": gather_ms,
            "per_rank": per_rank,
            "end_to_end": {
                "host_pinned_M_residues_s": round(host_pinned, 1),
                "host_pageable_M_residues_s": round(host_pageable, 1),
                "host_pinned_copy_pipeline_M_residues_s": round(host_pinned_copy, 1),
                "pinned_frac_of_value": round(host_pinned / (residues * args.steps / elapsed / 1e6), 4),
                "host_pinned_streamed_M_residues_s": round(host_streamed, 1),
                "streamed_frac_of_value": round(host_streamed / (residues * args.steps / elapsed / 1e6), 4),
                "resident_two_streams_M_residues_s": round(two_stream_rate, 1),
                "two_streams_frac_of_value": round(two_stream_rate / (residues * args.steps / elapsed / 1e6), 4),
                "note": "SURVEY 8(d)'s 'GPU timing' headline is host_pinned (packed residues in pinned host "
                        "memory -> msv_score_batch: offsets H2D, order, ONE kernel reading the residues in "
                        "place over PCIe (zero-copy), scores written to the pinned destination by the "
                        "kernel; rank 0, warm, mean of `steps` calls); host_pinned_copy_pipeline = the same "
                        "call with the residues copied in pieces under the kernels; host_pinned_streamed = the same batch as a stream of `steps` "
                        "msv_score_batch_async calls, three in flight (the copies of the next calls under the "
                        "current kernel, kernels on alternating streams); resident_two_streams = `steps` resident "
                        "steps before the timed ones, alternating over two streams so each step's blocks fill the previous "
                        "step's drain tail; `value` is the HBM-resident rate of serial steps the bench "
                        "contract prescribes",
            },
            "scores_finite_and_consistent": ok,
            "scores_checked": "the timed launches' own scores (copied to the host right after the timed "
                              "window, before the CLOCK-twin pass reuses the buffer): finiteness, the host paths, "
                              "the two-stream pass and cpu_baseline.bitwise_equal_to_gpu compare against them",
            "clock_twin_scores_bitwise_equal": twin_equal,
        }
        if args.config == "cfg2":  # the latency-bound config: its measured floor beside the kernel
            result["latency_ceiling"] = latency_ceiling(engine, dev, sh, n, lmax,
                                                        int(np.diff(offsets.astype(np.int64)).max()), kernel_ms,
                                                        hip_event, hip_elapsed_ms)
        if not args.no_viterbi:
            result["viterbi_stage"] = viterbi_stage(args, engine, prof_path, dev, stream, d_res, residues, d_off, n,
                                                    d_scores, None if args.no_order else d_order, codes, offsets,
                                                    lmax, leng, hip_event, hip_elapsed_ms)
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(prof_path, codes, offsets, scores, args.cpu_seconds,
                                                  cpu_threads(args.cpu_threads))
            cb = result["cpu_baseline"]
            result["speedup_vs_cpu_baseline"] = round(value / cb["value"], 1)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    _args = parse()
    if check_world(_args.gpus) == "launch":
        sys.exit(launch_ranks(sys.argv[1:], _args.gpus))
    main(_args)
