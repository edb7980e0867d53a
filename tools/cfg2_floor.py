"""cfg2's measured latency floor: the per-row time of the real g16_s8 row chain (cells,
per-lane E, J partials, the wave-level J >= N test, B) at 1, 2 and 3 waves per SIMD, and what the cfg2
launch would take if every lane group's sequence had the batch's longest length.

The "micro-benchmark" is the production kernel itself (no re-implementation to drift from it): batches of
uniform-length sequences (500 residues, cfg2's maximum) sized so that every SIMD holds exactly W waves
(100.hmm's 16-lane plan: 4 sequences per wave, 4 waves per workgroup, one workgroup per CU per round:
n = 4096 W), timed with HIP events; ns per row = kernel time / 500.  Then:
  floor_uniform500_ms -- cfg2's own occupancy (10,000 sequences -> 2,500 waves on 1,024 SIMDs) with every
                         sequence 500 residues long: the launch cannot end before its longest sequences do,
                         and no other length mix keeps more waves on a SIMD;
  cfg2_kernel_ms      -- the real cfg2 batch (bench.py's rank-0 batch, seed 1000, U[300,500]).

    python tools/cfg2_floor.py [--variant msv_g16_s8_w4_p2_d1] [--out profiles/r04_cfg2_floor.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="")
    ap.add_argument("--rows", type=int, default=500)
    ap.add_argument("--launches", type=int, default=30)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch

    eng = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", "100.hmm")))
    if args.variant:
        eng.set_variant(args.variant)
    native = _native.lib()
    native.msv_debug_time_next_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    eng.bind_stream(st.cuda_stream)

    def ev():
        e = C.c_void_p()
        assert hip.hipEventCreate(C.byref(e)) == 0
        return e.value

    def kernel_ms(codes, offsets):
        n = len(offsets) - 1
        r = torch.from_numpy(codes).to(dev)
        o = torch.from_numpy(offsets.view(np.int64)).to(dev)
        s = torch.empty(n, dtype=torch.float32, device=dev)
        order = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        times = []
        for k in range(args.launches + 10):
            eng.order_longest_first(o.data_ptr(), n, order.data_ptr(), st.cuda_stream)
            pair = (ev(), ev())
            native.msv_debug_time_next_launch(eng._p, pair[0], pair[1])
            eng.score_batch_device(r.data_ptr(), r.numel(), o.data_ptr(), n, s.data_ptr(), order.data_ptr(),
                                   st.cuda_stream)
            if k >= 10:
                times.append(pair)
        eng.check(st.cuda_stream)
        torch.cuda.synchronize()
        ms = []
        for a, b in times:
            t = C.c_float()
            assert hip.hipEventElapsedTime(C.byref(t), a, b) == 0
            ms.append(float(t.value))
        return float(np.median(ms)), eng.variant_for(n)

    rows = args.rows
    out = {"tool": "tools/cfg2_floor.py", "profile": "100.hmm", "rows": rows, "per_row_ns": {}}
    for w in (1, 2, 3):
        n = 4096 * w
        codes, offsets = random_batch(77 + w, n, rows, rows)
        ms, var = kernel_ms(codes, offsets)
        out["per_row_ns"][str(w)] = round(ms * 1e6 / rows, 2)
        out.setdefault("variant", var)
        out[f"kernel_ms_w{w}"] = round(ms, 4)
    codes, offsets = random_batch(90, 10_000, rows, rows)
    out["floor_uniform500_ms"], _ = kernel_ms(codes, offsets)
    codes, offsets = random_batch(1000, 10_000, 300, 500)  # bench.py --config cfg2, rank 0
    out["cfg2_kernel_ms"], out["cfg2_variant"] = kernel_ms(codes, offsets)
    out["cfg2_over_floor"] = round(out["cfg2_kernel_ms"] / out["floor_uniform500_ms"], 4)
    out["floor_uniform500_ms"] = round(out["floor_uniform500_ms"], 4)
    out["cfg2_kernel_ms"] = round(out["cfg2_kernel_ms"], 4)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
