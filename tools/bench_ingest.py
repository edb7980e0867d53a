"""FASTA ingest throughput: host reader vs GPU parse, and file -> scores end to end.

    python tools/bench_ingest.py [--n 1000000] [--profile 1400.hmm]

Writes a seeded FASTA file (random_FASTA_generator.py format, lengths U[300,500]) to /tmp, then:
  host_read    msv_fasta_read (chunked multi-threaded C++ reader)
  device_read  msv_fasta_read_device (pinned 64 MiB pieces, read/copy overlapped, tile-scan parse)
  device_parse msv_fasta_parse_device on text already in HBM (the parse kernels alone)
  end_to_end   device_read + longest-first order + MSV scores on the GPU
One JSON line.  Both parses are checked equal (codes, offsets) before timing is reported.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def best(fn, reps=3):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--profile", default="1400.hmm")
    ap.add_argument("--path", default="/tmp/msv_ingest.fsa")
    args = ap.parse_args()
    import torch
    import hmm_fasta_viterbi_amd as msv
    from hmm_fasta_viterbi_amd import _native
    from hmm_fasta_viterbi_amd.synthetic import random_batch, write_fasta

    codes, offsets = random_batch(3, args.n, 300, 500)
    write_fasta(args.path, codes, offsets)
    size = os.path.getsize(args.path)
    L = _native.lib()

    def host_read():
        f = C.c_void_p()
        assert L.msv_fasta_read(args.path.encode(), C.byref(f)) == 0
        L.msv_fasta_destroy(f)

    def device_read():
        msv.FASTA_device(args.path).close()

    t_host = best(host_read)
    t_dev = best(device_read)
    dev = msv.FASTA_device(args.path)
    c, o, _ = dev.download()
    host = msv.FASTA_protein_sequences(args.path)
    equal = bool(np.array_equal(c, host.codes) and np.array_equal(o, host.offsets))
    text_ptr = L.msv_fasta_device_text(dev._f)

    def device_parse():
        msv.FASTA_device(text_ptr=text_ptr, n=size).close()

    t_parse = best(device_parse)
    e = msv.MSV_HMM(msv.Profile_HMM(os.path.join(ROOT, "data", "profile_HMMs", args.profile)))
    e.reserve_length(500)
    scores = torch.empty(args.n, dtype=torch.float32, device="cuda:0")
    order = torch.empty(args.n, dtype=torch.int32, device="cuda:0")
    st = torch.cuda.Stream(torch.device("cuda:0"))

    def end_to_end():
        d = msv.FASTA_device(args.path, stream=st.cuda_stream)
        e.order_longest_first(d.offsets_ptr, d.count, order.data_ptr(), st.cuda_stream)
        e.score_batch_device(d.codes_ptr, d.residues, d.offsets_ptr, d.count, scores.data_ptr(), order.data_ptr(),
                             st.cuda_stream)
        e.check(st.cuda_stream)
        d.close()

    t_e2e = best(end_to_end, reps=2)
    residues = int(offsets[-1])
    print(json.dumps({
        "file_MB": round(size / 1e6, 1), "sequences": args.n, "residues": residues, "parse_equal": equal,
        "host_read_s": round(t_host, 4), "host_read_MBps": round(size / t_host / 1e6, 1),
        "device_read_s": round(t_dev, 4), "device_read_MBps": round(size / t_dev / 1e6, 1),
        "device_parse_s": round(t_parse, 5), "device_parse_GBps": round(size / t_parse / 1e9, 2),
        "end_to_end_s": round(t_e2e, 4), "end_to_end_M_residues_s": round(residues / t_e2e / 1e6, 1),
        "profile": args.profile,
        "note": "device_parse includes device allocation of the outputs and two small D2H count reads",
    }))
    dev.close()
    os.remove(args.path)


if __name__ == "__main__":
    main()
