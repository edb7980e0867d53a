"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own CPU path.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (where /root/reference exists) against
oracle/_ref/libref_msv.so, i.e. the reference sources compiled by oracle/Makefile:
    Profile_HMM / FASTA_protein_sequences parsers   data_readers/*.cpp
    MSV_HMM::run_on_sequence                          algorithms/MSV_HMM.cpp:74-113
Outputs are data only (inputs + expected outputs); no reference source is stored.

Usage:  python oracle/make_golden.py   (after `make -C oracle all ref`)
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "data")
GOLD = os.path.join(ROOT, "tests", "golden")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_msv.so")

PROFILES = sorted((f for f in os.listdir(os.path.join(DATA, "profile_HMMs")) if f.endswith(".hmm")),
                  key=lambda f: int(f.split(".")[0]))


def load_ref():
    lib = C.CDLL(REF_SO)
    lib.ref_score_fasta.restype = C.c_long
    lib.ref_score_fasta.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(C.c_float), C.POINTER(C.c_uint64), C.c_long]
    lib.ref_fasta_dump.restype = C.c_long
    lib.ref_fasta_dump.argtypes = [C.c_char_p, C.c_char_p, C.c_long]
    lib.ref_hmm_dump.restype = C.c_long
    lib.ref_hmm_dump.argtypes = [C.c_char_p, C.c_char_p, C.c_long, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                 C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_long]
    lib.ref_score_codes.restype = C.c_double
    lib.ref_score_codes.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_long, C.c_int, C.c_void_p]
    return lib


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def hexf(x: float) -> str:
    return float(np.float32(x)).hex()


def score_fasta(lib, hmm, fsa):
    scores = np.zeros(4096, np.float32)
    lens = np.zeros(4096, np.uint64)
    n = lib.ref_score_fasta(hmm.encode(), fsa.encode(), fptr(scores), lens.ctypes.data_as(C.POINTER(C.c_uint64)),
                            4096)
    return scores[:n].copy(), lens[:n].copy()


def fasta_dump(lib, fsa):
    need = lib.ref_fasta_dump(fsa.encode(), None, 0)
    buf = C.create_string_buffer(need)
    lib.ref_fasta_dump(fsa.encode(), buf, need)
    text = buf.value.decode("latin-1")
    return text.split("\n")[:-1]


def hmm_dump(lib, hmm):
    name = C.create_string_buffer(256)
    stats = np.zeros(6, np.float32)
    m = lib.ref_hmm_dump(hmm.encode(), name, 256, fptr(stats), None, None, None, 0)
    match = np.zeros((m, 20), np.float32)
    ins = np.zeros((m, 20), np.float32)
    tr = np.zeros((m, 7), np.float32)
    lib.ref_hmm_dump(hmm.encode(), name, 256, fptr(stats), fptr(match), fptr(ins), fptr(tr), m)
    return name.value.decode(), int(m), stats, match, ins, tr


def make_batch(seed: int, lengths):
    """Seeded synthetic residue-code batch (uniform over the 20 amino acids)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = np.asarray(lengths, dtype=np.uint64)
    offsets = np.zeros(len(lengths) + 1, np.uint64)
    offsets[1:] = np.cumsum(lengths)
    codes = rng.integers(0, 20, size=int(offsets[-1]), dtype=np.uint8)
    return codes, offsets


EDGE_LENGTHS = [0, 1, 2, 3, 4, 5, 7, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 255, 256, 257, 1000,
                3500]


def main():
    lib = load_ref()
    os.makedirs(GOLD, exist_ok=True)
    manifest = {"generator": "oracle/make_golden.py", "reference_cpu_path": "algorithms/MSV_HMM.cpp:74-113"}

    # (1) Appendix-B style: every profile x fasta_like_example.fsa (test_MSV.cpp:14-36 inputs)
    ex = os.path.join(DATA, "FASTA_files", "fasta_like_example.fsa")
    rows = []
    for p in PROFILES:
        s, lens = score_fasta(lib, os.path.join(DATA, "profile_HMMs", p), ex)
        for i, (x, L) in enumerate(zip(s, lens)):
            rows.append(f"{p}\t{i}\t{int(L)}\t{hexf(x)}\t{float(x):.9g}")
    with open(os.path.join(GOLD, "example_scores.tsv"), "w") as f:
        f.write("#profile\tseq\tlength\tscore_hex\tscore\n" + "\n".join(rows) + "\n")

    # (2) random_FASTA.fsa (benchmark_MSV_1400 input) x every profile
    rf = os.path.join(DATA, "FASTA_files", "random_FASTA.fsa")
    rows = []
    for p in PROFILES:
        s, lens = score_fasta(lib, os.path.join(DATA, "profile_HMMs", p), rf)
        for i, (x, L) in enumerate(zip(s, lens)):
            rows.append(f"{p}\t{i}\t{int(L)}\t{hexf(x)}\t{float(x):.9g}")
    with open(os.path.join(GOLD, "random_fasta_scores.tsv"), "w") as f:
        f.write("#profile\tseq\tlength\tscore_hex\tscore\n" + "\n".join(rows) + "\n")

    # (3) seeded synthetic batches with edge lengths, for the three north_star profiles
    rng = np.random.Generator(np.random.PCG64(12345))
    for p, seed in (("100.hmm", 101), ("1400.hmm", 1401), ("2405.hmm", 2406)):
        lengths = EDGE_LENGTHS + list(rng.integers(1, 800, size=120))
        codes, offsets = make_batch(seed, lengths)
        scores = np.zeros(len(lengths), np.float32)
        t = lib.ref_score_codes(os.path.join(DATA, "profile_HMMs", p).encode(), codes.ctypes.data,
                                offsets.ctypes.data, len(lengths), 8, scores.ctypes.data)
        assert t >= 0
        np.savez(os.path.join(GOLD, f"seeded_{p.split('.')[0]}.npz"), codes=codes, offsets=offsets, scores=scores)

    # (4) every profile x 24 seeded sequences (covers every kernel variant)
    allp = {}
    for k, p in enumerate(PROFILES):
        lengths = [0, 1, 2] + list(rng.integers(1, 700, size=21))
        codes, offsets = make_batch(7000 + k, lengths)
        scores = np.zeros(len(lengths), np.float32)
        t = lib.ref_score_codes(os.path.join(DATA, "profile_HMMs", p).encode(), codes.ctypes.data,
                                offsets.ctypes.data, len(lengths), 8, scores.ctypes.data)
        assert t >= 0
        key = p.split(".")[0]
        allp[f"codes_{key}"] = codes
        allp[f"offsets_{key}"] = offsets
        allp[f"scores_{key}"] = scores
    np.savez(os.path.join(GOLD, "seeded_all_profiles.npz"), **allp)

    # (5) parser fixtures: full arrays for 100.hmm and 1301.hmm (HMMER3.0 header), digests for all
    digests = {}
    for p in PROFILES:
        name, m, stats, match, ins, tr = hmm_dump(lib, os.path.join(DATA, "profile_HMMs", p))
        digests[p] = {
            "name": name, "model_length": m, "stats_hex": [hexf(x) for x in stats],
            "match_sha256": hashlib.sha256(match.tobytes()).hexdigest(),
            "insert_sha256": hashlib.sha256(ins.tobytes()).hexdigest(),
            "transitions_sha256": hashlib.sha256(tr.tobytes()).hexdigest(),
        }
        if p in ("100.hmm", "1301.hmm"):
            np.savez(os.path.join(GOLD, f"parsed_{p.split('.')[0]}.npz"), match=match, insert=ins, transitions=tr,
                     stats=stats)
    with open(os.path.join(GOLD, "parsed_profiles.json"), "w") as f:
        json.dump(digests, f, indent=1, sort_keys=True)

    # (6) FASTA parser fixtures (reference parse of the bundled files and of an edge-case file)
    edge = os.path.join(GOLD, "edge_cases.fsa")
    with open(edge, "w", newline="") as f:
        f.write(">ok plain\nACDEFGHIKLMNPQRSTVWY\n"
                ">lower case rejected\nACDEfGH\n"
                ">X rejected\nACDXEF\n"
                ">star rejected\nACD*\n"
                ">crlf rejected\r\nACDE\r\nFGH\r\n"
                ">empty record kept\n"
                ">hash kept by parser\nAC#DE\n"
                ">multi line joined\nAAAA\nCCCC\n\nDDDD\n"
                ">space rejected\nAC DE\n"
                ">last\nWWWWWWWWWW\n")
    dumps = {}
    for fsa in (ex, rf, edge):
        dumps[os.path.basename(fsa)] = fasta_dump(lib, fsa)
    with open(os.path.join(GOLD, "fasta_parsed.json"), "w") as f:
        json.dump(dumps, f, indent=1)

    manifest["files"] = sorted(os.listdir(GOLD))
    with open(os.path.join(GOLD, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("golden fixtures written to", GOLD)


if __name__ == "__main__":
    sys.exit(main())
