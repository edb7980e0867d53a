"""Test-side loader of the parity checkers under oracle/ (TEST INFRASTRUCTURE ONLY).

    oracle/_build/libmsv_oracle.so : plain-C restatement of the reference CPU path
    oracle/_ref/libref_msv.so      : the reference's own CPU path (built where /root/reference exists)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libmsv_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_msv.so")
DATA = os.path.join(ROOT, "data")
GOLD = os.path.join(ROOT, "tests", "golden")
PROFILES = sorted((f for f in os.listdir(os.path.join(DATA, "profile_HMMs")) if f.endswith(".hmm")),
                  key=lambda f: int(f.split(".")[0]))

_oracle = None


def profile_path(name: str) -> str:
    return os.path.join(DATA, "profile_HMMs", name if name.endswith(".hmm") else name + ".hmm")


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
        L = C.CDLL(ORACLE_SO)
        vp = C.c_void_p
        L.oracle_profile_load.restype = vp
        L.oracle_profile_load.argtypes = [C.c_char_p]
        L.oracle_profile_free.argtypes = [vp]
        L.oracle_profile_model_length.restype = C.c_size_t
        L.oracle_profile_model_length.argtypes = [vp]
        L.oracle_profile_name.restype = C.c_char_p
        L.oracle_profile_name.argtypes = [vp]
        for f in ("emission_scores", "match_emissions", "insert_emissions", "transitions"):
            fn = getattr(L, "oracle_profile_" + f)
            fn.restype = C.POINTER(C.c_float)
            fn.argtypes = [vp]
        L.oracle_profile_constants.argtypes = [vp, C.POINTER(C.c_float)]
        L.oracle_profile_stats.argtypes = [vp, C.POINTER(C.c_float)]
        L.oracle_profile_score_codes.restype = C.c_float
        L.oracle_profile_score_codes.argtypes = [vp, vp, C.c_size_t]
        L.oracle_profile_score_string.restype = C.c_float
        L.oracle_profile_score_string.argtypes = [vp, C.c_char_p]
        L.oracle_profile_score_batch.argtypes = [vp, vp, vp, C.c_size_t, vp]
        L.oracle_seq_transitions.argtypes = [C.c_size_t, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.oracle_profile_vit_prepare.restype = C.c_int
        L.oracle_profile_vit_prepare.argtypes = [vp, C.c_int]
        L.oracle_profile_vit_tables.argtypes = [vp, C.c_int, vp, vp]
        L.oracle_profile_vit_score_batch.argtypes = [vp, C.c_int, vp, vp, C.c_size_t, vp]
        L.oracle_vit_score_tables.argtypes = [vp, vp, vp, C.c_size_t, C.c_float, C.c_float, C.c_float, vp, vp,
                                              C.c_size_t, vp]
        _oracle = L
    return _oracle


class OracleProfile:
    def __init__(self, name: str):
        self.L = oracle()
        self.p = self.L.oracle_profile_load(profile_path(name).encode())
        assert self.p, name
        self.model_length = int(self.L.oracle_profile_model_length(self.p))

    def emission_scores(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.L.oracle_profile_emission_scores(self.p), (20, self.model_length)).copy()

    def constants(self):
        out = (C.c_float * 6)()
        self.L.oracle_profile_constants(self.p, out)
        return list(out)[:3]

    def stats(self):
        out = (C.c_float * 6)()
        self.L.oracle_profile_stats(self.p, out)
        return np.array(list(out), np.float32)

    def arrays(self):
        M = self.model_length
        g = lambda f, w: np.ctypeslib.as_array(getattr(self.L, "oracle_profile_" + f)(self.p), (M, w)).copy()
        return g("match_emissions", 20), g("insert_emissions", 20), g("transitions", 7)

    def name(self) -> str:
        return self.L.oracle_profile_name(self.p).decode()

    def score_batch(self, codes: np.ndarray, offsets: np.ndarray, threads: int = 1) -> np.ndarray:
        """Oracle scores of a CSR batch; `threads` > 1 splits the sequences over host threads (the
        oracle profile is read-only, and ctypes releases the GIL during each call)."""
        codes = np.ascontiguousarray(codes, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        out = np.zeros(n, np.float32)
        base = codes.ctypes.data if codes.size else None

        def run(lo, hi):
            if hi > lo:
                self.L.oracle_profile_score_batch(self.p, base, offsets[lo:].ctypes.data, hi - lo,
                                                  out[lo:].ctypes.data)

        if threads <= 1 or n < 2 * threads:
            run(0, n)
            return out
        from concurrent.futures import ThreadPoolExecutor
        cuts = np.linspace(0, n, threads + 1).astype(np.int64)
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda k: run(int(cuts[k]), int(cuts[k + 1])), range(threads)))
        return out

    def vit_tables(self, insert_mode: int = 0):
        """(insert scores [20][M], log transitions [M][7]) of the Viterbi restatement."""
        M = self.model_length
        isc = np.zeros((20, M), np.float32)
        tsc = np.zeros((M, 7), np.float32)
        assert self.L.oracle_profile_vit_prepare(self.p, insert_mode) == 0
        self.L.oracle_profile_vit_tables(self.p, insert_mode, isc.ctypes.data, tsc.ctypes.data)
        return isc, tsc

    def vit_score_batch(self, codes: np.ndarray, offsets: np.ndarray, insert_mode: int = 0,
                        threads: int = 1) -> np.ndarray:
        """Viterbi-stage scores of the serial restatement (oracle_vit_run_codes)."""
        codes = np.ascontiguousarray(codes, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        out = np.zeros(n, np.float32)
        assert self.L.oracle_profile_vit_prepare(self.p, insert_mode) == 0
        base = codes.ctypes.data if codes.size else None

        def run(lo, hi):
            if hi > lo:
                self.L.oracle_profile_vit_score_batch(self.p, insert_mode, base, offsets[lo:].ctypes.data, hi - lo,
                                                      out[lo:].ctypes.data)

        if threads <= 1 or n < 2 * threads:
            run(0, n)
            return out
        from concurrent.futures import ThreadPoolExecutor
        cuts = np.linspace(0, n, threads + 1).astype(np.int64)
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda k: run(int(cuts[k]), int(cuts[k + 1])), range(threads)))
        return out

    def score_string(self, seq: str) -> float:
        return float(self.L.oracle_profile_score_string(self.p, seq.encode()))

    def __del__(self):
        if getattr(self, "p", None):
            self.L.oracle_profile_free(self.p)
            self.p = None


def vit_score_tables(msc, isc, tsc, consts, codes, offsets) -> np.ndarray:
    """The oracle's Viterbi DP over caller tables (msc/isc [20][M], tsc [M][7]; isc None = zero)."""
    L = oracle()
    msc = np.ascontiguousarray(msc, np.float32)
    tsc = np.ascontiguousarray(tsc, np.float32)
    isc = None if isc is None else np.ascontiguousarray(isc, np.float32)
    codes = np.ascontiguousarray(codes, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    out = np.zeros(n, np.float32)
    L.oracle_vit_score_tables(msc.ctypes.data, None if isc is None else isc.ctypes.data, tsc.ctypes.data,
                              msc.shape[1], *[float(x) for x in consts], codes.ctypes.data if codes.size else None,
                              offsets.ctypes.data, n, out.ctypes.data)
    return out


def make_batch(seed: int, lengths) -> tuple[np.ndarray, np.ndarray]:
    """Seeded synthetic CSR batch (same generator as oracle/make_golden.py and bench.py)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = np.asarray(lengths, dtype=np.uint64)
    offsets = np.zeros(len(lengths) + 1, np.uint64)
    offsets[1:] = np.cumsum(lengths)
    codes = rng.integers(0, 20, size=int(offsets[-1]), dtype=np.uint8)
    return codes, offsets


def read_golden_tsv(name: str):
    rows = []
    with open(os.path.join(GOLD, name)) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            prof, idx, L, hx, _ = line.rstrip("\n").split("\t")
            rows.append((prof, int(idx), int(L), np.float32(float.fromhex(hx))))
    return rows


def bits(x) -> np.ndarray:
    return np.asarray(x, np.float32).view(np.uint32)
