"""hmm_fasta_viterbi_amd -- MI355X-native MSV (Multiple Segment Viterbi) scoring engine.

Python mirror of the reference's C++ class surface, bound to libmsv_hip.so (include/msv.h):

    Profile_HMM(path)                       data_readers/Profile_HMM.hpp:21-49
    FASTA_protein_sequences(path)           data_readers/FASTA_protein_sequences.hpp:9-14
    MSV_HMM(profile).run_on_sequence(seq)   algorithms/MSV_HMM.hpp:17-44
                    .parallel_run_on_sequence(seq, should_specialize=False)
                    .score_batch(...)       (new: one fused kernel launch per batch)
    Viterbi_HMM(profile)                    (new, SURVEY 8(f)-4: the Viterbi stage over the parse the
                                             reference never scores with, Profile_HMM.cpp:107-120)
    filter_pipeline(msv, vit, ...)          MSV -> P-value -> F1 -> Viterbi on the survivors, on the GPU

Sequences use the reference's form ('#' sentinel + one-letter residues) or packed codes
0..19 (alphabetical A C D E F G H I K L M N P Q R S T V W Y) with CSR offsets.
Every score is computed by the hand-written gfx950 kernel; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Sequence

import numpy as np

from . import _native
from ._native import MSVError, check

__all__ = [
    "AMINO_ACIDS", "MSVError", "Profile_HMM", "FASTA_protein_sequences", "MSV_HMM", "pack_sequences",
    "encode", "sequence_transitions", "device_count", "score_grid", "score_grid_device", "score_batch_multi",
    "shard_bounds", "FASTA_device", "MultiGPU", "Viterbi_HMM", "filter_pipeline", "INSERTS_ZERO",
    "INSERTS_LOG_ODDS",
]

INSERTS_ZERO = 0      # HMMER3's insert scores (background emissions: 0)
INSERTS_LOG_ODDS = 1  # logf(insert_emissions / background) of the reference's parse

AMINO_ACIDS = "ACDEFGHIKLMNPQRSTVWY"  # MSV_HMM.cpp:29-31
_LUT = np.full(256, 254, np.uint8)
for _i, _c in enumerate(AMINO_ACIDS):
    _LUT[ord(_c)] = _i
_LUT[ord("#")] = 255


def _loaded_lib():
    """The loaded library, or None (also during interpreter shutdown, when module globals such as
    `_native` may already be cleared before the last destructor runs)."""
    native = globals().get("_native")
    return getattr(native, "_lib", None) if native is not None else None


def device_count() -> int:
    n = C.c_int(0)
    _native.lib().msv_device_count(C.byref(n))
    return n.value


class _HostBuffer:
    """Owner of one msv_host_alloc block; freed when the last numpy view of it goes away."""

    def __init__(self, nbytes: int):
        self.ptr = C.c_void_p()
        check(_native.lib().msv_host_alloc(max(int(nbytes), 1), C.byref(self.ptr)), "msv_host_alloc")
        self.nbytes = int(nbytes)

    def __del__(self):
        lib = _loaded_lib()
        if lib is not None and self.ptr:
            lib.msv_host_free(self.ptr)
            self.ptr = C.c_void_p()


def pinned_empty(shape, dtype=np.uint8) -> np.ndarray:
    """A numpy array in page-locked host memory (msv_host_alloc).  score_batch reads residues from such
    an array in place on the GPU (no staging copy) and writes scores into one directly."""
    dt = np.dtype(dtype)
    count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
    owner = _HostBuffer(count * dt.itemsize)
    raw = (C.c_uint8 * max(owner.nbytes, 1)).from_address(owner.ptr.value)
    raw.owner = owner  # every view keeps `raw` (its base), `raw` keeps the allocation
    return np.frombuffer(raw, dtype=dt, count=count).reshape(shape)


def sequence_transitions(L: int) -> tuple[float, float]:
    """(tr_loop, tr_move) of MSV_HMM::init_transitions_depend_on_seq (MSV_HMM.cpp:59-64)."""
    a, b = C.c_float(), C.c_float()
    _native.lib().msv_sequence_transitions(L, C.byref(a), C.byref(b))
    return a.value, b.value


def encode(residues: str) -> np.ndarray:
    """One-letter residues (no '#') -> codes 0..19; IndexError on anything else (the
    reference's amino_acid_num.at throws std::out_of_range, MSV_HMM.cpp:101)."""
    codes = _LUT[np.frombuffer(residues.encode("latin-1"), np.uint8)]
    if codes.size and codes.max() >= 20:
        raise IndexError("residue outside the 20 amino acids")
    return codes


def pack_sequences(seqs: Sequence[str]) -> tuple[np.ndarray, np.ndarray]:
    """'#'-prefixed sequences -> (codes uint8, offsets uint64[n+1])."""
    lens = np.fromiter((max(len(s) - 1, 0) for s in seqs), np.uint64, count=len(seqs))
    offsets = np.zeros(len(seqs) + 1, np.uint64)
    np.cumsum(lens, out=offsets[1:])
    body = "".join(s[1:] for s in seqs)
    return encode(body), offsets


class Profile_HMM:
    """Parsed HMMER3 profile (C++ parser in libmsv_hip.so, Profile_HMM.cpp:48-60 semantics)."""

    def __init__(self, file_path: str):
        L = _native.lib()
        h = C.c_void_p()
        check(L.msv_hmm_read(str(file_path).encode(), C.byref(h)), f"Profile_HMM({file_path})")
        self._h = h
        self.path = str(file_path)
        self.model_length = int(L.msv_hmm_model_length(h))
        self.name = L.msv_hmm_name(h).decode("latin-1")
        st = (C.c_float * 6)()
        L.msv_hmm_stats(h, st)
        (self.stats_local_msv_mu, self.stats_local_msv_lambda, self.stats_local_viterbi_mu,
         self.stats_local_viterbi_lambda, self.stats_local_forward_theta,
         self.stats_local_forward_lambda) = [float(np.float32(x)) for x in st]
        M = self.model_length
        self.match_emissions = np.ctypeslib.as_array(L.msv_hmm_match_emissions(h), (M, 20)).copy()
        self.insert_emissions = np.ctypeslib.as_array(L.msv_hmm_insert_emissions(h), (M, 20)).copy()
        self.transitions = np.ctypeslib.as_array(L.msv_hmm_transitions(h), (M, 7)).copy()

    def msv_scores(self) -> tuple[np.ndarray, float, float, float]:
        """MSV host precompute (MSV_HMM.cpp:35-57): ([20, M] log-odds, tr_B_Mk, tr_E_C, tr_E_J)."""
        es = np.zeros((20, self.model_length), np.float32)
        b, c, j = C.c_float(), C.c_float(), C.c_float()
        check(_native.lib().msv_hmm_msv_scores(self._h, es.ctypes.data_as(C.POINTER(C.c_float)), C.byref(b),
                                                C.byref(c), C.byref(j)))
        return es, b.value, c.value, j.value

    def __del__(self):
        lib = _loaded_lib()
        if getattr(self, "_h", None) and lib is not None:
            lib.msv_hmm_destroy(self._h)
            self._h = None


class FASTA_protein_sequences:
    """FASTA reader (FASTA_protein_sequences.cpp:9-44 semantics), packed straight to codes."""

    def __init__(self, file_path: str):
        L = _native.lib()
        f = C.c_void_p()
        check(L.msv_fasta_read(str(file_path).encode(), C.byref(f)), f"FASTA_protein_sequences({file_path})")
        try:
            n = int(L.msv_fasta_count(f))
            self.offsets = np.ctypeslib.as_array(L.msv_fasta_offsets(f), (n + 1,)).copy()
            total = int(self.offsets[-1])
            self.codes = (np.ctypeslib.as_array(L.msv_fasta_codes(f), (total,)).copy() if total
                          else np.zeros(0, np.uint8))
            self.headers = [L.msv_fasta_header(f, i).decode("latin-1") for i in range(n)]
            self.rejected = int(L.msv_fasta_rejected(f))
        finally:
            L.msv_fasta_destroy(f)
        self._sequences = None

    @property
    def sequences(self) -> list[str]:
        """'#'-prefixed residue strings (FASTA_protein_sequences.cpp:19-20), built on first use; the
        packed `codes`/`offsets` are what the scorer consumes."""
        if self._sequences is None:
            letters = np.frombuffer((AMINO_ACIDS + "#").encode(), np.uint8)
            text = letters[np.minimum(self.codes, 20)].tobytes().decode()
            offs = self.offsets.tolist()
            self._sequences = ["#" + text[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
        return self._sequences

    def __len__(self):
        return len(self.offsets) - 1


class MSV_HMM:
    """MSV scorer for one profile on one GPU (MSV_HMM.hpp:17-44); every score comes from the
    fused gfx950 kernel.  Not thread-safe per instance, like the reference."""

    def __init__(self, base_hmm: Profile_HMM, device: int = 0):
        L = _native.lib()
        self.model_length = base_hmm.model_length
        self.emission_scores, self.tr_B_Mk, self.tr_E_C, self.tr_E_J = base_hmm.msv_scores()
        p = C.c_void_p()
        es = np.ascontiguousarray(self.emission_scores)
        check(L.msv_profile_create(device, es.ctypes.data, self.model_length, self.tr_B_Mk, self.tr_E_C,
                                   self.tr_E_J, C.byref(p)), "msv_profile_create")
        self._p = p
        self._inflight = {}  # msv_score_batch_async tickets -> the arrays the device still reads/writes
        self.device = device
        # STATS LOCAL MSV (Profile_HMM.cpp:83-85): parsed by the reference, used here for P-values
        self.msv_mu = base_hmm.stats_local_msv_mu
        self.msv_lambda = base_hmm.stats_local_msv_lambda

    # -- reference surface ------------------------------------------------------------------
    def run_on_sequence(self, seq: str) -> float:
        return float(self.score_batch([seq])[0])

    def parallel_run_on_sequence(self, seq: str, should_specialize: bool = False) -> float:
        # should_specialize (JIT -D constants, MSV_HMM.cpp:322-337) is always on here: the kernel
        # is a compile-time specialisation on (G, S); both settings return the same score.
        return self.run_on_sequence(seq)

    # -- batch API --------------------------------------------------------------------------
    def score_batch(self, seqs: Sequence[str] | None = None, *, codes: np.ndarray | None = None,
                    offsets: np.ndarray | None = None, out: np.ndarray | None = None) -> np.ndarray:
        """Scores of a host batch (msv_score_batch).  Page-locked `codes` (msv.pinned_empty, torch
        pin_memory().numpy()) are read by the kernel in place, with no staging copy; a page-locked `out`
        (float32[n]) is written by the kernel directly."""
        if seqs is not None:
            codes, offsets = pack_sequences(seqs)
        codes = np.ascontiguousarray(codes, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        if out is None:
            out = np.zeros(n, np.float32)
        elif out.dtype != np.float32 or out.shape != (n,) or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous float32 array of n scores")
        st = _native.lib().msv_score_batch(self._p, codes.ctypes.data if codes.size else None, offsets.ctypes.data,
                                           n, out.ctypes.data, None)
        if st == _native.MSV_ERR_BAD_RESIDUE:
            raise IndexError("residue outside the 20 amino acids")
        check(st, "msv_score_batch")
        return out

    def score_batch_async(self, codes: np.ndarray, offsets: np.ndarray, out: np.ndarray | None = None) -> int:
        """Enqueue a host batch (msv_score_batch_async) and return a ticket; `wait(ticket)` returns
        the scores.  At most three calls outstanding; pinned arrays (torch pin_memory().numpy()) make
        the copies overlap the previous call's kernel.  The arrays are held until the wait."""
        codes = np.ascontiguousarray(codes, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        if out is None:
            out = np.zeros(n, np.float32)
        if out.dtype != np.float32 or out.shape != (n,) or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous float32 array of n scores")
        t = C.c_uint64(0)
        check(_native.lib().msv_score_batch_async(self._p, codes.ctypes.data if codes.size else None,
                                                  offsets.ctypes.data, n, out.ctypes.data, C.byref(t)),
              "msv_score_batch_async")
        self._inflight[t.value] = (codes, offsets, out)
        return t.value

    def wait(self, ticket: int) -> np.ndarray:
        """Scores of an msv_score_batch_async call (raises its kernel-latched errors)."""
        st = _native.lib().msv_profile_wait(self._p, ticket)
        _, _, out = self._inflight.pop(ticket, (None, None, None))
        if st == _native.MSV_ERR_BAD_RESIDUE:
            raise IndexError("residue outside the 20 amino acids")
        check(st, "msv_profile_wait")
        return out

    def score_batch_device(self, residues_ptr: int, residues_len: int, offsets_ptr: int, n: int, scores_ptr: int,
                           order_ptr: int | None = None, stream: int | None = None) -> None:
        """Device-resident batch (raw device pointers, e.g. torch tensor .data_ptr()); async on
        `stream` (a hipStream_t handle, e.g. torch.cuda.current_stream().cuda_stream)."""
        check(_native.lib().msv_score_batch_device(self._p, residues_ptr, residues_len, offsets_ptr, n, order_ptr,
                                                   scores_ptr, stream), "msv_score_batch_device")

    def order_longest_first(self, offsets_ptr: int, n: int, order_ptr: int, stream: int | None = None) -> None:
        check(_native.lib().msv_order_longest_first(self._p, offsets_ptr, n, order_ptr, stream))

    def bind_stream(self, stream: int | None) -> None:
        """Declare `stream` (a hipStream_t handle that outlives the binding) as this profile's working
        stream: its launches skip the per-launch slot event (msv_profile_bind_stream).  None unbinds."""
        check(_native.lib().msv_profile_bind_stream(self._p, stream), "msv_profile_bind_stream")

    def check(self, stream: int | None = None) -> None:
        st = _native.lib().msv_profile_check(self._p, stream)
        if st == _native.MSV_ERR_BAD_RESIDUE:
            raise IndexError("residue outside the 20 amino acids")
        check(st, "msv_profile_check")

    def reserve_length(self, max_length: int) -> None:
        check(_native.lib().msv_profile_reserve_length(self._p, max_length))

    # -- MSV filter stage (HMMER3 formula, parity unpinned) --------------------
    def pvalues(self, scores: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        """P-values of MSV scores against this profile's STATS LOCAL MSV Gumbel (msv.h)."""
        scores = np.ascontiguousarray(scores, np.float32)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        if scores.shape != (n,):
            raise ValueError("scores and offsets disagree")
        out = np.zeros(n, np.float64)
        check(_native.lib().msv_pvalues(scores.ctypes.data, offsets.ctypes.data, n, self.msv_mu, self.msv_lambda,
                                        out.ctypes.data), "msv_pvalues")
        return out

    def pvalues_device(self, scores_ptr: int, offsets_ptr: int, n: int, pvalues_ptr: int,
                       stream: int | None = None) -> None:
        """Device P-values (float64 out) for device scores/offsets, async on `stream`."""
        check(_native.lib().msv_pvalues_device(self.device, scores_ptr, offsets_ptr, n, self.msv_mu, self.msv_lambda,
                                               pvalues_ptr, stream), "msv_pvalues_device")

    def msv_filter(self, seqs: Sequence[str] | None = None, *, codes: np.ndarray | None = None,
                   offsets: np.ndarray | None = None, F1: float = 0.02):
        """Scores, P-values and the pass mask of HMMER3's MSV filter threshold (P <= F1, default
        0.02 as hmmsearch's --F1)."""
        if seqs is not None:
            codes, offsets = pack_sequences(seqs)
        sc = self.score_batch(codes=codes, offsets=offsets)
        pv = self.pvalues(sc, offsets)
        return sc, pv, pv <= F1

    def score_fasta_device(self, fasta: "FASTA_device") -> np.ndarray:
        """Scores of a GPU-parsed FASTA set (msv_score_fasta_device): no host parse, no H2D of residues."""
        out = np.zeros(fasta.count, np.float32)
        st = _native.lib().msv_score_fasta_device(self._p, fasta._f, out.ctypes.data)
        if st == _native.MSV_ERR_BAD_RESIDUE:
            raise IndexError("residue outside the 20 amino acids")
        check(st, "msv_score_fasta_device")
        return out

    def set_variant(self, name: str) -> None:
        check(_native.lib().msv_profile_set_variant(self._p, name.encode()), f"set_variant({name})")

    @staticmethod
    def variants() -> list[str]:
        L = _native.lib()
        return [L.msv_variant_name(i).decode() for i in range(L.msv_variant_count())]

    def describe(self) -> dict:
        info = _native.KernelInfo()
        check(_native.lib().msv_profile_describe(self._p, C.byref(info)))
        return info.as_dict()

    def variant_for(self, n: int) -> str:
        """The kernel variant a batch of n sequences runs (latency / mid / throughput plan)."""
        return _native.lib().msv_profile_variant_for(self._p, n).decode()

    def close(self):
        lib = _loaded_lib()
        if getattr(self, "_p", None) and lib is not None:
            lib.msv_profile_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()


class Viterbi_HMM:
    """Viterbi stage for one profile on one GPU: HMMER3's generic local Viterbi over the
    reference's parse (insert emissions, 7 transitions per node: Profile_HMM.cpp:107-120) with the MSV
    path's specials (MSV_HMM.cpp:49-64); msv.h states the recurrence.  Every score comes from the gfx950
    kernel (vit_kernel.hip) except run_on_sequence, which -- like the reference's MSV run_on_sequence --
    is the library's serial CPU DP.  P-values use STATS LOCAL VITERBI (Profile_HMM.cpp:86-87)."""

    def __init__(self, base_hmm: Profile_HMM, device: int = 0, insert_mode: int = INSERTS_ZERO):
        L = _native.lib()
        M = base_hmm.model_length
        self.model_length = M
        self.insert_mode = insert_mode
        self.match_scores = np.zeros((20, M), np.float32)
        self.insert_scores = np.zeros((20, M), np.float32)
        self.transition_scores = np.zeros((M, 7), np.float32)
        b, c, j = C.c_float(), C.c_float(), C.c_float()
        check(L.msv_hmm_viterbi_scores(base_hmm._h, insert_mode, self.match_scores.ctypes.data,
                                       self.insert_scores.ctypes.data, self.transition_scores.ctypes.data,
                                       C.byref(b), C.byref(c), C.byref(j)), "msv_hmm_viterbi_scores")
        self.tr_B_Mk, self.tr_E_C, self.tr_E_J = b.value, c.value, j.value
        p = C.c_void_p()
        check(L.msv_vit_profile_create(device, self.match_scores.ctypes.data,
                                       self.insert_scores.ctypes.data if insert_mode == INSERTS_LOG_ODDS else None,
                                       self.transition_scores.ctypes.data, M, self.tr_B_Mk, self.tr_E_C, self.tr_E_J,
                                       C.byref(p)), "msv_vit_profile_create")
        self._p = p
        self.device = device
        self.viterbi_mu = base_hmm.stats_local_viterbi_mu
        self.viterbi_lambda = base_hmm.stats_local_viterbi_lambda

    def run_on_sequence(self, seq: str) -> float:
        """The serial CPU Viterbi (msv_vit_cpu_score); IndexError on a residue outside the 20."""
        codes = encode(seq[1:] if seq.startswith("#") else seq)
        out = C.c_float()
        st = _native.lib().msv_vit_cpu_score(
            self.match_scores.ctypes.data, self.insert_scores.ctypes.data if self.insert_mode else None,
            self.transition_scores.ctypes.data, self.model_length, self.tr_B_Mk, self.tr_E_C, self.tr_E_J,
            codes.ctypes.data if codes.size else None, codes.size, C.byref(out))
        check(st, "msv_vit_cpu_score")
        return out.value

    def parallel_run_on_sequence(self, seq: str) -> float:
        return float(self.score_batch([seq])[0])

    def score_batch(self, seqs: Sequence[str] | None = None, *, codes: np.ndarray | None = None,
                    offsets: np.ndarray | None = None) -> np.ndarray:
        """Viterbi scores of every sequence of a host batch (msv_vit_score_batch, one launch)."""
        if seqs is not None:
            codes, offsets = pack_sequences(seqs)
        codes = np.ascontiguousarray(codes, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        out = np.zeros(n, np.float32)
        st = _native.lib().msv_vit_score_batch(self._p, codes.ctypes.data if codes.size else None,
                                               offsets.ctypes.data, n, out.ctypes.data, None)
        if st == _native.MSV_ERR_BAD_RESIDUE:
            raise IndexError("residue outside the 20 amino acids")
        check(st, "msv_vit_score_batch")
        return out

    def score_batch_device(self, residues_ptr: int, residues_len: int, offsets_ptr: int, n: int, scores_ptr: int,
                           select_ptr: int | None = None, select_count_ptr: int | None = None,
                           stream: int | None = None) -> None:
        """Device-resident batch (raw device pointers), optionally only the sequences listed at select_ptr
        (uint32; their count in the device uint32 at select_count_ptr, else n); async on `stream`."""
        check(_native.lib().msv_vit_score_batch_device(self._p, residues_ptr, residues_len, offsets_ptr, n,
                                                       select_ptr, select_count_ptr, scores_ptr, stream),
              "msv_vit_score_batch_device")

    def reserve_length(self, max_length: int) -> None:
        check(_native.lib().msv_vit_profile_reserve_length(self._p, max_length))

    def bind_stream(self, stream: int | None) -> None:
        """msv_vit_profile_bind_stream: launches on this (caller-kept-alive) stream skip the slot event."""
        check(_native.lib().msv_vit_profile_bind_stream(self._p, stream), "msv_vit_profile_bind_stream")

    def check(self, stream: int | None = None) -> None:
        st = _native.lib().msv_vit_profile_check(self._p, stream)
        if st == _native.MSV_ERR_BAD_RESIDUE:
            raise IndexError("residue outside the 20 amino acids")
        check(st, "msv_vit_profile_check")

    def pvalues(self, scores: np.ndarray, offsets: np.ndarray) -> np.ndarray:
        """P-values of Viterbi scores against STATS LOCAL VITERBI (HMMER3's formula, msv_pvalues)."""
        scores = np.ascontiguousarray(scores, np.float32)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        if scores.shape != (n,):
            raise ValueError("scores and offsets disagree")
        out = np.zeros(n, np.float64)
        check(_native.lib().msv_pvalues(scores.ctypes.data, offsets.ctypes.data, n, self.viterbi_mu,
                                        self.viterbi_lambda, out.ctypes.data), "msv_pvalues")
        return out

    def set_variant(self, name: str) -> None:
        check(_native.lib().msv_vit_profile_set_variant(self._p, name.encode()), f"set_variant({name})")

    @staticmethod
    def variants() -> list[str]:
        L = _native.lib()
        return [L.msv_vit_variant_name(i).decode() for i in range(L.msv_vit_variant_count())]

    def describe(self) -> dict:
        info = _native.VitInfo()
        check(_native.lib().msv_vit_profile_describe(self._p, C.byref(info)))
        return info.as_dict()

    def close(self):
        lib = _loaded_lib()
        if getattr(self, "_p", None) and lib is not None:
            lib.msv_vit_profile_destroy(self._p)
            self._p = None

    def __del__(self):
        self.close()


def filter_pipeline(msv_engine: MSV_HMM, vit_engine: Viterbi_HMM, seqs: Sequence[str] | None = None, *,
                    codes: np.ndarray | None = None, offsets: np.ndarray | None = None, F1: float = 0.02):
    """HMMER3's MSV -> Viterbi cascade on the GPU (msv_vit_filter_batch): MSV scores of every sequence,
    the survivors P <= F1 (STATS LOCAL MSV), their Viterbi scores (-inf elsewhere) and Viterbi P-values
    (STATS LOCAL VITERBI, NaN elsewhere).  Returns (msv_scores, passed, vit_scores, vit_pvalues)."""
    if seqs is not None:
        codes, offsets = pack_sequences(seqs)
    codes = np.ascontiguousarray(codes, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    msc = np.zeros(n, np.float32)
    passed = np.zeros(n, np.uint8)
    vsc = np.zeros(n, np.float32)
    npass = C.c_uint64(0)
    st = _native.lib().msv_vit_filter_batch(msv_engine._p, vit_engine._p, codes.ctypes.data if codes.size else None,
                                            offsets.ctypes.data, n, msv_engine.msv_mu, msv_engine.msv_lambda, F1,
                                            msc.ctypes.data, passed.ctypes.data, vsc.ctypes.data, C.byref(npass))
    if st == _native.MSV_ERR_BAD_RESIDUE:
        raise IndexError("residue outside the 20 amino acids")
    check(st, "msv_vit_filter_batch")
    mask = passed.astype(bool)
    vpv = np.full(n, np.nan)
    if mask.any():
        vpv[mask] = vit_engine.pvalues(vsc, offsets)[mask]
    return msc, mask, vsc, vpv


def _handles(engines: Sequence[MSV_HMM]):
    arr = (C.c_void_p * len(engines))(*[e._p for e in engines])
    return arr


def score_grid(engines: Sequence[MSV_HMM], seqs: Sequence[str] | None = None, *, codes: np.ndarray | None = None,
               offsets: np.ndarray | None = None, out: np.ndarray | None = None) -> np.ndarray:
    """Profiles x sequences grid -> float32 [len(engines), n]: the reference's
    benchmark loop over every profile for one FASTA set (benchmark_MSV.cpp:12-24,31-41), as one
    host call: one upload, one longest-first order, then ONE fused launch over all profiles for a
    few sequences, else one launch per profile forked onto the profiles' own streams.  `out`: an
    optional C-contiguous float32 [len(engines), n] destination (page-locked, e.g. pinned_empty,
    is written by the kernels directly); page-locked `codes` are read in place."""
    if not engines:
        raise ValueError("score_grid needs at least one profile")
    if seqs is not None:
        codes, offsets = pack_sequences(seqs)
    codes = np.ascontiguousarray(codes, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    if out is None:
        out = np.zeros((len(engines), n), np.float32)
    elif out.dtype != np.float32 or out.shape != (len(engines), n) or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous float32 array of shape (len(engines), n)")
    st = _native.lib().msv_score_grid(_handles(engines), len(engines), codes.ctypes.data if codes.size else None,
                                      offsets.ctypes.data, n, out.ctypes.data, None)
    if st == _native.MSV_ERR_BAD_RESIDUE:
        raise IndexError("residue outside the 20 amino acids")
    check(st, "msv_score_grid")
    return out


def score_grid_device(engines: Sequence[MSV_HMM], residues_ptr: int, residues_len: int, offsets_ptr: int, n: int,
                      scores_ptr: int, order_ptr: int | None = None, stream: int | None = None) -> None:
    """Device-resident grid: scores_ptr -> float32 [len(engines)][n]; async on `stream`; errors via
    each engine's check()."""
    check(_native.lib().msv_score_grid_device(_handles(engines), len(engines), residues_ptr, residues_len,
                                              offsets_ptr, n, order_ptr, scores_ptr, stream), "msv_score_grid_device")


def shard_bounds(offsets: np.ndarray, n_shards: int) -> np.ndarray:
    """uint64[n_shards + 1] contiguous, residue-balanced shard boundaries (msv_shard_bounds)."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    out = np.zeros(n_shards + 1, np.uint64)
    check(_native.lib().msv_shard_bounds(offsets.ctypes.data, len(offsets) - 1, n_shards, out.ctypes.data),
          "msv_shard_bounds")
    return out


def score_batch_multi(engines: Sequence[MSV_HMM], seqs: Sequence[str] | None = None, *,
                      codes: np.ndarray | None = None, offsets: np.ndarray | None = None) -> np.ndarray:
    """One batch over several devices from this one process (engines[k] = the profile on device k):
    residue-balanced contiguous shards scored concurrently, scores in input order."""
    if not engines:
        raise ValueError("score_batch_multi needs at least one engine")
    if seqs is not None:
        codes, offsets = pack_sequences(seqs)
    codes = np.ascontiguousarray(codes, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    out = np.zeros(n, np.float32)
    st = _native.lib().msv_score_batch_multi(_handles(engines), len(engines), codes.ctypes.data if codes.size else None,
                                             offsets.ctypes.data, n, out.ctypes.data)
    if st == _native.MSV_ERR_BAD_RESIDUE:
        raise IndexError("residue outside the 20 amino acids")
    check(st, "msv_score_batch_multi")
    return out


class MultiGPU:
    """One batch over several GPUs from this process, scores gathered over RCCL (msv_multi_*):
    engines[k] = the same model on DISTINCT devices; residue-balanced shards, one grouped RCCL
    send/recv into device 0, one D2H."""

    def __init__(self, engines: Sequence[MSV_HMM]):
        if not engines:
            raise ValueError("MultiGPU needs at least one engine")
        self._engines = list(engines)  # the context refers to their profiles
        m = C.c_void_p()
        check(_native.lib().msv_multi_create(_handles(self._engines), len(self._engines), C.byref(m)),
              "msv_multi_create")
        self._m = m

    def score_batch(self, seqs: Sequence[str] | None = None, *, codes: np.ndarray | None = None,
                    offsets: np.ndarray | None = None) -> np.ndarray:
        if seqs is not None:
            codes, offsets = pack_sequences(seqs)
        codes = np.ascontiguousarray(codes, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        out = np.zeros(n, np.float32)
        st = _native.lib().msv_multi_score_batch(self._m, codes.ctypes.data if codes.size else None,
                                                 offsets.ctypes.data, n, out.ctypes.data)
        if st == _native.MSV_ERR_BAD_RESIDUE:
            raise IndexError("residue outside the 20 amino acids")
        check(st, "msv_multi_score_batch")
        return out

    def close(self):
        lib = _loaded_lib()
        if getattr(self, "_m", None) and lib is not None:
            lib.msv_multi_destroy(self._m)
            self._m = None

    def __del__(self):
        self.close()


class FASTA_device:
    """FASTA parsed on the GPU (msv_fasta_read_device / msv_fasta_parse_device): the
    same records as FASTA_protein_sequences, left in device memory as the scorer's CSR input.
    `codes_ptr`/`offsets_ptr` feed MSV_HMM.score_batch_device directly."""

    def __init__(self, path: str | None = None, *, text_ptr: int | None = None, n: int = 0, device: int = 0,
                 stream: int | None = None):
        L = _native.lib()
        f = C.c_void_p()
        if path is not None:
            check(L.msv_fasta_read_device(device, str(path).encode(), stream, C.byref(f)), f"FASTA_device({path})")
        else:
            check(L.msv_fasta_parse_device(device, text_ptr, n, stream, C.byref(f)), "msv_fasta_parse_device")
        self._f = f
        self.device = device
        self.count = int(L.msv_fasta_device_count(f))
        self.rejected = int(L.msv_fasta_device_rejected(f))
        self.residues = int(L.msv_fasta_device_residues(f))
        self.max_length = int(L.msv_fasta_device_max_length(f))
        self.codes_ptr = L.msv_fasta_device_codes(f)
        self.offsets_ptr = L.msv_fasta_device_offsets(f)
        self.spans_ptr = L.msv_fasta_device_header_spans(f)

    def download(self):
        """(codes uint8, offsets uint64[count+1], spans uint64[count, 2]) on the host."""
        codes = np.zeros(self.residues, np.uint8)
        offsets = np.zeros(self.count + 1, np.uint64)
        spans = np.zeros((self.count, 2), np.uint64)
        check(_native.lib().msv_fasta_device_download(self._f, codes.ctypes.data if self.residues else None,
                                                      offsets.ctypes.data, spans.ctypes.data if self.count else None),
              "msv_fasta_device_download")
        return codes, offsets, spans

    def close(self):
        lib = _loaded_lib()
        if getattr(self, "_f", None) and lib is not None:
            lib.msv_fasta_device_destroy(self._f)
            self._f = None

    def __del__(self):
        self.close()

    def __len__(self):
        return self.count
