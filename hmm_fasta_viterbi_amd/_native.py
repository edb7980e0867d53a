"""ctypes binding of the C-ABI in include/msv.h (libmsv_hip.so, built in-tree).

There is no fallback: if the shared library is missing the import of the device path fails
loudly with a message saying how to build it.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# MSV_LIB_PATH: another build of the same library (tools/ab.py compares two builds in one process
# run); unset in every test and product run.
LIB_PATH = os.environ.get("MSV_LIB_PATH") or os.path.join(LIB_DIR, "libmsv_hip.so")

STATUS = {
    0: "MSV_OK",
    1: "MSV_ERR_INVALID_ARGUMENT",
    2: "MSV_ERR_IO",
    3: "MSV_ERR_PARSE",
    4: "MSV_ERR_BAD_RESIDUE",
    5: "MSV_ERR_SEQUENCE_TOO_LONG",
    6: "MSV_ERR_UNSUPPORTED_MODEL",
    7: "MSV_ERR_NO_DEVICE",
    8: "MSV_ERR_HIP",
    9: "MSV_ERR_OUT_OF_MEMORY",
    10: "MSV_ERR_RCCL",
}
MSV_OK = 0
MSV_ERR_BAD_RESIDUE = 4

# Every symbol include/msv.h declares (checked by tests/test_capi.py).
EXPORTED = [
    "msv_status_string", "msv_version", "msv_device_count",
    "msv_hmm_read", "msv_hmm_destroy", "msv_hmm_model_length", "msv_hmm_name", "msv_hmm_stats",
    "msv_hmm_match_emissions", "msv_hmm_insert_emissions", "msv_hmm_transitions", "msv_hmm_msv_scores",
    "msv_sequence_transitions",
    "msv_fasta_read", "msv_fasta_destroy", "msv_fasta_count", "msv_fasta_rejected", "msv_fasta_codes",
    "msv_fasta_offsets", "msv_fasta_header", "msv_encode_residues",
    "msv_profile_create", "msv_profile_create_from_hmm", "msv_profile_destroy", "msv_profile_describe",
    "msv_profile_reserve_length", "msv_score_batch", "msv_score_batch_device", "msv_profile_check",
    "msv_order_longest_first", "msv_variant_count", "msv_variant_name", "msv_profile_set_variant",
    "msv_score_grid", "msv_score_grid_device", "msv_pvalues", "msv_pvalues_device",
    "msv_shard_bounds", "msv_score_batch_multi",
    "msv_fasta_parse_device", "msv_fasta_read_device", "msv_fasta_device_destroy", "msv_fasta_device_count",
    "msv_fasta_device_rejected", "msv_fasta_device_residues", "msv_fasta_device_codes", "msv_fasta_device_offsets",
    "msv_fasta_device_header_spans", "msv_fasta_device_text", "msv_fasta_device_download",
    "msv_fasta_device_max_length", "msv_score_fasta_device", "msv_fasta_device_device",
    "msv_score_batch_async", "msv_profile_wait", "msv_profile_bind_stream",
    "msv_multi_create", "msv_multi_score_batch", "msv_multi_destroy",
    "msv_host_alloc", "msv_host_free", "msv_profile_variant_for",
    "msv_filter_select_device", "msv_hmm_viterbi_scores", "msv_vit_cpu_score", "msv_vit_profile_create",
    "msv_vit_profile_create_from_hmm", "msv_vit_profile_destroy", "msv_vit_profile_reserve_length",
    "msv_vit_profile_describe", "msv_vit_variant_count", "msv_vit_variant_name", "msv_vit_profile_set_variant",
    "msv_vit_score_batch_device", "msv_vit_score_batch", "msv_vit_profile_check", "msv_vit_filter_batch",
    "msv_vit_profile_bind_stream",
]


class MSVError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        self.name = STATUS.get(status, f"MSV_ERR_{status}")
        super().__init__(f"{what}: {self.name}" if what else self.name)


class KernelInfo(C.Structure):
    _fields_ = [
        ("model_length", C.c_uint32),
        ("lanes_per_group", C.c_uint32),
        ("states_per_lane", C.c_uint32),
        ("waves_per_block", C.c_uint32),
        ("lds_rows", C.c_uint32),
        ("lds_bytes", C.c_uint32),
        ("blocks", C.c_uint32),
        ("max_length", C.c_uint32),
        ("device", C.c_int),
        ("variant", C.c_char * 64),
        ("latency_variant", C.c_char * 64),
        ("latency_blocks", C.c_uint32),
        ("latency_max_n", C.c_uint64),
        ("mid_variant", C.c_char * 64),
        ("mid_blocks", C.c_uint32),
        ("mid_max_n", C.c_uint64),
        ("coop_variant", C.c_char * 64),
        ("coop_blocks", C.c_uint32),
        ("coop_max_n", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["variant"] = self.variant.decode()
        d["latency_variant"] = self.latency_variant.decode()
        d["mid_variant"] = self.mid_variant.decode()
        d["coop_variant"] = self.coop_variant.decode()
        return d


class VitInfo(C.Structure):
    _fields_ = [
        ("model_length", C.c_uint32),
        ("states_per_lane", C.c_uint32),
        ("transitions_in_registers", C.c_uint32),
        ("match_in_lds", C.c_uint32),
        ("insert_scores", C.c_uint32),
        ("waves_per_block", C.c_uint32),
        ("blocks", C.c_uint32),
        ("lds_bytes", C.c_uint32),
        ("max_length", C.c_uint32),
        ("device", C.c_int),
        ("variant", C.c_char * 64),
        ("scratch_bytes", C.c_uint32),
        ("waves_per_sequence", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["variant"] = self.variant.decode()
        return d


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: the MSV HIP library is not built. "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C hmm_fasta_viterbi_amd/csrc`.")
    # One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7, the
    # same soname /opt/rocm's has).  Loading torch first makes our DT_NEEDED bind to torch's copy,
    # so streams, events and device pointers from torch are valid handles for this library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, sz, u64, u32, f32 = C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint32, C.c_float
    fp = C.POINTER(C.c_float)
    sig = {
        "msv_status_string": (C.c_char_p, [C.c_int]),
        "msv_version": (C.c_char_p, []),
        "msv_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "msv_hmm_read": (C.c_int, [C.c_char_p, C.POINTER(vp)]),
        "msv_hmm_destroy": (None, [vp]),
        "msv_hmm_model_length": (sz, [vp]),
        "msv_hmm_name": (C.c_char_p, [vp]),
        "msv_hmm_stats": (None, [vp, fp]),
        "msv_hmm_match_emissions": (fp, [vp]),
        "msv_hmm_insert_emissions": (fp, [vp]),
        "msv_hmm_transitions": (fp, [vp]),
        "msv_hmm_msv_scores": (C.c_int, [vp, fp, fp, fp, fp]),
        "msv_sequence_transitions": (None, [u64, fp, fp]),
        "msv_fasta_read": (C.c_int, [C.c_char_p, C.POINTER(vp)]),
        "msv_fasta_destroy": (None, [vp]),
        "msv_fasta_count": (sz, [vp]),
        "msv_fasta_rejected": (sz, [vp]),
        "msv_fasta_codes": (C.POINTER(C.c_uint8), [vp]),
        "msv_fasta_offsets": (C.POINTER(C.c_uint64), [vp]),
        "msv_fasta_header": (C.c_char_p, [vp, sz]),
        "msv_encode_residues": (C.c_int, [C.c_char_p, sz, vp]),
        "msv_profile_create": (C.c_int, [C.c_int, vp, u32, f32, f32, f32, C.POINTER(vp)]),
        "msv_profile_create_from_hmm": (C.c_int, [C.c_int, vp, C.POINTER(vp)]),
        "msv_profile_destroy": (None, [vp]),
        "msv_profile_describe": (C.c_int, [vp, C.POINTER(KernelInfo)]),
        "msv_profile_variant_for": (C.c_char_p, [vp, C.c_uint64]),
        "msv_profile_reserve_length": (C.c_int, [vp, u64]),
        "msv_score_batch": (C.c_int, [vp, vp, vp, u64, vp, vp]),
        "msv_host_alloc": (C.c_int, [sz, C.POINTER(vp)]),
        "msv_host_free": (C.c_int, [vp]),
        "msv_score_batch_device": (C.c_int, [vp, vp, u64, vp, u64, vp, vp, vp]),
        "msv_score_batch_async": (C.c_int, [vp, vp, vp, u64, vp, C.POINTER(C.c_uint64)]),
        "msv_profile_wait": (C.c_int, [vp, u64]),
        "msv_profile_bind_stream": (C.c_int, [vp, vp]),
        "msv_multi_create": (C.c_int, [vp, C.c_uint32, C.POINTER(vp)]),
        "msv_multi_score_batch": (C.c_int, [vp, vp, vp, u64, vp]),
        "msv_multi_destroy": (None, [vp]),
        "msv_profile_check": (C.c_int, [vp, vp]),
        "msv_order_longest_first": (C.c_int, [vp, vp, u64, vp, vp]),
        "msv_variant_count": (C.c_int, []),
        "msv_variant_name": (C.c_char_p, [C.c_int]),
        "msv_profile_set_variant": (C.c_int, [vp, C.c_char_p]),
        "msv_score_grid": (C.c_int, [vp, C.c_uint32, vp, vp, u64, vp, vp]),
        "msv_score_grid_device": (C.c_int, [vp, C.c_uint32, vp, u64, vp, u64, vp, vp, vp]),
        "msv_pvalues": (C.c_int, [vp, vp, u64, C.c_float, C.c_float, vp]),
        "msv_shard_bounds": (C.c_int, [vp, u64, C.c_uint32, vp]),
        "msv_fasta_parse_device": (C.c_int, [C.c_int, vp, u64, vp, vp]),
        "msv_fasta_read_device": (C.c_int, [C.c_int, C.c_char_p, vp, vp]),
        "msv_fasta_device_destroy": (None, [vp]),
        "msv_fasta_device_count": (u64, [vp]),
        "msv_fasta_device_device": (C.c_int, [vp]),
        "msv_fasta_device_rejected": (u64, [vp]),
        "msv_fasta_device_residues": (u64, [vp]),
        "msv_fasta_device_codes": (vp, [vp]),
        "msv_fasta_device_offsets": (vp, [vp]),
        "msv_fasta_device_header_spans": (vp, [vp]),
        "msv_fasta_device_text": (vp, [vp]),
        "msv_fasta_device_download": (C.c_int, [vp, vp, vp, vp]),
        "msv_fasta_device_max_length": (u64, [vp]),
        "msv_score_fasta_device": (C.c_int, [vp, vp, vp]),
        "msv_score_batch_multi": (C.c_int, [vp, C.c_uint32, vp, vp, u64, vp]),
        "msv_pvalues_device": (C.c_int, [C.c_int, vp, vp, u64, C.c_float, C.c_float, vp, vp]),
        "msv_filter_select_device": (C.c_int, [C.c_int, vp, vp, vp, u64, f32, f32, C.c_double, vp, vp, vp, vp]),
        "msv_hmm_viterbi_scores": (C.c_int, [vp, C.c_int, vp, vp, vp, fp, fp, fp]),
        "msv_vit_cpu_score": (C.c_int, [vp, vp, vp, u32, f32, f32, f32, vp, u64, fp]),
        "msv_vit_profile_create": (C.c_int, [C.c_int, vp, vp, vp, u32, f32, f32, f32, C.POINTER(vp)]),
        "msv_vit_profile_create_from_hmm": (C.c_int, [C.c_int, vp, C.c_int, C.POINTER(vp)]),
        "msv_vit_profile_destroy": (None, [vp]),
        "msv_vit_profile_reserve_length": (C.c_int, [vp, u64]),
        "msv_vit_profile_describe": (C.c_int, [vp, C.POINTER(VitInfo)]),
        "msv_vit_variant_count": (C.c_int, []),
        "msv_vit_variant_name": (C.c_char_p, [C.c_int]),
        "msv_vit_profile_set_variant": (C.c_int, [vp, C.c_char_p]),
        "msv_vit_score_batch_device": (C.c_int, [vp, vp, u64, vp, u64, vp, vp, vp, vp]),
        "msv_vit_profile_bind_stream": (C.c_int, [vp, vp]),
        "msv_vit_score_batch": (C.c_int, [vp, vp, vp, u64, vp, vp]),
        "msv_vit_profile_check": (C.c_int, [vp, vp]),
        "msv_vit_filter_batch": (C.c_int, [vp, vp, vp, vp, u64, f32, f32, C.c_double, vp, vp, vp,
                                           C.POINTER(C.c_uint64)]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("MSV_LIB_PATH") and not hasattr(L, name):
            continue  # an older build under A/B timing may predate an entry point
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int, what: str = "") -> None:
    if status != MSV_OK:
        raise MSVError(status, what)
