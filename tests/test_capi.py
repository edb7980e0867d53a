"""The C-ABI library loads and exports every entry point include/msv.h declares; host-only calls
behave; device calls fail with a status (never a crash) when no GPU is visible.  CPU only."""
import ctypes as C
import os
import re
import subprocess

import pytest

from hmm_fasta_viterbi_amd import _native
from oracle_lib import ROOT


def declared_functions():
    text = open(os.path.join(ROOT, "include", "msv.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(msv_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_bound_symbols():
    assert declared_functions() == sorted(_native.EXPORTED)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (msv_[a-z0-9_]+)$", out, flags=re.M))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    L = _native.lib()
    for f in declared_functions():
        assert getattr(L, f) is not None


def test_status_strings_and_version():
    L = _native.lib()
    for code, name in _native.STATUS.items():
        assert L.msv_status_string(code).decode() == name
    assert b"gfx950" in L.msv_version()


def test_kernel_family_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", "-h", _native.LIB_PATH],
                         capture_output=True, text=True)
    blob = out.stdout + out.stderr
    assert "gfx950" in blob or "hipv4-amdgcn-amd-amdhsa--gfx950" in open(_native.LIB_PATH, "rb").read().decode(
        "latin-1")


def test_invalid_arguments_return_status():
    L = _native.lib()
    p = C.c_void_p()
    assert L.msv_profile_create(0, None, 101, 0.0, 0.0, 0.0, C.byref(p)) == 1
    assert L.msv_score_batch(None, None, None, 0, None, None) == 1
    assert L.msv_hmm_read(None, C.byref(p)) == 1


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd"),
                    reason="a GPU may be present")
def test_no_device_is_a_status_not_a_crash():
    L = _native.lib()
    n = C.c_int(-1)
    L.msv_device_count(C.byref(n))
    if n.value == 0:
        import numpy as np
        es = np.zeros(20 * 101, np.float32)
        p = C.c_void_p()
        assert L.msv_profile_create(0, es.ctypes.data, 101, -8.5, -0.69, -0.69, C.byref(p)) == 7
