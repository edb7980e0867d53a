"""Host sanitizer builds (ASan/UBSan on the host CPU path; TSan for the chunked,
multi-threaded FASTA reader).  `make asan` / `make tsan` in hmm_fasta_viterbi_amd/csrc build the
host-only translation units (parsers, precompute, CPU DP, shard bounds) with plain g++ and run
tests/cpp/test_parsers.cpp and tests/cpp/sanitize_host.cpp under them: the golden scores of all 24
profiles, the golden FASTA edge cases, first-line / EOF cases, truncated .hmm files, a 40 MiB file
through the chunked reader.  Any sanitizer report aborts the run (halt_on_error)."""
import os
import subprocess

import pytest

from oracle_lib import ROOT

CSRC = os.path.join(ROOT, "hmm_fasta_viterbi_amd", "csrc")


@pytest.mark.parametrize("target", ["asan", "tsan"])
def test_host_sanitizer(target):
    p = subprocess.run(["make", "-s", "-C", CSRC, target], capture_output=True, text=True, timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "sanitize_host passed" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out and "WARNING: ThreadSanitizer" not in out
