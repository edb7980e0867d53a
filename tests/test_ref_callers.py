"""The drop-in proof of SURVEY 8(b): the reference's OWN callers of the MSV path, compiled unchanged against this
library (tests/ref_callers/Makefile: the sources read where they lie under /root/reference, the forwarding headers
include/drop_in/{MSV_HMM,Profile_HMM,FASTA_protein_sequences}.hpp, libmsv_hip.so), run the way the reference runs
them: from a build/<subdir> working directory with ../profile_HMMs and ../FASTA_files beside it
(compile_clang_in_build_dir.sh:4-7).

  test_hmm_parsing, test_fasta_parsing   CPU: rc 0 with their asserts live  (test_hmm_parsing.cpp:19-36,
                                         test_fasta_parsing.cpp:5-14)
  test_MSV                               GPU: rc 0 over all 24 profiles -- run_on_sequence (this library's CPU DP)
                                         vs parallel_run_on_sequence(seq) and (seq, true) (the gfx950 kernel),
                                         1e-4 as the reference asserts (test_MSV.cpp:9-31)
  benchmark_MSV, benchmark_MSV_1400      GPU: rc 0, every "best time" line printed (benchmark_helper.hpp:40-41)

The binaries are built in the build container (build() or `make -C tests/ref_callers`, which needs
/root/reference) and travel to the GPU box with the tree; the recipe fails the build if any reference header
other than benchmark_helper.hpp was compiled in, and the dependency lists it writes are checked again here."""
import os
import re
import subprocess
import time

import pytest

from oracle_lib import ROOT

BIN = os.path.join(ROOT, "build", "ref_callers")
REF = "/root/reference"
PROFILES = sorted(f for f in os.listdir(os.path.join(ROOT, "data", "profile_HMMs")) if f.endswith(".hmm"))


def binary(name):
    if os.path.isdir(os.path.join(REF, "algorithms")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "ref_callers")], check=True)
    path = os.path.join(BIN, name)
    assert os.path.exists(path), f"{path} missing: build it with `make -C tests/ref_callers` where /root/reference exists"
    return path


def run_from_build_dir(tmp_path, subdir, name, timeout):
    """Run `name` with cwd build/<subdir>, ../profile_HMMs and ../FASTA_files -> data/ (the reference's layout)."""
    exe = binary(name)
    for d in ("profile_HMMs", "FASTA_files"):
        os.symlink(os.path.join(ROOT, "data", d), tmp_path / d)
    (tmp_path / subdir).mkdir()
    t0 = time.perf_counter()
    p = subprocess.run([exe], cwd=tmp_path / subdir, capture_output=True, text=True, timeout=timeout)
    return p, time.perf_counter() - t0


@pytest.mark.parametrize("name", ["test_MSV", "benchmark_MSV", "benchmark_MSV_1400", "test_hmm_parsing",
                                  "test_fasta_parsing"])
def test_only_the_library_headers_were_compiled_in(name):
    binary(name)
    deps = open(os.path.join(BIN, name + ".d")).read().replace("\\\n", " ").split()[1:]
    ref_headers = [d for d in deps if d.startswith(REF) and d.endswith(".hpp")]
    assert all(d.endswith("/benchmark_helper.hpp") for d in ref_headers), ref_headers
    for h in ("MSV_HMM.hpp", "Profile_HMM.hpp", "FASTA_protein_sequences.hpp"):
        if any(d.endswith("/" + h) for d in deps):
            assert os.path.join(ROOT, "include", "drop_in", h) in deps
    assert os.path.join(ROOT, "include", "msv_hmm.hpp") in deps


@pytest.mark.parametrize("name", ["test_hmm_parsing", "test_fasta_parsing"])
def test_reference_parser_tests_pass_against_the_library(tmp_path, name):
    syms = subprocess.run(["nm", "-D", "--undefined-only", binary(name)], capture_output=True, text=True,
                          check=True).stdout
    assert "__assert_fail" in syms, "asserts compiled out: the test would prove nothing"
    assert re.search(r"\bProfile_HMM|FASTA_protein_sequences", subprocess.run(
        ["nm", "-DC", "--undefined-only", binary(name)], capture_output=True, text=True, check=True).stdout)
    p, _ = run_from_build_dir(tmp_path, "data_readers", name, 60)
    assert p.returncode == 0, (p.returncode, p.stdout, p.stderr)


def test_msv_callers_reach_the_device_path(tmp_path):
    """Without a GPU (this container) test_MSV must fail loudly in MSV_HMM's device set-up -- it scores through
    the library's kernel, never a CPU fallback."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the gpu tests below run the binary for real")
    p, _ = run_from_build_dir(tmp_path, "algorithms", "test_MSV", 60)
    assert p.returncode != 0
    assert "msv_error" in p.stderr or "terminate" in p.stderr, p.stderr


@pytest.mark.gpu
def test_reference_test_MSV_passes_on_every_profile(tmp_path):
    p, secs = run_from_build_dir(tmp_path, "algorithms", "test_MSV", 110)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    assert "failed" not in p.stdout
    print(f"test_MSV: rc 0 over {len(PROFILES)} profiles x 4 sequences x (seq, par, par_spec) in {secs:.2f} s")


@pytest.mark.gpu
@pytest.mark.parametrize("name,n_lines", [("benchmark_MSV_1400", 2), ("benchmark_MSV", 2 * len(PROFILES))])
def test_reference_benchmarks_run(tmp_path, name, n_lines):
    p, secs = run_from_build_dir(tmp_path, "algorithms", name, 110)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    best = re.findall(r"^(.*): best time is (\d+) msec from (\d+) times", p.stdout, flags=re.M)
    assert len(best) == n_lines, p.stdout
    out = os.environ.get("REF_CALLERS_OUT")
    if out:
        with open(os.path.join(out, name + ".txt"), "w") as f:
            f.write(f"# {name}, cwd build/algorithms, wall {secs:.3f} s (process, incl. parse + profile uploads)\n")
            f.write(p.stdout)
    print(f"{name}: {len(best)} best-time lines, wall {secs:.2f} s")


def test_integration_cmake_swap_builds_the_reference_tree(tmp_path):
    """INTEGRATION.md §2 applied literally to a scratch copy of the reference tree (tests/ref_callers/cmake_swap.sh:
    the reference's class sources deleted, its two library CMakeLists.txt replaced by INTERFACE targets on
    include/drop_in + include + libmsv_hip.so): the reference's own CMake build (-Wall -Wextra -pedantic -Werror,
    Debug) makes all six executables and its ctest parser tests pass.  The copy lives in pytest's tmp dir only."""
    import shutil
    if not os.path.isdir(os.path.join(REF, "algorithms")) or not shutil.which("cmake"):
        pytest.skip("needs /root/reference and cmake (the build container)")
    p = subprocess.run(["bash", os.path.join(ROOT, "tests", "ref_callers", "cmake_swap.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])
    assert "100% tests passed" in p.stdout
    built = (tmp_path / "make.log").read_text()
    for target in ("test_MSV", "benchmark_MSV", "benchmark_MSV_1400", "test_hmm_parsing", "test_fasta_parsing",
                   "HMM_FASTA_Viterbi"):
        assert f"Built target {target}" in built, target
