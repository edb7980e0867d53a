"""the W = 2 team exchange (csrc/vit_team.hip) trusts a record once its stamp word matches, so
each record must reach LDS in ONE store and be polled with ONE load that also carries the stamp -- a record
split over several LDS instructions could be seen half old, half new.  This CPU test compiles vit_team.hip for
gfx950 (the library's own flags) and checks the ISA of every W = 2 team kernel:

  * every poll loop (a backward branch over an LDS read whose readfirstlane'd word is compared with the stamp)
    reads with exactly one ds_read_b128 (the boundary record {M, I, D, stamp}) or ds_read_b64 (the E and
    `next` records {value, stamp}), and the compared word is that load's LAST dword -- the stamp;
  * after the workgroup barrier (the table staging), every LDS store is one ds_write_b128 or ds_write_b64;
  * the boundary and E polls are present (>= 1 ds_read_b128 poll, >= 2 ds_read_b64 polls).

What the hardware must then provide is single-copy atomicity of one lane's aligned 16-byte (boundary) and 8-byte
(E, next) LDS access; only lane 0's copy of the boundary is used (it enters lane 0 of wave 1 as the DPP shift's
`old` operand) and its stamp is the one compared.  Per-half stamps that would need only 8-byte atomicity were
built and measured: 3-9% slower on cfg5's survivors in every form (seven forms) (profiles/r06_ab/README.md), so the 16-byte
record stays, guarded by this check."""
import os
import re
import subprocess

import pytest

from oracle_lib import ROOT

HIPCC = "/opt/rocm/bin/hipcc"
CSRC = os.path.join(ROOT, "hmm_fasta_viterbi_amd", "csrc")


@pytest.fixture(scope="module")
def team_isa(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "vit_team.s"
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-fno-honor-nans", "-fno-slp-vectorize",
             "-ffp-contract=off", f"-I{ROOT}/include", f"-I{CSRC}", "--cuda-device-only", "-S"]
    subprocess.run([HIPCC, *flags, os.path.join(CSRC, "vit_team.hip"), "-o", str(out)], check=True,
                   capture_output=True, timeout=600)
    text = out.read_text()
    kernels = {}
    for name in re.findall(r"^(_ZN4vitk15vit_team_kernelILi2E\S*):", text, re.M):
        i = text.index(name + ":")
        kernels[name] = text[i:text.index(".Lfunc_end", i)].split("\n")
    assert kernels, "no W = 2 team kernel in the ISA"
    return kernels


def _instr(line):
    return line.split(";")[0].strip()


def poll_loops(lines):
    """(LDS reads, readfirstlanes) of every innermost loop that polls an LDS record: a backward branch over an LDS
    read whose word is readfirstlane'd and compared (outer loops that merely contain polls are skipped)."""
    labels = {m.group(1): k for k, l in enumerate(lines) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    ranges = []
    for k, l in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < k:
            ranges.append((labels[m.group(1)], k))
    loops = []
    for a, b in ranges:
        if any((c, d) != (a, b) and a <= c and d <= b for c, d in ranges):
            continue  # not innermost
        body = [_instr(x) for x in lines[a:b + 1]]
        reads = [x for x in body if x.startswith("ds_read")]
        rfl = [x for x in body if x.startswith("v_readfirstlane_b32")]
        if reads and rfl and any(x.startswith(("s_cmp_eq_u32", "s_cmp_lg_u32")) for x in body):
            loops.append((reads, rfl))
    return loops


def test_records_are_polled_with_one_load_that_carries_the_stamp(team_isa):
    for name, lines in team_isa.items():
        loops = poll_loops(lines)
        kinds = {"ds_read_b128": 0, "ds_read_b64": 0}
        for reads, rfl in loops:
            assert len(reads) == 1, (name, reads)
            m = re.match(r"(ds_read_b128|ds_read_b64)\s+v\[(\d+):(\d+)\]", reads[0])
            assert m, (name, reads[0])
            last = int(m.group(3))
            assert any(re.search(rf",\s*v{last}$", r) for r in rfl), (name, reads[0], rfl)
            kinds[m.group(1)] += 1
        assert kinds["ds_read_b128"] >= 1 and kinds["ds_read_b64"] >= 2, (name, kinds)


def test_every_store_after_the_staging_barrier_is_one_record(team_isa):
    for name, lines in team_isa.items():
        b = next(k for k, l in enumerate(lines) if _instr(l).startswith("s_barrier"))
        stores = [_instr(l).split()[0] for l in lines[b:] if _instr(l).startswith("ds_write")]
        assert stores and set(stores) <= {"ds_write_b128", "ds_write_b64"}, (name, sorted(set(stores)))
