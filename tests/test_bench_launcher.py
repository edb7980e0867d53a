"""bench.py's rank launcher (CPU): `python bench.py --gpus N` started without torch.distributed.run
runs N ranks as a child process tree; under a launcher, WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

import pytest

from oracle_lib import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launcher_command_plumbing():
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "5", "--config", "cfg4"], 8, 29999)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29999" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5", "--config", "cfg4"]


def test_check_world():
    assert bench.check_world(1, {}) == "run"
    assert bench.check_world(4, {}) == "launch"
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) == "run"
    with pytest.raises(SystemExit):
        bench.check_world(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.check_world(1, {"WORLD_SIZE": "2"})


def test_gpus_2_spawns_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--config", "cfg4"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks"] == 2 and lines[0]["config"] == "cfg4"


def test_world_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in p.stderr


def test_kernel_symbols():
    from hmm_fasta_viterbi_amd.kernel_names import kernel_symbol
    assert kernel_symbol("msv_g16_s88_w16_p2_d1") == "msv_batch_kernel<16, 88, 16, 2, false, 1, 0, 0>"
    assert kernel_symbol("msv_g16_s88_w16_p2_d1", zero_copy=True).endswith(", 2>")
    # zero-copy twins mirror msv_kernel_impl.h zc_fn: wide blocks for <= 40-state rows, none for 4/8 lanes,
    # whole-row rings (PF > 2), split or BIG variants
    assert kernel_symbol("msv_g16_s8_w4_p2_d1", zero_copy=True).endswith(", 0, 64>")
    assert kernel_symbol("msv_g64_s8_w16_p2_d1", zero_copy=True).endswith(", 0, 64>")
    assert kernel_symbol("msv_g64_s34_w16_p2_d1", zero_copy=True).endswith(", true, 1, 0, 0>")  # BIG
    assert kernel_symbol("msv_g4_s28_w16_p2_d1", zero_copy=True).endswith(", 0, 0>")
    assert kernel_symbol("msv_g16_s28_w16_p7_d1", zero_copy=True).endswith(", 0, 0>")
    assert kernel_symbol("msv_g32_s76_a64_w16_p2_d1", zero_copy=True).endswith(", 64, 0>")
    assert kernel_symbol("msv_g64_s48_w16_p2_d1", zero_copy=True).endswith(", 0, 0>")
    assert kernel_symbol("msv_g32_s76_a64_w16_p2_d1") == "msv_batch_kernel<32, 76, 16, 2, false, 1, 64, 0>"
    assert kernel_symbol("msv_g64_s48_w16_p2_d1") == "msv_batch_kernel<64, 48, 16, 2, true, 1, 0, 0>"
    assert kernel_symbol("msv_coop_w4_s6") == "msv_coop_kernel<4, 6, 6>"
    assert kernel_symbol("msv_coop_w4_s10_a6") == "msv_coop_kernel<4, 10, 6>"
    with pytest.raises(ValueError):
        kernel_symbol("not_a_variant")


def test_per_rank_summary():
    """The N-rank line's per-rank block (bench.py per_rank_summary): each rank's step and kernel time, residues,
    and the max-over-min imbalance of each."""
    import numpy as np
    from bench import per_rank_summary
    allr = np.array([[0.060, 2.80, 40_000_000, 100_000], [0.063, 2.95, 41_000_000, 100_000]])
    d = per_rank_summary(allr, 20, "strong")
    assert d["ms_per_step"] == [3.0, 3.15] and d["kernel_ms"] == [2.8, 2.95]
    assert d["residues"] == [40_000_000, 41_000_000] and d["sequences"] == [100_000, 100_000]
    assert d["imbalance"]["residues"]["max_over_min"] == round(41 / 40, 4)
    assert d["imbalance"]["kernel_ms"]["max"] == 2.95 and d["step_minus_kernel_ms"] == [0.2, 0.2]
    assert "all-gather" in d["note"]

