"""World-size-2 gloo run of the multi-GPU sharding path on CPU (the GPU scorer replaced by the
oracle restatement): shards are contiguous, residue-balanced, cover the batch exactly once, and
the gathered scores equal the single-process result bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from hmm_fasta_viterbi_amd.distributed import shard, shard_bounds
from hmm_fasta_viterbi_amd.synthetic import random_batch
from oracle_lib import ROOT


def test_shard_bounds_cover_and_balance():
    codes, offsets = random_batch(3, 10_000, 1, 2000)
    for world in (1, 2, 3, 8):
        b = [shard_bounds(offsets, world, r) for r in range(world)]
        assert b[0][0] == 0 and b[-1][1] == 10_000
        assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
        res = [int(offsets[hi] - offsets[lo]) for lo, hi in b]
        assert max(res) - min(res) <= 2 * 2000 + 1
    # degenerate: more ranks than sequences, empty sequences
    _, offs = random_batch(4, 3, 0, 0)
    b = [shard_bounds(offs, 8, r) for r in range(8)]
    assert sum(hi - lo for lo, hi in b) == 3


def test_shard_rebases_offsets():
    codes, offsets = random_batch(5, 100, 1, 50)
    c, o, first, last = shard(codes, offsets, 4, 2)
    assert o[0] == 0 and len(c) == int(o[-1])
    assert np.array_equal(c, codes[int(offsets[first]):int(offsets[last])])


WORKER = r'''
import os, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, "tests"))
import numpy as np, torch.distributed as dist
from hmm_fasta_viterbi_amd.distributed import score_sharded
from hmm_fasta_viterbi_amd.synthetic import random_batch
from oracle_lib import OracleProfile
dist.init_process_group("gloo")
prof = OracleProfile("100")
codes, offsets = random_batch(11, 300, 0, 400)
got = score_sharded(prof.score_batch, codes, offsets)
if dist.get_rank() == 0:
    want = prof.score_batch(codes, offsets)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    print("MULTIRANK_OK")
dist.destroy_process_group()
'''


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world_size_2(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "MULTIRANK_OK" in outs[0]


GPU_WORKER = r'''
import os, sys
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, "tests"))
import numpy as np, torch.distributed as dist
import hmm_fasta_viterbi_amd as msv
from hmm_fasta_viterbi_amd.distributed import score_sharded
from hmm_fasta_viterbi_amd.synthetic import random_batch
from oracle_lib import OracleProfile, profile_path
dist.init_process_group("gloo")
engine = msv.MSV_HMM(msv.Profile_HMM(profile_path("1400")), device=0)
codes, offsets = random_batch(3, 40_000, 300, 500)  # the cfg4 shape (seed 3), 40k of its 1M
got = score_sharded(lambda c, o: engine.score_batch(codes=c, offsets=o), codes, offsets)
if dist.get_rank() == 0:
    want = engine.score_batch(codes=codes, offsets=offsets)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    idx = np.arange(0, 40_000, 1999)
    parts = [codes[int(offsets[i]):int(offsets[i + 1])] for i in idx]
    o = np.zeros(len(idx) + 1, np.uint64); o[1:] = np.cumsum([len(p) for p in parts])
    assert np.array_equal(got[idx].view(np.uint32), OracleProfile("1400").score_batch(np.concatenate(parts), o).view(np.uint32))
    print("MULTIRANK_GPU_OK")
dist.destroy_process_group()
'''


@pytest.mark.gpu
def test_gloo_world_size_2_hip_scorer(tmp_path):
    """The sharded path with the HIP scorer under a process group: 2 ranks on the one GPU of the box
    (gloo for the gather), gathered scores bitwise equal to one process scoring everything."""
    script = tmp_path / "gpu_worker.py"
    script.write_text(GPU_WORKER.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = [p.communicate(timeout=180)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "MULTIRANK_GPU_OK" in outs[0]
