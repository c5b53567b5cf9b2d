"""The benchmark's N > 1 code paths, rehearsed on one GPU: two ranks launched as the driver launches
them (torch.distributed.run, one process per rank), here both on GPU 0 with torch.distributed over
gloo and the engine's host transport instead of RCCL (SHD_BENCH_REHEARSAL=1, bench.py).  Every
sharded leg runs -- the replicated C2 build with its status agreement, the sharded C5 relay round,
the relay + queue rounds -- and the bench's own all-rank parity checks must pass."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_rehearsal():
    env = dict(os.environ, SHD_BENCH_REHEARSAL="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", "--steps", "4",
           "--warmup", "1", "--relay-steps", "2", "--no-c3", "--no-c4", "--no-codel", "--no-tbucket"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["parity_check"] == {"c2_table_bit_exact_all_ranks": True, "relay_round_bit_exact_all_ranks": True}
    assert d["relay"]["pipeline"] == 8   # the stamp's bins went to their ranks as stamped
    assert d["relay"]["equeue"]["popped_per_round_rank0"] > 0
