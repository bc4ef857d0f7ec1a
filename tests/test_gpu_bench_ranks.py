"""bench.py's N > 1 path, run as the driver runs it (`bench.py --gpus 2`,
which starts the rank processes itself), on a one-GPU box: GG_BENCH_ONE_GPU=1
puts both ranks on GPU 0 and their process group on gloo, everything else --
the sharded C2 solve over the device-initiated IPC exchange with CGS2, the
max-over-ranks timing, rank 0's JSON line -- is the production code.  The
two-rank solve must take exactly the iterations of the same decomposition run
in one process (GG_DD_LOCAL): the exchanges move bits, not arithmetic."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _bench(args, env_extra):
    env = dict(os.environ, **env_extra)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_ipc_matches_local():
    common = ["--workload", "dd", "--dd-grid", "c2", "--grid", "200", "--steps", "1", "--warmup", "1"]
    two = _bench(["--gpus", "2"] + common, {"GG_BENCH_ONE_GPU": "1"})
    assert two["n_gpus"] == 2 and two["config"]["parallelism"] == "dd2"
    assert "GG_DD_IPC" in two["config"]["exchange"] and two["config"]["exchange_ranks"] == 2
    assert two["value"] > 0 and two["scaling"] == "strong"
    one = _bench(["--gpus", "1", "--dd-parts", "2"] + common, {})
    assert one["config"]["parts"] == 2
    assert two["config"]["iters_per_solve"] == one["config"]["iters_per_solve"]
    assert two["config"]["relres"] == one["config"]["relres"]
