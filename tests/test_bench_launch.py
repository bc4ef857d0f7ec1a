"""bench.py's multi-GPU launch contract, on CPU (no GPU call is made).

`bench.py --gpus N` without torchrun must start N rank processes with the
torch.distributed environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), exit
with their status, stop the others when one fails, and refuse N larger than
the visible GPU count; under torchrun WORLD_SIZE must equal --gpus.
"""
import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

CHILD = r"""
import json, os, sys, time
out = sys.argv[1]
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
if len(sys.argv) > 2 and os.environ["RANK"] == sys.argv[2]:
    sys.exit(3)                      # this rank fails
if len(sys.argv) > 2:
    time.sleep(60)                   # the others would wait in a collective
"""


def test_spawn_sets_rank_environment(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    rc = bench.spawn_ranks(4, [sys.executable, str(script), str(tmp_path)], visible=4)
    assert rc == 0
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(4)]
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1"
    assert len({e["MASTER_PORT"] for e in envs}) == 1


def test_spawn_failure_stops_the_other_ranks(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    t0 = time.time()
    rc = bench.spawn_ranks(3, [sys.executable, str(script), str(tmp_path), "1"], visible=3)
    assert rc == 3
    assert time.time() - t0 < 30          # the sleeping ranks were terminated


def test_spawn_refuses_more_ranks_than_gpus(tmp_path):
    assert bench.spawn_ranks(8, [sys.executable, "-c", "pass"], visible=1) == 2


@pytest.mark.parametrize("argv, env, code", [
    (["--gpus", "2"], {}, 2),                                   # no GPU in this container
    (["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0"}, 2),     # torchrun world != --gpus
])
def test_bench_refuses_bad_world(argv, env, code):
    e = dict(os.environ, **env)
    e.pop("WORLD_SIZE", None) if "WORLD_SIZE" not in env else None
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + argv, env=e,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == code, p.stderr[-2000:]
    assert "bench.py:" in p.stderr
