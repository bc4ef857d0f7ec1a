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


LOCKSTEP = r"""
import json, os, sys
sys.path.insert(0, sys.argv[1])
import torch, torch.distributed as dist
import bench
dist.init_process_group("gloo", init_method="env://")
rank = dist.get_rank()
fail = sys.argv[3]                   # "<phase>:<rank>" or "none"
ran = []

def step(name):
    def fn():
        ran.append(name)
        if name == "connect":        # a collective inside a step, as bench_dd's all_gather_object
            lst = [None] * dist.get_world_size()
            dist.all_gather_object(lst, rank)
        if fail == f"{name}:{rank}":
            raise RuntimeError("injected")
    return fn

ok = bench.lockstep(torch, dist, None, rank, [(n, step(n)) for n in ("create", "connect", "check")])
with open(os.path.join(sys.argv[2], f"r{rank}.json"), "w") as f:
    json.dump({"ok": ok, "ran": ran}, f)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("fail", ["none", "create:1", "connect:0", "check:1"])
def test_ipc_setup_lockstep_fallback(tmp_path, fail):
    """bench_dd's IPC setup (bench.lockstep): a step failing on ONE rank takes
    every rank to the RCCL fallback at that step -- no rank is left waiting in a
    later step's collective (2 gloo ranks on CPU)"""
    script = tmp_path / "lockstep.py"
    script.write_text(LOCKSTEP)
    t0 = time.time()
    rc = bench.spawn_ranks(2, [sys.executable, str(script), REPO, str(tmp_path), fail], visible=2)
    assert rc == 0 and time.time() - t0 < 120
    res = [json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(2)]
    order = ["create", "connect", "check"]
    stop = order.index(fail.split(":")[0]) + 1 if fail != "none" else 3
    for r in res:
        assert r["ok"] == (fail == "none")
        assert r["ran"] == order[:stop]          # every rank stopped after the same step


@pytest.mark.parametrize("argv", [["--gpus", "2"], ["--dd-rank", "8"], ["--dd-rank", "-1"]])
def test_loopback_refuses_other_than_one_rank_alone(argv, monkeypatch, capsys):
    """--dd-comm loopback times ONE rank of --dd-parts alone on one GPU"""
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "dd", "--dd-comm", "loopback", "--dd-parts", "8"] + argv)
    with pytest.raises(SystemExit) as e:
        bench.parse()
    assert e.value.code == 2
    assert "loopback" in capsys.readouterr().err


def test_loopback_arguments_parse(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "dd", "--dd-comm", "loopback", "--dd-parts", "8",
                                      "--dd-rank", "7"])
    a = bench.parse()
    assert (a.dd_comm, a.dd_parts, a.dd_rank, a.gpus) == ("loopback", 8, 7, 1)
