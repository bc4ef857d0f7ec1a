"""Exchange latency of the sharded solve's GG_DD_IPC all-gather with P
processes on ONE GPU (the pool's boxes have one GPU each): the device-initiated
store / flag / poll protocol of k_ipc_allgather without the xGMI hop, i.e. a
lower bound for the 8-GPU figure.  Usage: python tools/ipc_exchange_probe.py [side]"""
import os
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "dd_rank_worker.py")
side = sys.argv[1] if len(sys.argv) > 1 else "1000"
for P in (2, 4):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [subprocess.Popen([sys.executable, "-u", WORKER, f"xtime:{side}", "/tmp"],
                              env=dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(P),
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2"),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(P)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    rc = [p.returncode for p in procs]
    print(f"P = {P} (C2 side {side}), exit codes {rc}")
    print("".join(o for o in outs if "IPC all-gather" in o) or "\n".join(o[-1500:] for o in outs), flush=True)
    if any(rc):
        sys.exit(1)
