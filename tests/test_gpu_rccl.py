"""The N > 1 code path over RCCL on one GPU (run with -m gpu): bench.py
launched by torch.distributed.run with PG_FORCE_DIST=1 initialises the "nccl"
(= RCCL) process group at world size 1 and runs what the driver's N > 1
scaling runs run -- the barriers around the timed region, the max-over-ranks
and sum all-reduces of the timings and counters, and DeviceGA's per-generation
all-gather of fitness -- as one-rank RCCL collectives on device memory.  The
multi-rank data path itself is covered by the gloo tests (test_dist.py,
test_gpu_dist.py); an 8-GPU node is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_distributed_path_over_rccl(gpu):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PG_FORCE_DIST="1", OMP_NUM_THREADS="1")
    env.pop("PG_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--pop", "4096", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["config"]["process_group"] == "nccl", out["config"]
    assert out["n_gpus"] == 1 and out["steps"] == 2
    assert out["value"] > 0 and out["config"]["population"] == 4096
