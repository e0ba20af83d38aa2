"""DeviceGA sharded over ranks (run with -m gpu): 1, 2 and 3 ranks (gloo,
all on cuda:0, launched by torch.distributed.run as child processes) end three
generations in exactly the same state -- the replicated GA state never
diverges and the all-gather reassembles the shards in row order."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "_dist_ga_worker.py")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, out):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    if world == 1:
        cmd = [sys.executable, WORKER, out]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", WORKER, out]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


def test_sharded_device_ga_equals_single_process(gpu, tmp_path):
    outs = {}
    for world in (1, 2, 3):
        out = str(tmp_path / f"w{world}")
        _run(world, out)
        outs[world] = {k: np.load(os.path.join(out, f"{k}.npy"))
                       for k in ("population", "fitness", "hof", "hof_fitness")}
    for world in (2, 3):
        for k in outs[1]:
            np.testing.assert_array_equal(outs[world][k], outs[1][k], err_msg=f"{k} at world {world}")
