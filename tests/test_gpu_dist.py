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


def _run(world, out, *extra, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    if world == 1:
        cmd = [sys.executable, WORKER, out, *extra]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", WORKER, out, *extra]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:  # the first rank's traceback, not just the launcher's tail
        err = r.stderr
        at = err.find("Traceback")
        raise AssertionError(r.stdout[-1000:] + (err[at:at + 4000] if at >= 0 else "") + err[-2000:])


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


def test_config4_sharded_524k_equals_single_process(gpu, oracle, tmp_path):
    """BASELINE config 4 readiness: population 524 288, [6,64,3] self-play vs a
    131 072-row hall of fame, two generations (the initial evaluation and one
    eaSimple step), sharded over 8 gloo ranks on cuda:0 (the N = 8 code path:
    rank shards, one all-gather of fitness per generation) -- equal to the
    single-process run row for row, and 48 of rank 0's evaluated genomes
    re-played by the oracle."""
    import json
    outs = {}
    for world in (1, 8):
        out = str(tmp_path / f"c4w{world}")
        _run(world, out, "config4", timeout=600)
        outs[world] = {k: np.load(os.path.join(out, f"{k}.npy"))
                       for k in ("pop_hash", "fitness", "hof_hash", "hof_fitness")}
        with open(os.path.join(out, "profile.json")) as fh:
            outs[world]["profile"] = json.load(fh)
        if world == 8:
            smp = dict(np.load(os.path.join(out, "sample.npz")))
    for k in ("pop_hash", "fitness", "hof_hash", "hof_fitness"):
        np.testing.assert_array_equal(outs[8][k], outs[1][k], err_msg=k)
    assert outs[8]["profile"]["logbook"] == outs[1]["profile"]["logbook"]
    played = smp["played"].astype(bool)
    assert played.sum() > 0
    ref = oracle.eval_population(smp["genomes"][played], [6, 64, 3], smp["kind"][played], smp["opp"][played],
                                 smp["mult"][played], opponents=smp["opponents"], n_threads=8)
    np.testing.assert_array_equal(smp["fitness"][played], ref["fitness"])
    np.testing.assert_array_equal(smp["frames"][played], ref["frames"])
    rec = {w: outs[w]["profile"] for w in (1, 8)}
    repo = os.path.dirname(HERE)
    if os.path.isdir(os.path.join(repo, "gpurun_out")):
        with open(os.path.join(repo, "gpurun_out", "config4_profile.json"), "w") as fh:
            json.dump(rec, fh, indent=1)


def test_wide_config5_split_equals_single_process(gpu, oracle, tmp_path):
    """BASELINE config 5's 1 -> N split: the [6,512,512,3] network (f32 genomes,
    k_wide), P = 256 self-play vs a 64-row hall, two generations, at 1 rank, 2
    ranks (contiguous shards) and 2 and 8 ranks with length-balanced shards
    (the rows dealt by predicted game length, DeviceGA.balance_shards) -- every
    run ends in the same population, fitness and hall of fame, and 4 of rank
    0's last evaluated genomes are re-played by the oracle."""
    import json
    outs = {}
    for world, mode in ((1, "wide"), (2, "wide"), (2, "wide_balanced"), (8, "wide_balanced")):
        out = str(tmp_path / f"{mode}{world}")
        _run(world, out, mode, timeout=600)
        outs[(world, mode)] = {k: np.load(os.path.join(out, f"{k}.npy"))
                               for k in ("pop_hash", "fitness", "hof_hash", "hof_fitness")}
        with open(os.path.join(out, "profile.json")) as fh:
            outs[(world, mode)]["logbook"] = json.load(fh)["logbook"]
        smp = dict(np.load(os.path.join(out, "sample.npz")))
        ref = oracle.eval_population(smp["genomes"], [6, 512, 512, 3], smp["kind"], smp["opp"], smp["mult"],
                                     opponents=smp["opponents"], n_threads=8)
        np.testing.assert_array_equal(smp["fitness"], ref["fitness"], err_msg=f"{mode} {world}")
        np.testing.assert_array_equal(smp["frames"], ref["frames"], err_msg=f"{mode} {world}")
    base = outs[(1, "wide")]
    for key, o in outs.items():
        for k in ("pop_hash", "fitness", "hof_hash", "hof_fitness"):
            np.testing.assert_array_equal(o[k], base[k], err_msg=f"{k} at {key}")
        assert o["logbook"] == base["logbook"], key


def test_sliced_hall_smaller_than_blocks(gpu, tmp_path):
    """A sliced hall with fewer members than row blocks (P = 96 in four
    24-row blocks, a 3-member hall: K = 3, block 3 plays slice 0): four ranks,
    one block each, each passing only its slice, end three generations equal to
    the single process that passes the whole hall (round-5 review)."""
    outs = {}
    for world in (1, 4):
        out = str(tmp_path / f"s{world}")
        _run(world, out, "slices")
        outs[world] = {k: np.load(os.path.join(out, f"{k}.npy"))
                       for k in ("population", "fitness", "hof", "hof_fitness", "rows")}
    assert tuple(outs[4]["rows"][2:]) == (3, 0)  # rank 0: 3 slices, its block 0 plays slice 0
    for k in ("population", "fitness", "hof", "hof_fitness"):
        np.testing.assert_array_equal(outs[4][k], outs[1][k], err_msg=k)
