"""Checkpoint formats without a GPU: the block-streamed safetensors writer
round-trips and is readable by safetensors itself; the reference-format export
(save_checkpoint's pickle, utils.py:116-125) is what the drop-in
ga.load_population_from_file (ga.py:41-53) resumes from."""
import os
import subprocess
import sys
import types

import numpy as np
import torch

from pong_amd import checkpoint as C

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "neuro-genetic-pong-self-play_amd")


def test_tensor_file_round_trip_and_safetensors_compatible(tmp_path):
    rng = np.random.default_rng(0)
    tensors = {"population": torch.from_numpy(rng.standard_normal((37, 11))),
               "fitness": torch.from_numpy(rng.standard_normal(37)),
               "valid": torch.from_numpy(rng.integers(0, 2, 37).astype(np.uint8)),
               "hall_of_fame": torch.from_numpy(rng.standard_normal((0, 11)).astype(np.float32)),
               "hof_fitness": torch.zeros(0, dtype=torch.float64)}
    path = str(tmp_path / "ga.safetensors")
    C.write_tensors(path, tensors, {"format": C.FORMAT, "x": 3}, block_bytes=64)  # many small blocks
    got, meta = C.read_tensors(path, block_bytes=100)
    assert meta["format"] == C.FORMAT and meta["x"] == "3"
    for k, v in tensors.items():
        assert got[k].dtype == v.dtype and torch.equal(got[k], v), k
    from safetensors.torch import load_file
    ref = load_file(path)
    for k, v in tensors.items():
        assert torch.equal(ref[k], v), k


def test_export_reference_loads_in_dropin_ga(tmp_path):
    rng = np.random.default_rng(1)
    G = 20  # NETWORK_SHAPE [6, 2, 2]
    state = types.SimpleNamespace(
        nodes=[6, 2, 2], H=4,
        population=torch.from_numpy(rng.standard_normal((8, G))),
        fitness=torch.from_numpy(np.arange(8, dtype=np.float64) - 3.0),
        valid=torch.tensor([True] * 7 + [False]),
        hall_of_fame=torch.from_numpy(rng.standard_normal((3, G))),
        hof_member_fitness=np.array([9.0, 7.5, 7.5]))
    path = C.export_reference(state, str(tmp_path / "c_00_00_00.pkl"))
    r = C.read_reference(path)
    np.testing.assert_array_equal(r["genes"], state.population.numpy())
    np.testing.assert_array_equal(r["valid"], state.valid.numpy())
    np.testing.assert_array_equal(r["fitness"][:7], state.fitness.numpy()[:7])
    np.testing.assert_array_equal(r["hof_genes"], state.hall_of_fame.numpy())
    np.testing.assert_array_equal(r["hof_fitness"], state.hof_member_fitness)
    assert r["network_shape"] == [6, 2, 2] and r["hof_size"] == 4
    # the drop-in ga module resumes from an all-evaluated export (in a clean
    # process: ga loads checkpoints at import; ga.py:49 sorts by fitness, so
    # every individual must be valid, as after any eaSimple call)
    state.valid = torch.ones(8, dtype=torch.bool)
    path = C.export_reference(state, str(tmp_path / "c_00_00_01.pkl"))
    code = ("import sys; sys.path.insert(0, %r); import ga; pop = ga.load_population_from_file(%r); "
            "print(len(pop), pop[0].fitness.values[0], pop[-1].fitness.values[0], len(ga.hall_of_fame), "
            "ga.hall_of_fame[0].fitness.values[0], ga.NETWORK_SHAPE)" % (PKG, path))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=str(tmp_path), timeout=120)
    assert out.returncode == 0, out.stderr
    assert "8 4.0 -3.0 3 9.0 [6, 2, 2]" in out.stdout, out.stdout
