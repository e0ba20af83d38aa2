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


# ------------------------------------------- reference checkpoints both ways
GOLD = os.path.join(REPO, "tests", "golden")
STUB_DEAP = os.path.join(GOLD, "stub_deap")
REF_PKL = os.path.join(GOLD, "deap_checkpoint.pkl")


def _side():
    import json
    with open(os.path.join(GOLD, "deap_checkpoint.json")) as fh:
        return json.load(fh)


def _run(code, cwd):
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=str(cwd), timeout=120)
    assert out.returncode == 0, out.stderr
    import json
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_reference_checkpoint_names_deap_classes():
    from pong_amd import deap_pickle as D
    names = D.global_names(open(REF_PKL, "rb").read())
    assert names == {"deap.creator.Individual", "deap.creator.Fitness", "deap.tools.support.HallOfFame",
                     "_operator.eq"}


def test_reference_checkpoint_resumes_in_dropin_ga(tmp_path):
    """A pickle written by the reference's save_checkpoint (deap class paths)
    loads through the drop-in ga.load_population_from_file (ga.py:41-53)
    without deap: sorted population, hall of fame, NETWORK_SHAPE and the
    random state all come back."""
    side = _side()
    code = ("import sys, json, random; sys.path.insert(0, %r); import ga\n"
            "assert 'deap' not in sys.modules\n"
            "pop = ga.load_population_from_file(%r)\n"
            "print(json.dumps({'genes': [list(i) for i in pop], 'fit': [i.fitness.values[0] for i in pop],\n"
            " 'cls': type(pop[0]).__module__ + '.' + type(pop[0]).__name__,\n"
            " 'hof_genes': [list(i) for i in ga.hall_of_fame], 'hof_fit': [i.fitness.values[0] for i in ga.hall_of_fame],\n"
            " 'hof_keys': [k.values[0] for k in ga.hall_of_fame.keys], 'maxsize': ga.hall_of_fame.maxsize,\n"
            " 'shape': ga.NETWORK_SHAPE, 'next': [random.random() for _ in range(4)]}))" % (PKG, REF_PKL))
    got = _run(code, tmp_path)
    order = sorted(range(len(side["fitness"])), key=lambda i: side["fitness"][i], reverse=True)  # stable, ga.py:49
    assert got["fit"] == [side["fitness"][i] for i in order]
    assert got["genes"] == [side["genes"][i] for i in order]
    assert got["cls"] == "pong_amd.deap_compat.creator.Individual"
    assert got["hof_genes"] == side["hof_genes"] and got["hof_fit"] == side["hof_fitness"]
    assert got["hof_keys"] == sorted(side["hof_fitness"]) and got["maxsize"] == side["hof_maxsize"]
    assert got["shape"] == side["network_shape"]
    assert got["next"] == side["next_random"]


def test_reference_checkpoint_continues_bit_exact(tmp_path):
    """Resuming eaSimple from the reference's pickle equals resuming it from the
    same state rebuilt from plain numbers (population, hall of fame, rndstate)."""
    code = ("import sys, json, random; sys.path.insert(0, %r); import ga\n"
            "from pong_amd.deap_compat import algorithms, creator, tools\n"
            "def run(pop, hof):\n"
            "    ga.toolbox.register('evaluate', lambda ind: (sum(ind) - 0.01 * ind[0] ** 2,))\n"
            "    ga.toolbox.register('map', map)\n"
            "    pop, log = algorithms.eaSimple(pop, ga.toolbox, 0.9, 0.9, 3, halloffame=hof, verbose=False)\n"
            "    return [list(i) for i in pop] + [list(i) for i in hof], [random.random()]\n"
            "pop = ga.load_population_from_file(%r)\n"
            "a = run(pop, ga.hall_of_fame)\n"
            "side = json.load(open(%r))\n"
            "pop2 = []\n"
            "for g, f in zip(side['genes'], side['fitness']):\n"
            "    i = creator.Individual(g); i.fitness.values = (f,); pop2.append(i)\n"
            "pop2 = sorted(pop2, key=lambda x: x.fitness.values[0], reverse=True)\n"
            "hof2 = tools.HallOfFame(side['hof_maxsize'])\n"
            "for g, f in zip(side['hof_genes'], side['hof_fitness']):\n"
            "    i = creator.Individual(g); i.fitness.values = (f,); hof2.insert(i)\n"
            "ga.load_population_from_file(%r)  # rndstate only\n"
            "b = run(pop2, hof2)\n"
            "print(json.dumps({'same': a == b, 'n': len(a[0])}))"
            % (PKG, REF_PKL, os.path.join(GOLD, "deap_checkpoint.json"), REF_PKL))
    got = _run(code, tmp_path)
    assert got["same"] and got["n"] == 64 + 16  # population + the hall of fame, refilled to maxsize


def test_export_reference_pickles_deap_class_paths(tmp_path):
    """export_reference names DEAP's classes, so a process with a DEAP-layout
    package (stub_deap) and a plain pickle.load -- the reference's
    ga.load_population_from_file -- reads it; sys.modules is left as it was."""
    from pong_amd import deap_pickle as D
    rng = np.random.default_rng(3)
    G = 20
    state = types.SimpleNamespace(
        nodes=[6, 2, 2], H=4, population=torch.from_numpy(rng.standard_normal((8, G))),
        fitness=torch.from_numpy(np.arange(8, dtype=np.float64) - 3.0), valid=torch.ones(8, dtype=torch.bool),
        hall_of_fame=torch.from_numpy(rng.standard_normal((3, G))), hof_member_fitness=np.array([9.0, 7.5, 7.5]))
    before = {k for k in sys.modules if k == "deap" or k.startswith("deap.")}
    path = C.export_reference(state, str(tmp_path / "c_00_00_02.pkl"))
    assert {k for k in sys.modules if k == "deap" or k.startswith("deap.")} == before
    from pong_amd.deap_compat import creator as cc, tools as ct
    assert cc.Individual.__module__ == "pong_amd.deap_compat.creator"
    assert ct.HallOfFame.__module__ == "pong_amd.deap_compat.tools"
    names = D.global_names(open(path, "rb").read())
    assert names <= {"deap.creator.Individual", "deap.creator.Fitness", "deap.tools.support.HallOfFame",
                     "_operator.eq"}, names
    assert not any("pong_amd" in n for n in names)
    code = ("import sys, json, pickle; sys.path.insert(0, %r)\n"
            "from deap import base, creator\n"
            "creator.create('Fitness', base.Fitness, weights=(1.0,))\n"
            "creator.create('Individual', list, fitness=creator.Fitness)\n"
            "cp = pickle.load(open(%r, 'rb'))\n"
            "pop, hof = cp['population'], cp['hall_of_fame']\n"
            "print(json.dumps({'mod': type(pop[0]).__module__, 'hmod': type(hof).__module__,\n"
            " 'genes': [list(i) for i in pop], 'fit': [i.fitness.values[0] for i in pop],\n"
            " 'hof_fit': [i.fitness.values[0] for i in hof.items], 'maxsize': hof.maxsize,\n"
            " 'shape': cp['network_shape']}))" % (STUB_DEAP, path))
    got = _run(code, tmp_path)
    assert got["mod"] == "deap.creator" and got["hmod"] == "deap.tools.support"
    assert got["genes"] == state.population.numpy().tolist()
    assert got["fit"] == state.fitness.numpy().tolist()
    assert got["hof_fit"] == [9.0, 7.5, 7.5] and got["maxsize"] == 4 and got["shape"] == [6, 2, 2]


def test_checkpoint_unpickler_refuses_foreign_globals():
    import pickle

    import pytest

    from pong_amd import deap_pickle as D
    with pytest.raises(pickle.UnpicklingError):
        D.loads(pickle.dumps(os.getcwd))  # posix.getcwd: not a checkpoint global
    with pytest.raises(pickle.UnpicklingError):
        D.loads(b"cos\nsystem\n(S'true'\ntR.")


def test_checkpoint_unpickler_refuses_operator_gadgets():
    """Only operator.eq of the operator modules: attrgetter / getitem /
    methodcaller reach eval through a reconstructor's __globals__ with GLOBAL
    and REDUCE alone, and a dotted name walks attributes (protocol 4)."""
    import pickle

    import pytest

    from pong_amd import deap_pickle as D
    attr_globals = b"c_operator\nattrgetter\n(S'__globals__'\ntR(ccopyreg\n_reconstructor\ntR."
    with pytest.raises(pickle.UnpicklingError):
        D.loads(attr_globals)
    getitem = (b"c_operator\ngetitem\n(c_operator\nattrgetter\n(S'__globals__'\ntR(ccopyreg\n_reconstructor\n"
               b"tRS'__builtins__'\ntR.")
    with pytest.raises(pickle.UnpicklingError):
        D.loads(getitem)
    for mod in ("_operator", "operator"):
        for name in ("methodcaller", "itemgetter", "attrgetter", "getitem"):
            with pytest.raises(pickle.UnpicklingError):
                D.loads(b"c" + mod.encode() + b"\n" + name.encode() + b"\n.")
    # a dotted name of an allowed global (STACK_GLOBAL, protocol 4)
    dotted = b"\x80\x04\x95\x00\x00\x00\x00\x00\x00\x00\x00\x8c\x07copyreg\x8c\x1a_reconstructor.__globals__\x93."
    with pytest.raises(pickle.UnpicklingError):
        D.loads(dotted)
    # what a hall of fame does hold still loads
    import operator
    assert D.loads(pickle.dumps(operator.eq)) is operator.eq


def test_dropin_save_checkpoint_is_reference_readable(tmp_path):
    """The drop-in main()'s checkpoint (utils.save_checkpoint after one
    GENERATIONS_BEFORE_SAVE block of eaSimple at POPULATION_SIZE 64, as
    main.py:165-173; a CPU evaluate stands in for the device map) names only
    DEAP's classes, and a process with a DEAP-layout package and the
    reference's plain pickle.load (ga.py:41-45) reads it back."""
    code = ("import sys, json; sys.path.insert(0, %r); import ga, utils\n"
            "from pong_amd.deap_compat import algorithms\n"
            "ga.toolbox.register('evaluate', lambda ind: (sum(ind) - 0.01 * ind[0] ** 2,))\n"
            "ga.toolbox.register('map', map)\n"
            "pop, log = algorithms.eaSimple(ga.population, ga.toolbox, ga.CROSSOVER_BLEND_PROBABILITY,\n"
            "    ga.GAUSSIAN_MUTATION_PROBABILITY, ga.GENERATIONS_BEFORE_SAVE, halloffame=ga.hall_of_fame,\n"
            "    verbose=False)\n"
            "path = utils.save_checkpoint(pop, ga.hall_of_fame)\n"
            "print(json.dumps({'path': path, 'genes': [list(i) for i in pop], 'fit': [i.fitness.values[0] for i in pop],\n"
            " 'hof_fit': [i.fitness.values[0] for i in ga.hall_of_fame.items], 'maxsize': ga.hall_of_fame.maxsize}))"
            % PKG)
    saved = _run(code, tmp_path)
    path = os.path.join(str(tmp_path), saved["path"])
    from pong_amd import deap_pickle as D
    data = open(path, "rb").read()
    names = D.global_names(data)
    assert names <= {"deap.creator.Individual", "deap.creator.Fitness", "deap.tools.support.HallOfFame",
                     "_operator.eq"}, names
    assert "deap.creator.Individual" in names and "deap.tools.support.HallOfFame" in names
    assert len(saved["genes"]) == 64 and saved["maxsize"] == 16 and len(saved["hof_fit"]) == 16
    code = ("import sys, json, pickle; sys.path.insert(0, %r)\n"
            "from deap import base, creator\n"
            "creator.create('Fitness', base.Fitness, weights=(1.0,))\n"
            "creator.create('Individual', list, fitness=creator.Fitness)\n"
            "cp = pickle.load(open(%r, 'rb'))\n"
            "pop, hof = cp['population'], cp['hall_of_fame']\n"
            "print(json.dumps({'mod': type(pop[0]).__module__, 'hmod': type(hof).__module__,\n"
            " 'genes': [list(i) for i in pop], 'fit': [i.fitness.values[0] for i in pop],\n"
            " 'hof_fit': [i.fitness.values[0] for i in hof.items], 'maxsize': hof.maxsize,\n"
            " 'shape': cp['network_shape'], 'rnd': cp['rndstate'][0]}))" % (STUB_DEAP, path))
    got = _run(code, tmp_path)
    assert got["mod"] == "deap.creator" and got["hmod"] == "deap.tools.support"
    assert got["genes"] == saved["genes"] and got["fit"] == saved["fit"]
    assert got["hof_fit"] == saved["hof_fit"] and got["maxsize"] == 16
    assert got["shape"] == [6, 2, 2] and got["rnd"] == 3
    # and the drop-in ga resumes from it (ga.py:13-29 at import: the newest checkpoint)
    code = ("import sys, json; sys.path.insert(0, %r); import ga\n"
            "print(json.dumps({'n': len(ga.population), 'best': ga.population[0].fitness.values[0],\n"
            " 'hof': len(ga.hall_of_fame)}))" % PKG)
    got = _run(code, tmp_path)
    assert got == {"n": 64, "best": max(saved["fit"]), "hof": 16}
