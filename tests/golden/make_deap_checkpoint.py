#!/usr/bin/env python3
"""Write ``deap_checkpoint.pkl``: a checkpoint as the reference writes it.

The pickle is produced by the REFERENCE's own ``utils.save_checkpoint``
(/root/reference/utils.py:116-125), imported in this container, on a
population and hall of fame made with the classes ga.py:78-81 registers.  deap
is not installed here, so those classes come from ``stub_deap/`` -- a
stand-in with DEAP's module layout (``deap.creator.Individual``,
``deap.creator.Fitness``, ``deap.tools.support.HallOfFame``, instance
attributes ``fitness`` / ``wvalues`` / ``maxsize, keys, items, similar``), so
the file names exactly the class paths a real-DEAP run pickles.
``deap_checkpoint.json`` holds the same data as plain numbers for the tests.

Shims: ``np.int = int`` (config.py:21,26), a stub ``scoop`` with ``logger``.
Usage:  python tests/golden/make_deap_checkpoint.py
"""
from __future__ import annotations

import glob
import json
import logging
import os
import random
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

np.int = int  # type: ignore[attr-defined]
_scoop = types.ModuleType("scoop")
_scoop.logger = logging.getLogger("scoop-stub")
sys.modules["scoop"] = _scoop
sys.path.insert(0, os.path.join(HERE, "stub_deap"))
sys.path.insert(1, REF)

from deap import base, creator, tools  # noqa: E402  (the stand-in)
import config as ref_config  # noqa: E402
import utils as ref_utils  # noqa: E402

POP, SEED = 64, 20261016


def main():
    creator.create("Fitness", base.Fitness, weights=(1.0,))       # ga.py:80
    creator.create("Individual", list, fitness=creator.Fitness)   # ga.py:81
    G = ref_utils.calculate_gene_size()                           # utils.py:128-136, [6,2,2] -> 20
    random.seed(SEED)
    population = [creator.Individual([random.random() for _ in range(G)]) for _ in range(POP)]  # ga.py:85-87
    # an evolved-looking population: genes moved by a few N(0, 0.9) steps, fitness
    # of evaluate()'s range, two exact ties (the sort at ga.py:49 must keep order)
    for ind in population:
        for i in range(G):
            ind[i] += random.gauss(0.0, 0.9)
        ind.fitness.values = (round(random.uniform(-3.0, 6.0), 6),)
    population[7].fitness.values = population[3].fitness.values
    population[40].fitness.values = population[3].fitness.values
    hof = tools.HallOfFame(ref_config.HALL_OF_FAME_AMOUNT)        # ga.py:78
    for ind in sorted(population, key=lambda x: x.fitness.values[0], reverse=True)[:12]:
        hof.insert(ind)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            ref_utils.save_checkpoint(population, hof)            # utils.py:116-125
            next_random = [random.random() for _ in range(4)]     # the saved rndstate continues here
            written = glob.glob(os.path.join(tmp, "checkpoints", "checkpoints", "*.pkl"))
            assert len(written) == 1, written
            shutil.copyfile(written[0], os.path.join(HERE, "deap_checkpoint.pkl"))
        finally:
            os.chdir(cwd)
    side = {"generator": "tests/golden/make_deap_checkpoint.py (reference utils.save_checkpoint + stub_deap)",
            "network_shape": list(ref_config.NETWORK_SHAPE), "hof_maxsize": hof.maxsize,
            "genes": [list(map(float, ind)) for ind in population],
            "fitness": [ind.fitness.values[0] for ind in population],
            "hof_genes": [list(map(float, ind)) for ind in hof.items],
            "hof_fitness": [ind.fitness.values[0] for ind in hof.items],
            "next_random": next_random}
    with open(os.path.join(HERE, "deap_checkpoint.json"), "w") as fh:
        json.dump(side, fh)
    print("wrote deap_checkpoint.pkl / .json:", POP, "individuals x", G, "genes, hall of fame", len(hof))


if __name__ == "__main__":
    main()
