"""The reference's GA module surface (ga.py:1-99): ``toolbox``, ``hall_of_fame``,
``population``, ``creator.Fitness`` / ``creator.Individual`` and the checkpoint
loaders, with the operators DEAP registers there.

Changes from the reference:
  * ``toolbox.map`` is the batched map (pong_amd.batched): one device launch
    evaluates every invalid individual, in place of SCOOP's futures.map.
  * DEAP is taken from ``deap`` when installed, else from the in-repo
    restatement (pong_amd.deap_compat; deap is not installable offline).
"""
import glob
import os
import random

try:  # the real DEAP when present
    from deap import base, creator, tools
except ImportError:  # offline: DEAP's algorithms restated in-repo
    from pong_amd.deap_compat import base, creator, tools

from config import *  # noqa: F401,F403
from pong_amd import deap_pickle
from pong_amd.batched import batched_map
from utils import calculate_gene_size

CHECKPOINT_GLOB = 'checkpoints/checkpoints/*'


def _register_individual():
    toolbox.register("individual", tools.initRepeat, creator.Individual, toolbox.attr_float,
                     n=calculate_gene_size())


def load_population_from_file(checkpoint):
    """Unpickle a save_checkpoint file (utils.py:116-125): population sorted by
    fitness (best first); restores ``random``'s state, the hall of fame and
    NETWORK_SHAPE as module globals, like ga.py:41-53.  A file the reference
    wrote names ``deap.creator.*`` / ``deap.tools.support.HallOfFame``; without
    deap installed those resolve to the restatement (pong_amd.deap_pickle)."""
    global hall_of_fame, NETWORK_SHAPE
    print("Loading: {}".format(checkpoint))
    with open(checkpoint, "rb") as cp_file:
        cp = deap_pickle.load(cp_file)
    ranked = sorted(cp["population"], key=lambda ind: ind.fitness.values[0], reverse=True)
    random.setstate(cp["rndstate"])
    hall_of_fame = cp.get("hall_of_fame", hall_of_fame)
    NETWORK_SHAPE = cp.get("network_shape", NETWORK_SHAPE)  # noqa: F405
    return ranked


def load_latest_population():
    """The newest checkpoint by ctime, or None (ga.py:32-38)."""
    files = glob.glob(CHECKPOINT_GLOB)
    if not files:
        return None
    return load_population_from_file(max(files, key=os.path.getctime))


def load_best_population():
    """Scan every checkpoint and reload the one whose best individual is best (ga.py:56-74)."""
    global population
    best_score, best_checkpoint = 0, None
    for f in glob.glob(CHECKPOINT_GLOB):
        try:
            population = load_population_from_file(f)
            if best_score < population[0].fitness.values[0]:
                best_score, best_checkpoint = population[0].fitness.values[0], f
        except Exception as e:
            print(e)
    if best_checkpoint is None:
        return None
    print("Loading best model: {}\nwith score: {}".format(best_checkpoint, best_score))
    return load_population_from_file(best_checkpoint)


def load_or_create_pop():
    """Resume from the latest checkpoint, topped up to POPULATION_SIZE with fresh individuals (ga.py:13-29)."""
    global hall_of_fame, population
    population = load_latest_population()
    have = 0 if population is None else len(population)
    if have >= POPULATION_SIZE:  # noqa: F405
        return population[:POPULATION_SIZE]  # noqa: F405
    fresh = toolbox.population(n=(POPULATION_SIZE - have))  # noqa: F405
    return fresh if have == 0 else population + fresh


toolbox = base.Toolbox()
hall_of_fame = tools.HallOfFame(HALL_OF_FAME_AMOUNT)  # noqa: F405

creator.create("Fitness", base.Fitness, weights=(1.0,))
creator.create("Individual", list, fitness=creator.Fitness)

toolbox.register("map", batched_map)
toolbox.register("attr_float", random.random)
_register_individual()
toolbox.register("population", tools.initRepeat, list, toolbox.individual)
toolbox.register("mate", tools.cxBlend, alpha=CROSSOVER_BLEND_ALPHA)  # noqa: F405
toolbox.register("mutate", tools.mutGaussian, mu=GAUSSIAN_MUTATION_MEAN,  # noqa: F405
                 sigma=GAUSSIAN_MUTATION_SIGMA, indpb=PROBABILITY_OF_MUTATING_A_SINGLE_GENE)  # noqa: F405
toolbox.register("select", tools.selTournament, tournsize=TOURNAMENT_SIZE)  # noqa: F405

population = load_or_create_pop()
# re-registered: a loaded checkpoint may carry another gene count (ga.py:97-99)
_register_individual()
