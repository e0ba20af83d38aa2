"""The reference's main.py surface (main.py:28-185) on the MI355X path.

``evaluate(individual)`` keeps its signature and meaning (average reward of
GAMES_TO_PLAY games, as a 1-tuple); ``evaluate_population(individuals)`` is
the same computation for a whole batch in one device launch
(pg_eval_population), and ``toolbox.map`` routes eaSimple's
``map(evaluate, invalid_ind)`` there.  ``main()`` is the reference's endless
eaSimple + checkpoint loop.  Rendering and human play are out of scope.
"""
import numpy as np
import torch

try:
    from deap import algorithms, tools
except ImportError:
    from pong_amd.deap_compat import algorithms, tools

import ga
import utils
from config import *  # noqa: F401,F403
from ga import hall_of_fame, toolbox
from pong_amd import runtime, schedule
from utils import pick_hall_of_famer, save_checkpoint


def _evaluator():
    # the network shape is utils' binding, as create_model_from_genes sees it (utils.py:80-87)
    return runtime.evaluator(utils.NETWORK_SHAPE, utils.BIAS, GAMES_TO_PLAY, GENOME_DTYPE,  # noqa: F405
                             PRECISION, PHYSICS_SEED, DEVICE)  # noqa: F405


def _fitness_tuples(fitness, status):
    for f, failed in zip(fitness, status):
        if failed:  # calculate_reward with total_frames == 0 (utils.py:106-108)
            raise ZeroDivisionError("float division by zero")
        yield (float(f),)


def evaluate_population(individuals):
    """evaluate() for every individual, in order; returns an iterator of 1-tuples.

    Hall-of-fame picks are drawn up front in the order a sequential map would
    draw them; an individual whose evaluation would raise ZeroDivisionError
    raises it when its result is reached, as a lazy map does.
    """
    individuals = list(individuals)
    n = len(individuals)
    if n == 0:
        return iter(())
    ev = _evaluator()
    genes = utils.calculate_gene_size()
    kind, opp, mult, members = schedule.reference_schedule(n, GAMES_TO_PLAY, hall_of_fame,  # noqa: F405
                                                           pick_hall_of_famer)
    dev = ev.device
    genomes = runtime.genomes_to_device(individuals, genes, ev)
    opponents = runtime.genomes_to_device(members, genes, ev) if members else None
    res, _ = ev.evaluate(genomes, torch.from_numpy(kind).to(dev), torch.from_numpy(opp).to(dev),
                         torch.from_numpy(mult).to(dev), opponents=opponents)
    return _fitness_tuples(res.fitness.cpu().numpy(), res.status.cpu().numpy())


def evaluate(individual=None, render=RENDER):  # noqa: F405
    """Average reward of the individual's GAMES_TO_PLAY games (main.py:28-66).

    ``render=True`` (render_game, main.py:115-125) writes each game as an
    animated GIF under REPLAY_DIR instead of a gym viewer window: the games are
    replayed from their action traces and rasterised on the device
    (pong_amd.replay)."""
    if render:
        return _evaluate_rendered(individual)
    return next(evaluate_population([individual]))


def _evaluate_rendered(individual):
    import os

    from pong_amd import replay
    ev = _evaluator()
    genes = utils.calculate_gene_size()
    kind, opp, mult, members = schedule.reference_schedule(1, GAMES_TO_PLAY, hall_of_fame,  # noqa: F405
                                                           pick_hall_of_famer)
    genomes = runtime.genomes_to_device([individual], genes, ev)
    opponents = runtime.genomes_to_device(members, genes, ev) if members else None
    res, frames = replay.replay(ev, genomes[0], kind[0], opp[0], mult[0], opponents=opponents)
    for g, f in enumerate(frames):
        if len(f):
            replay.write_gif(f, os.path.join(REPLAY_DIR, f"game_{g}.gif"), fps=FPS)  # noqa: F405
    return next(_fitness_tuples(res.fitness.cpu().numpy(), res.status.cpu().numpy()))


evaluate.__pong_batch__ = evaluate_population


def calculate_timeout_and_frames(last_score, score_info, timeout_counter, total_frames):
    """Frames without a score change, folded into total_frames at each change (main.py:128-135)."""
    if last_score is None:
        return timeout_counter, total_frames
    if last_score == score_info:
        return timeout_counter + 1.0, total_frames
    return 0.0, total_frames + timeout_counter


def main():
    stats = tools.Statistics(lambda ind: ind.fitness.values)
    for name, fn in (("avg", np.mean), ("std", np.std), ("min", np.min), ("max", np.max)):
        stats.register(name, fn)
    while True:
        ga.population, log = algorithms.eaSimple(
            ga.population, toolbox,
            cxpb=CROSSOVER_BLEND_PROBABILITY, mutpb=GAUSSIAN_MUTATION_PROBABILITY,  # noqa: F405
            ngen=GENERATIONS_BEFORE_SAVE,  # noqa: F405
            stats=stats, halloffame=hall_of_fame, verbose=True)
        print(log)
        save_checkpoint(ga.population, hall_of_fame)


toolbox.register("evaluate", evaluate)

if __name__ == '__main__':
    main()
