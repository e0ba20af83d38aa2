"""The drop-in surface on the MI355X (run with -m gpu): the reference's
``toolbox.map(toolbox.evaluate, individuals)`` and ``NeuralNetwork.run``
through ga.py / main.py / numpy_nn.py give the reference's own numbers."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class _Fit:
    def __init__(self, v):
        self.values = (v,)
        self.valid = True


class _Member(list):
    def __init__(self, genes, fit):
        super().__init__(genes)
        self.fitness = _Fit(fit)


class _HoF:
    def __init__(self, items):
        self.items = items


def test_toolbox_map_evaluate_matches_reference(gpu, golden):
    """evaluate.json / evaluate_s3.json: fitness of the REAL evaluate() (incl.
    hall-of-fame games; _s3: N(0, 3) genes, negative hall-of-fame fitness)."""
    import ga
    import main
    import utils
    saved = (utils.NETWORK_SHAPE, main.hall_of_fame)
    try:
        for case in golden("evaluate.json") + golden("evaluate_s3.json"):
            utils.NETWORK_SHAPE = case["shape"]
            main.hall_of_fame = _HoF([_Member(g, f) for g, f in zip(case["hof_genes"], case["hof_fitness"])])
            random.seed(case["random_seed"])
            inds = [list(g) for g in case["individuals"]]
            got = [fit[0] for fit in ga.toolbox.map(ga.toolbox.evaluate, inds)]
            assert got == case["fitness"]
    finally:
        utils.NETWORK_SHAPE, main.hall_of_fame = saved


@pytest.mark.parametrize("key", ["6x2x2", "6x64x3", "6x8x8x3"])
def test_neural_network_run_matches_reference(gpu, golden, key):
    from numpy_nn import NeuralNetwork
    g = golden("nn_forward.npz")
    shape = [int(v) for v in g[f"{key}__shape"]]
    genes, gidx, x = g[f"{key}__genes"], g[f"{key}__gidx"], g[f"{key}__x"]
    for s in range(0, len(x), 37):  # a spread of samples: one device call each
        net = NeuralNetwork(nodes=shape, weights=list(genes[gidx[s]]), bias=True)
        action = net.run(list(x[s]))
        idx = int(g[f"{key}__idx"][s])
        assert action == ([1, 0] if idx == 0 else [0, 1] if idx == 1 else [0, 0])
        np.testing.assert_allclose(net.list_of_transitional_arrays[-1][:-1], g[f"{key}__act"][s], atol=1e-5)


def test_easimple_device_equals_sequential_oracle(gpu, oracle):
    """Three generations of the reference's eaSimple (pop 64, [6,2,2]): the
    batched device map and a sequential per-individual oracle evaluate draw the
    same hall-of-fame opponents and produce identical populations and logs."""
    import copy

    import ga
    import main
    import utils
    from pong_amd import schedule
    from pong_amd.deap_compat import algorithms, tools

    def oracle_evaluate(individual):
        kind, opp, mult, members = schedule.reference_schedule(1, 6, main.hall_of_fame, utils.pick_hall_of_famer)
        opps = np.array([list(m) for m in members]) if members else None
        r = oracle.eval_population(np.array([list(individual)[:20]]), [6, 2, 2], kind, opp, mult, opponents=opps)
        return (float(r["fitness"][0]),)

    def run(evaluate_fn, map_fn):
        tb = copy.copy(ga.toolbox)
        tb.register("evaluate", evaluate_fn)
        tb.register("map", map_fn)
        random.seed(2024)
        pop = tb.population(n=64)
        hof = tools.HallOfFame(16)
        main.hall_of_fame = hof
        stats = tools.Statistics(lambda ind: ind.fitness.values)
        stats.register("max", np.max)
        stats.register("avg", np.mean)
        pop, log = algorithms.eaSimple(pop, tb, cxpb=0.9, mutpb=0.9, ngen=3, stats=stats, halloffame=hof,
                                       verbose=False)
        return [list(i) for i in pop], [i.fitness.values for i in pop], list(log)

    saved = main.hall_of_fame
    try:
        dev = run(main.evaluate, ga.toolbox.map)
        seq = run(oracle_evaluate, map)
    finally:
        main.hall_of_fame = saved
    assert dev[1] == seq[1]
    assert dev[0] == seq[0]
    assert dev[2] == seq[2]


def test_main_block_checkpoint_reference_readable(gpu, tmp_path, monkeypatch):
    """One block of the drop-in main() (main.py:165-173: eaSimple for
    GENERATIONS_BEFORE_SAVE generations through the device map at
    POPULATION_SIZE 64, then save_checkpoint): the pickle names only DEAP's
    classes and the reference's plain pickle.load, with a DEAP-layout package,
    reads back the same population and hall of fame."""
    import json
    import os
    import subprocess
    import sys

    import ga
    import main
    import utils
    from pong_amd import deap_pickle as D
    from pong_amd.deap_compat import algorithms, tools

    monkeypatch.chdir(tmp_path)
    random.seed(7)
    pop = ga.toolbox.population(n=ga.POPULATION_SIZE)
    hof = tools.HallOfFame(ga.HALL_OF_FAME_AMOUNT)
    saved = main.hall_of_fame
    try:
        main.hall_of_fame = hof
        stats = tools.Statistics(lambda ind: ind.fitness.values)
        stats.register("max", np.max)
        pop, log = algorithms.eaSimple(pop, ga.toolbox, cxpb=ga.CROSSOVER_BLEND_PROBABILITY,
                                       mutpb=ga.GAUSSIAN_MUTATION_PROBABILITY, ngen=ga.GENERATIONS_BEFORE_SAVE,
                                       stats=stats, halloffame=hof, verbose=False)
        path = utils.save_checkpoint(pop, hof)
    finally:
        main.hall_of_fame = saved
    names = D.global_names(open(path, "rb").read())
    assert names <= {"deap.creator.Individual", "deap.creator.Fitness", "deap.tools.support.HallOfFame",
                     "_operator.eq"}, names
    stub = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stub_deap")
    code = ("import sys, json, pickle; sys.path.insert(0, %r)\n"
            "from deap import base, creator\n"
            "creator.create('Fitness', base.Fitness, weights=(1.0,))\n"
            "creator.create('Individual', list, fitness=creator.Fitness)\n"
            "cp = pickle.load(open(%r, 'rb'))\n"
            "print(json.dumps({'genes': [list(i) for i in cp['population']],\n"
            " 'fit': [i.fitness.values[0] for i in cp['population']],\n"
            " 'hof': [i.fitness.values[0] for i in cp['hall_of_fame'].items]}))" % (stub, os.path.abspath(path)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = json.loads(out.stdout.strip().splitlines()[-1])
    assert got["genes"] == [list(i) for i in pop]
    assert got["fit"] == [i.fitness.values[0] for i in pop]
    assert got["hof"] == [i.fitness.values[0] for i in hof.items]


def test_perform_episode_and_get_actions(gpu, oracle):
    """perform_episode (main.py:69-112) on the drop-in: each opponent kind in
    its evaluate() slot equals the oracle's game of the same slot (reward
    bit for bit, the hall-of-fame multiplier included) and evaluate()'s own
    game; get_actions (main.py:138-154) decides as the oracle's forward on the
    x-flipped left view and the right view."""
    import main
    import utils
    from dumb_ais import HardcodedAi, ScoreHardcodedAi
    from numpy_nn import NeuralNetwork
    shape = [6, 64, 3]
    saved = utils.NETWORK_SHAPE
    utils.NETWORK_SHAPE = shape
    try:
        rng = np.random.default_rng(31)
        G = sum((shape[i] + 1) * shape[i + 1] for i in range(len(shape) - 1))
        me, other = rng.standard_normal(G) * 3.0, rng.standard_normal(G) * 3.0
        right = NeuralNetwork(nodes=shape, weights=list(me), bias=True)
        left = NeuralNetwork(nodes=shape, weights=list(other), bias=True)
        cases = [(0, 2, HardcodedAi(), 1.0, 0), (1, 1, HardcodedAi(), 1.0, 1), (2, 2, ScoreHardcodedAi(), 1.0, 2),
                 (4, 2, left, -0.375, 3)]
        for game, players, lm, mult, kind in cases:
            got = main.perform_episode(main.make_env(game, players), lm, right, False, mult)
            ref = oracle.play_game(me, shape, kind, other if kind == 3 else None, mult,
                                   seed=oracle.game_seed(main.PHYSICS_SEED, game))
            assert got == ref["reward"], (game, got, ref)
        # get_actions: [row, column] locations (find_stuff's order), doubled-centroid grid points
        for _ in range(40):
            ball = [float(rng.integers(0, 160)), float(rng.integers(0, 160))]
            last = [float(rng.integers(0, 160)), float(rng.integers(0, 160))]
            lpad, rpad = [float(rng.integers(8, 152)), 17.5], [float(rng.integers(8, 152)), 141.5]
            la, ra = main.get_actions(ball, last, lpad, left, rpad, right)
            # the oracle's forward on the features utils.inference builds (the left view x-flipped)
            W, Hh = utils.GAME_WIDTH, utils.GAME_PLAYABLE_HEIGHT
            for act, net_genes, b, lb, mine, enemy in ((la, other, [ball[0], W - ball[1]], [last[0], W - last[1]],
                                                        lpad, rpad),
                                                       (ra, me, ball, last, rpad, lpad)):
                feats = [b[1] / W, b[0] / Hh, lb[1] / W, lb[0] / Hh, mine[0] / Hh, enemy[0] / Hh]
                idx, _ = oracle.nn_run(net_genes, shape, np.array(feats))
                assert list(act) == ([1, 0] if idx == 0 else [0, 1] if idx == 1 else [0, 0])
        assert main.get_actions(None, None, [80.0, 17.5], left, [80.0, 141.5], right) == ([0, 0], [0, 0])
    finally:
        utils.NETWORK_SHAPE = saved
