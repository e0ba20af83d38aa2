"""The in-repo DEAP restatement (deap is absent offline; GA parity unpinned):
the operator formulas, the random-call order, HallOfFame ordering and the
eaSimple control flow the reference's main() relies on (main.py:157-173)."""
import pickle
import random

import numpy as np
import pytest

from pong_amd.deap_compat import algorithms, base, creator, tools


@pytest.fixture(scope="module")
def types_():
    creator.create("FitT", base.Fitness, weights=(1.0,))
    creator.create("IndT", list, fitness=creator.FitT)
    return creator.FitT, creator.IndT


def test_fitness_and_individual(types_):
    Fit, Ind = types_
    a, b = Ind([1.0, 2.0]), Ind([3.0])
    assert not a.fitness.valid
    a.fitness.values = (0.5,)
    b.fitness.values = (0.25,)
    assert a.fitness.valid and a.fitness > b.fitness and b.fitness < a.fitness
    del a.fitness.values
    assert not a.fitness.valid
    c = pickle.loads(pickle.dumps(b))
    assert c == b and c.fitness.values == (0.25,)


def test_cxblend_formula_and_draw_order():
    random.seed(3)
    x1, x2 = [1.0, -2.0, 0.5], [4.0, 3.0, -1.0]
    a, b = tools.cxBlend(list(x1), list(x2), 0.9)
    random.seed(3)
    for i in range(3):
        g = (1. + 2. * 0.9) * random.random() - 0.9
        assert a[i] == (1. - g) * x1[i] + g * x2[i]
        assert b[i] == g * x1[i] + (1. - g) * x2[i]


def test_mutgaussian_draw_order():
    random.seed(5)
    ind = [0.0] * 50
    tools.mutGaussian(ind, 0, 0.9, 0.9)
    random.seed(5)
    want = [0.0] * 50
    for i in range(50):
        if random.random() < 0.9:
            want[i] += random.gauss(0, 0.9)
    assert ind == want


def test_seltournament_picks_first_best(types_):
    _, Ind = types_
    pop = []
    for v in (1.0, 3.0, 3.0, 2.0):
        ind = Ind([v])
        ind.fitness.values = (v,)
        pop.append(ind)
    random.seed(1)
    got = tools.selTournament(pop, 200, tournsize=3)
    random.seed(1)
    for g in got:
        asp = [random.choice(pop) for _ in range(3)]
        best = asp[0]
        for a in asp[1:]:
            if a.fitness > best.fitness:
                best = a
        assert g is best


def test_hall_of_fame_update(types_):
    _, Ind = types_
    hof = tools.HallOfFame(3)

    def mk(v, genes):
        ind = Ind(genes)
        ind.fitness.values = (v,)
        return ind

    pop = [mk(0.1, [1]), mk(0.5, [2]), mk(0.3, [3]), mk(0.5, [2]), mk(0.9, [4]), mk(0.2, [5])]
    hof.update(pop)
    assert [i.fitness.values[0] for i in hof] == [0.9, 0.5, 0.3]   # best first, duplicate [2] skipped
    assert [k.values[0] for k in hof.keys] == [0.3, 0.5, 0.9]     # keys ascending
    assert hof[0] is not pop[4] and hof[0] == pop[4]              # deep copies
    hof.update([mk(0.4, [6])])
    assert [i.fitness.values[0] for i in hof] == [0.9, 0.5, 0.4]


def test_easimple_flow(types_):
    _, Ind = types_
    tb = base.Toolbox()
    random.seed(0)
    tb.register("attr", random.random)
    tb.register("individual", tools.initRepeat, Ind, tb.attr, n=5)
    tb.register("population", tools.initRepeat, list, tb.individual)
    tb.register("evaluate", lambda ind: (sum(ind),))
    tb.register("mate", tools.cxBlend, alpha=0.9)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.9, indpb=0.9)
    tb.register("select", tools.selTournament, tournsize=4)
    seen = []

    def counting_map(f, xs):
        xs = list(xs)
        seen.append(len(xs))
        return map(f, xs)

    tb.register("map", counting_map)
    pop = tb.population(n=16)
    hof = tools.HallOfFame(4)
    stats = tools.Statistics(lambda ind: ind.fitness.values)
    stats.register("max", np.max)
    pop, log = algorithms.eaSimple(pop, tb, cxpb=0.9, mutpb=0.9, ngen=3, stats=stats, halloffame=hof, verbose=False)
    assert seen[0] == 16 and len(seen) == 4 and len(log) == 4
    assert all(ind.fitness.valid for ind in pop)
    assert hof[0].fitness.values[0] >= max(ind.fitness.values[0] for ind in pop)
    assert log.select("gen") == [0, 1, 2, 3]
