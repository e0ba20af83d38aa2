# This module restates part of DEAP (Distributed Evolutionary Algorithms in Python,
# https://github.com/DEAP/deap, Copyright (C) the DEAP developers), which is
# distributed under the GNU Lesser General Public License v3 or later.  The call
# order and messages follow DEAP on purpose (a seeded run must draw the same
# random numbers as DEAP would); this file is therefore LGPL-3.0-or-later.
"""deap.tools restated: the operators ga.py registers (ga.py:85-94) and the
HallOfFame / Statistics / Logbook that main.py uses (main.py:158-170)."""
import random
from bisect import bisect_right
from collections import defaultdict
from collections.abc import Sequence
from copy import deepcopy
from functools import partial
from itertools import repeat
from operator import attrgetter, eq


def initRepeat(container, func, n):
    return container(func() for _ in range(n))


def initIterate(container, generator):
    return container(generator())


def initCycle(container, seq_func, n=1):
    return container(func() for _ in range(n) for func in seq_func)


def cxBlend(ind1, ind2, alpha):
    """Blend crossover: gamma = (1 + 2 alpha) U - alpha per gene."""
    for i, (x1, x2) in enumerate(zip(ind1, ind2)):
        gamma = (1. + 2. * alpha) * random.random() - alpha
        ind1[i] = (1. - gamma) * x1 + gamma * x2
        ind2[i] = gamma * x1 + (1. - gamma) * x2
    return ind1, ind2


def mutGaussian(individual, mu, sigma, indpb):
    """Adds N(mu, sigma) to each gene with probability indpb."""
    size = len(individual)
    if not isinstance(mu, Sequence):
        mu = repeat(mu, size)
    elif len(mu) < size:
        raise IndexError("mu must be at least the size of individual: %d < %d" % (len(mu), size))
    if not isinstance(sigma, Sequence):
        sigma = repeat(sigma, size)
    elif len(sigma) < size:
        raise IndexError("sigma must be at least the size of individual: %d < %d" % (len(sigma), size))
    for i, m, s in zip(range(size), mu, sigma):
        if random.random() < indpb:
            individual[i] += random.gauss(m, s)
    return individual,


def selRandom(individuals, k):
    return [random.choice(individuals) for i in range(k)]


def selBest(individuals, k, fit_attr="fitness"):
    return sorted(individuals, key=attrgetter(fit_attr), reverse=True)[:k]


def selWorst(individuals, k, fit_attr="fitness"):
    return sorted(individuals, key=attrgetter(fit_attr))[:k]


def selTournament(individuals, k, tournsize, fit_attr="fitness"):
    """k tournaments of tournsize aspirants drawn with replacement; the first best wins."""
    chosen = []
    for i in range(k):
        aspirants = selRandom(individuals, tournsize)
        chosen.append(max(aspirants, key=attrgetter(fit_attr)))
    return chosen


class HallOfFame(object):
    """The best individuals ever seen, best first (``items``), with their
    fitnesses kept sorted ascending in ``keys``."""

    def __init__(self, maxsize, similar=eq):
        self.maxsize = maxsize
        self.keys = list()
        self.items = list()
        self.similar = similar

    def update(self, population):
        for ind in population:
            if len(self) == 0 and self.maxsize != 0:
                # an empty hall of fame takes population[0] (DEAP's for-else workaround)
                self.insert(population[0])
                continue
            if ind.fitness > self[-1].fitness or len(self) < self.maxsize:
                for hofer in self:
                    if self.similar(ind, hofer):
                        break
                else:
                    if len(self) >= self.maxsize:
                        self.remove(-1)
                    self.insert(ind)

    def insert(self, item):
        item = deepcopy(item)
        i = bisect_right(self.keys, item.fitness)
        self.items.insert(len(self) - i, item)
        self.keys.insert(i, item.fitness)

    def remove(self, index):
        del self.keys[len(self) - (index % len(self) + 1)]
        del self.items[index]

    def clear(self):
        del self.items[:]
        del self.keys[:]

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]

    def __iter__(self):
        return iter(self.items)

    def __reversed__(self):
        return reversed(self.items)

    def __str__(self):
        return str(self.items)


def identity(obj):
    return obj


class Statistics(object):
    def __init__(self, key=identity):
        self.key = key
        self.functions = dict()
        self.fields = []

    def register(self, name, function, *args, **kargs):
        self.functions[name] = partial(function, *args, **kargs)
        self.fields.append(name)

    def compile(self, data):
        values = tuple(self.key(elem) for elem in data)
        entry = dict()
        for key, func in self.functions.items():
            entry[key] = func(values)
        return entry


class Logbook(list):
    """Chronological records; ``stream`` renders the rows not yet streamed."""

    def __init__(self):
        super().__init__()
        self.buffindex = 0
        self.chapters = defaultdict(Logbook)
        self.columns_len = None
        self.header = None
        self.log_header = True

    def record(self, **infos):
        self.append(infos)

    def select(self, *names):
        if len(names) == 1:
            return [entry.get(names[0], None) for entry in self]
        return tuple([entry.get(name, None) for entry in self] for name in names)

    @property
    def stream(self):
        startindex, self.buffindex = self.buffindex, len(self)
        return self.__str__(startindex)

    def __txt__(self, startindex):
        columns = self.header or (sorted(self[0].keys()) if self else [])
        rows = [[str(entry.get(c, "")) for c in columns] for entry in self[startindex:]]
        if self.columns_len is None or len(self.columns_len) != len(columns):
            self.columns_len = [len(c) for c in columns]
        for row in rows:
            self.columns_len = [max(a, len(b)) for a, b in zip(self.columns_len, row)]
        lines = []
        if startindex == 0 and self.log_header:
            lines.append("\t".join(c.ljust(w) for c, w in zip(columns, self.columns_len)))
        for row in rows:
            lines.append("\t".join(v.ljust(w) for v, w in zip(row, self.columns_len)))
        return lines

    def __str__(self, startindex=0):
        return "\n".join(self.__txt__(startindex))
