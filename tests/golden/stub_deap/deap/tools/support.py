"""deap.tools.support layout stand-in: HallOfFame's pickled attributes."""
from bisect import bisect_right
from copy import deepcopy
from operator import eq


class HallOfFame(object):
    def __init__(self, maxsize, similar=eq):
        self.maxsize = maxsize
        self.keys = list()
        self.items = list()
        self.similar = similar

    def insert(self, item):
        item = deepcopy(item)
        i = bisect_right(self.keys, item.fitness)
        self.items.insert(len(self) - i, item)
        self.keys.insert(i, item.fitness)

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]
