"""deap.base layout stand-in: Fitness keeps ``wvalues`` in the instance dict."""


class Fitness(object):
    weights = None
    wvalues = ()

    def __init__(self, values=()):
        if len(values) > 0:
            self.values = values

    @property
    def values(self):
        return tuple(w / k for w, k in zip(self.wvalues, self.weights))

    @values.setter
    def values(self, values):
        self.wvalues = tuple(v * k for v, k in zip(values, self.weights))

    @values.deleter
    def values(self):
        self.wvalues = ()

    @property
    def valid(self):
        return len(self.wvalues) != 0

    def __lt__(self, other):
        return self.wvalues < other.wvalues

    def __le__(self, other):
        return self.wvalues <= other.wvalues

    def __eq__(self, other):
        return self.wvalues == other.wvalues

    __hash__ = object.__hash__


class Toolbox(object):
    pass
