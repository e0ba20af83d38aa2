# This module restates part of DEAP (Distributed Evolutionary Algorithms in Python,
# https://github.com/DEAP/deap, Copyright (C) the DEAP developers), which is
# distributed under the GNU Lesser General Public License v3 or later.  The call
# order and messages follow DEAP on purpose (a seeded run must draw the same
# random numbers as DEAP would); this file is therefore LGPL-3.0-or-later.
"""deap.base restated: Toolbox and Fitness (used at ga.py:77,80)."""
from collections.abc import Sequence
from copy import deepcopy
from functools import partial
from operator import mul, truediv


class Toolbox(object):
    """Registry of partial functions; ``clone`` = deepcopy and ``map`` = builtin map by default."""

    def __init__(self):
        self.register("clone", deepcopy)
        self.register("map", map)

    def register(self, alias, function, *args, **kargs):
        pfunc = partial(function, *args, **kargs)
        pfunc.__name__ = alias
        pfunc.__doc__ = function.__doc__
        if hasattr(function, "__dict__") and not isinstance(function, type):
            pfunc.__dict__.update(function.__dict__.copy())
        setattr(self, alias, pfunc)

    def unregister(self, alias):
        delattr(self, alias)

    def decorate(self, alias, *decorators):
        pfunc = getattr(self, alias)
        function, args, kargs = pfunc.func, pfunc.args, pfunc.keywords
        for decorator in decorators:
            function = decorator(function)
        self.register(alias, function, *args, **kargs)


class Fitness(object):
    """Weighted, lexicographically compared fitness values (weights set by creator.create)."""

    weights = None
    wvalues = ()

    def __init__(self, values=()):
        if self.weights is None:
            raise TypeError("Can't instantiate abstract %r with abstract attribute weights." % (self.__class__))
        if not isinstance(self.weights, Sequence):
            raise TypeError("Attribute weights of %r must be a sequence." % self.__class__)
        if len(values) > 0:
            self.values = values

    def getValues(self):
        return tuple(map(truediv, self.wvalues, self.weights))

    def setValues(self, values):
        assert len(values) == len(self.weights), "Assigned values have not the same length than fitness weights"
        try:
            self.wvalues = tuple(map(mul, values, self.weights))
        except TypeError as e:
            raise TypeError("Both weights and assigned values must be a sequence of numbers when assigning "
                            "to values of %r. Currently assigning value(s) %r of %r to a fitness with weights %s."
                            % (self.__class__, values, type(values), self.weights)) from e

    def delValues(self):
        self.wvalues = ()

    values = property(getValues, setValues, delValues)

    def dominates(self, other, obj=slice(None)):
        not_equal = False
        for self_wvalue, other_wvalue in zip(self.wvalues[obj], other.wvalues[obj]):
            if self_wvalue > other_wvalue:
                not_equal = True
            elif self_wvalue < other_wvalue:
                return False
        return not_equal

    @property
    def valid(self):
        return len(self.wvalues) != 0

    def __hash__(self):
        return hash(self.wvalues)

    def __gt__(self, other):
        return not self.__le__(other)

    def __ge__(self, other):
        return not self.__lt__(other)

    def __le__(self, other):
        return self.wvalues <= other.wvalues

    def __lt__(self, other):
        return self.wvalues < other.wvalues

    def __eq__(self, other):
        return self.wvalues == other.wvalues

    def __ne__(self, other):
        return not self.__eq__(other)

    def __deepcopy__(self, memo):
        copy_ = self.__class__()
        copy_.wvalues = self.wvalues
        return copy_

    def __str__(self):
        return str(self.values if self.valid else tuple())

    def __repr__(self):
        return "%s.%s(%r)" % (self.__module__, self.__class__.__name__, self.values if self.valid else tuple())
