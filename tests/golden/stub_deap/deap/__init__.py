"""A stand-in with DEAP's module layout, for building and reading checkpoint
fixtures in a container where deap is not installed (test infrastructure;
never imported by the product).  It reproduces what a pickled DEAP object
looks like -- the module path of each class and the instance attributes in
its ``__dict__`` -- not DEAP's algorithms:

* ``deap.creator.create(name, base, **kw)`` makes the class inside
  ``deap.creator`` (so it pickles as ``deap.creator.<name>``); class-valued
  keywords become per-instance attributes, the rest class attributes;
* ``deap.base.Fitness`` stores ``wvalues`` (values x weights) per instance;
* ``deap.tools.support.HallOfFame`` holds ``maxsize``, ``keys`` (fitnesses,
  ascending), ``items`` (individuals, best first) and ``similar``.
"""
