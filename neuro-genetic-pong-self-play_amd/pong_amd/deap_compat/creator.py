# This module restates part of DEAP (Distributed Evolutionary Algorithms in Python,
# https://github.com/DEAP/deap, Copyright (C) the DEAP developers), which is
# distributed under the GNU Lesser General Public License v3 or later.  The call
# order and messages follow DEAP on purpose (a seeded run must draw the same
# random numbers as DEAP would); this file is therefore LGPL-3.0-or-later.
"""deap.creator restated: ``create(name, base, **attrs)`` makes a class in
this module's namespace (so instances pickle), e.g. ga.py:80-81."""
import warnings


def create(name, base, **kargs):
    if name in globals():
        warnings.warn("A class named '{0}' has already been created and it will be overwritten. "
                      "Consider deleting previous creation of that class or rename it.".format(name),
                      RuntimeWarning)
    dict_inst = {}
    dict_cls = {}
    for obj_name, obj in kargs.items():
        if isinstance(obj, type):
            dict_inst[obj_name] = obj
        else:
            dict_cls[obj_name] = obj

    def initType(self, *args, **kargs):
        """Instance attributes given as classes are instantiated per object."""
        for obj_name, obj in dict_inst.items():
            setattr(self, obj_name, obj())
        if base.__init__ is not object.__init__:
            base.__init__(self, *args, **kargs)

    objtype = type(str(name), (base,), dict_cls)
    objtype.__init__ = initType
    objtype.__module__ = __name__
    globals()[name] = objtype
