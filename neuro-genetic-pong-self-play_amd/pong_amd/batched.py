"""The batched ``toolbox.map`` (replaces ``futures.map``, ga.py:83).

DEAP's eaSimple calls ``toolbox.map(toolbox.evaluate, invalid_ind)``.  When
the mapped function carries a ``__pong_batch__`` attribute (main.evaluate
does), the whole list goes to that batch function -- one device launch for
all individuals -- and the results come back in input order.  Any other
function is mapped with the builtin ``map``.
"""
from __future__ import annotations

import functools


def _target(func):
    while isinstance(func, functools.partial):
        if func.args or func.keywords:
            return None  # extra bound arguments: not the plain evaluate(individual)
        func = func.func
    return func


def batched_map(func, *iterables):
    target = _target(func)
    batch = getattr(target, "__pong_batch__", None) if target is not None else None
    if batch is not None and len(iterables) == 1:
        return batch(list(iterables[0]))
    return map(func, *iterables)
