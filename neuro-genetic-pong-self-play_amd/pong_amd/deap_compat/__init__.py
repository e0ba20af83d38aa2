# This module restates part of DEAP (Distributed Evolutionary Algorithms in Python,
# https://github.com/DEAP/deap, Copyright (C) the DEAP developers), which is
# distributed under the GNU Lesser General Public License v3 or later.  The call
# order and messages follow DEAP on purpose (a seeded run must draw the same
# random numbers as DEAP would); this file is therefore LGPL-3.0-or-later.
"""DEAP's creator / base / tools / algorithms, restated (deap is not installed
and there is no package index).  Used by ga.py only when ``import deap``
fails.  It follows DEAP's published algorithms (deap 1.3/1.4: eaSimple,
varAnd, cxBlend, mutGaussian, selTournament, selRandom, HallOfFame,
Statistics, Logbook) and draws from Python's ``random`` in the same order, so
a seeded run makes the same calls as DEAP would.  No DEAP file or golden
vector is available offline, so GA parity is UNPINNED (DESIGN.md "GA").
"""
from . import algorithms, base, creator, tools  # noqa: F401
