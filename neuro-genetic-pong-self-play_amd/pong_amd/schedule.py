"""Host side of evaluate() (main.py:28-66): which opponent each game faces.

The reference plays GAMES_TO_PLAY games per individual: game 0 against
HardcodedAi, game 1 against the 1-player ROM opponent, game 2 against
ScoreHardcodedAi, and every later game against a hall-of-fame member picked by
create_model_from_hall_of_fame (utils.py:90-101: shuffle in place, first
valid member; its fitness becomes right_score_multiplier).  This module makes
those picks for a whole batch, in the order a sequential ``map(evaluate, ...)``
would, so the ``random`` stream and the in-place shuffles match.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L


def reference_schedule(n: int, games: int, hall_of_fame, pick):
    """Returns (kind [n, games] int32, opp [n, games] int32, mult [n, games] f64,
    opponents: list of distinct hall-of-fame members indexed by ``opp``).

    ``pick(hall_of_fame) -> (member or None, multiplier)`` is
    utils.pick_hall_of_famer.  ``hall_of_fame`` None means no hall of fame
    (main.py:44-45): HardcodedAi with multiplier 1.
    """
    kind = np.empty((n, games), dtype=np.int32)
    opp = np.zeros((n, games), dtype=np.int32)
    mult = np.ones((n, games), dtype=np.float64)
    members, rows = [], {}
    fixed = (L.PG_OPP_HARDCODED, L.PG_OPP_ROM_CPU, L.PG_OPP_SCORE)
    for r in range(n):
        multiplier = 1  # right_score_multiplier, main.py:32 (carried across games)
        for g in range(games):
            k = fixed[g] if g < len(fixed) else L.PG_OPP_HARDCODED
            if g >= len(fixed) and hall_of_fame is not None:
                member, multiplier = pick(hall_of_fame)
                if member is not None:
                    k = L.PG_OPP_NN
                    key = id(member)
                    if key not in rows:
                        rows[key] = len(members)
                        members.append(member)
                    opp[r, g] = rows[key]
            kind[r, g] = k
            mult[r, g] = multiplier
    return kind, opp, mult, members
