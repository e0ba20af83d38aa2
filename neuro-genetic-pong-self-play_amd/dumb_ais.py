"""Scripted opponents (reference dumb_ais.py:1-25) as host-side models.

On the device these are game kinds (PG_OPP_HARDCODED, PG_OPP_SCORE); the
classes keep the duck-typed ``run(features) -> [up, down]`` API that
perform_episode drives (main.py:78-79, 148-150).
"""


def _chase(features):
    """[up, down] toward the ball: compares ball y (features[1]) with own y (features[4])."""
    ball_y, own_y = features[1], features[4]
    return [int(ball_y < own_y), int(ball_y > own_y)]


class HardcodedAi:
    """Always chases the ball vertically (dumb_ais.py:1-8)."""

    def run(self, input_vector):
        return _chase(input_vector)


class ScoreHardcodedAi:
    """Chases the ball only while the left player (score1) is not ahead
    (dumb_ais.py:11-25).  As in the reference -- whose ``__int__`` typo leaves it
    without a constructor -- ``score_info`` exists once ``set_score`` has run,
    which perform_episode does every frame before ``run``."""

    def set_score(self, score_info):
        self.score_info = score_info

    def run(self, input_vector):
        info = self.score_info
        if info["score1"] > info["score2"]:
            return [0, 0]
        return _chase(input_vector)
