"""The reference's per-frame numpy loop, restated -- the CPU baseline of bench.py.

TEST INFRASTRUCTURE ONLY (like everything under ``oracle/``): only
``bench.py``'s ``cpu_baseline`` leg, ``tests/`` and the calibration script
``tools/cpu_calibrate.py`` use it, as the timed CPU path that the reference
itself runs.  The product never imports it.

What it restates, operation for operation, per frame (the reference's hot
loop, one ``evaluate()`` per genome):

* ``evaluate``          /root/reference/main.py:28-66   (6 games, ``sum / 6.0``)
* ``perform_episode``   /root/reference/main.py:69-112
* ``get_actions``       /root/reference/main.py:138-154 (two
  ``get_random_action`` draws per frame, utils.py:112-113, as the reference)
* ``find_stuff``        /root/reference/utils.py:14-19 with
  ``get_rect_quickly``  utils.py:59-66 (``np.argwhere`` of the per-channel
  colour match, ``np.average`` of its row/column indices)
* ``keep_within_game_bounds_please`` utils.py:70-76,
  ``calculate_timeout_and_frames`` main.py:128-135,
  ``calculate_reward`` utils.py:104-109, ``inference`` utils.py:139-153
* ``NeuralNetwork.run`` /root/reference/numpy_nn.py:120-137 (``np.dot`` of
  each weight matrix with the bias-extended activation vector, the sigmoid
  ``1 / (1 + np.e ** -x)`` of numpy_nn.py:22-23, first-index argmax), weights
  laid out by ``populate_weights`` numpy_nn.py:52-69
* ``HardcodedAi`` / ``ScoreHardcodedAi`` /root/reference/dumb_ais.py

The emulator (gym-retro, absent) is the build's physics (``or_env_step``) and
its frame is ``or_render`` -- both C, as the emulator's step and frame are.
Everything the reference does in Python/numpy per frame is done here in
Python/numpy, so the timing stands for the reference's own CPU path.
``tools/cpu_calibrate.py`` runs the real reference code (imported in the
build container) on the same games and checks that rewards and fitness agree
and that the per-frame rates match (profiles/r02/cpu_calibration.json).
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle as O  # noqa: E402

# config.py constants (/root/reference/config.py:3-54)
BALL_COLOUR = (236, 236, 236)
LEFT_GUY_COLOUR = (213, 130, 74)
RIGHT_GUY_COLOUR = (92, 186, 92)
GAME_BOTTOM, GAME_TOP = 194, 34
SCALED_PADDLE_HEIGHT = 16.0
GAME_PLAYABLE_HEIGHT = GAME_BOTTOM - GAME_TOP
GAME_WIDTH = 160
RIGHT_ACTION_START, RIGHT_ACTION_END, LEFT_ACTION_END = 4, 6, 8
TIMEOUT_THRESH = 2000
WIN_SCORE = 3
TIME_SCALER = 100.0
GAMES_TO_PLAY = 6
ALL_ACTIONS = np.eye(2, dtype=int)


def _blank_action():
    a = np.zeros(16, dtype=int)
    a[-1] = 1
    a[0] = 1
    return a


def _sigmoid(x):
    return 1 / (1 + np.e ** -x)


class NumpyNet:
    """numpy_nn.NeuralNetwork(nodes, bias=True, weights=genes).run, restated."""

    def __init__(self, nodes, genes):
        self.weights = []
        idx = 0
        for i in range(len(nodes) - 1):
            n = (nodes[i] + 1) * nodes[i + 1]
            self.weights.append(np.array(genes[idx:idx + n]).reshape(nodes[i + 1], nodes[i] + 1))
            idx += n
        self.acts = [np.ones(n + 1) for n in nodes]

    def run(self, x):
        a = self.acts
        a[0][:len(x)] = x
        for i, w in enumerate(self.weights):
            a[i + 1][:-1] = np.dot(w, a[i])
            a[i + 1][:-1] = _sigmoid(a[i + 1][:-1])
        inx = np.argmax(np.squeeze(a[-1][:-1]))
        if inx == 0:
            return [1, 0]
        if inx == 1:
            return [0, 1]
        return [0, 0]  # index 2: the build's no-op extension (the reference raises)


class Hardcoded:
    def run(self, v):
        r = [0, 0]
        if v[1] < v[4]:
            r[0] = 1
        elif v[1] > v[4]:
            r[1] = 1
        return r


class ScoreHardcoded(Hardcoded):
    score_info = None

    def run(self, v):
        if self.score_info["score1"] <= self.score_info["score2"]:
            return Hardcoded.run(self, v)
        return [0, 0]


def _rect(chopped, colour):
    value = np.average(np.argwhere(chopped == colour)[:, :-1], axis=0)
    if np.isnan(value).any():
        return None
    return value


def find_stuff(frame):
    c = frame[GAME_TOP:GAME_BOTTOM, :]
    return _rect(c, BALL_COLOUR), _rect(c, LEFT_GUY_COLOUR), _rect(c, RIGHT_GUY_COLOUR)


def _inference(ball, last, me, enemy, model):
    return model.run([ball[1] / GAME_WIDTH, ball[0] / GAME_PLAYABLE_HEIGHT,
                      last[1] / GAME_WIDTH, last[0] / GAME_PLAYABLE_HEIGHT,
                      me[0] / GAME_PLAYABLE_HEIGHT, enemy[0] / GAME_PLAYABLE_HEIGHT])


def _random_action():
    return ALL_ACTIONS[np.random.choice(ALL_ACTIONS.shape[0], size=None, replace=False), :]


def _get_actions(ball, last_ball, left, left_model, right, right_model):
    left_action = _random_action()
    right_action = _random_action()
    if last_ball is None:
        last_ball = ball
    if ball is not None:
        if left is not None:
            left_action = _inference([ball[0], GAME_WIDTH - ball[1]], [last_ball[0], GAME_WIDTH - last_ball[1]],
                                     left, right, left_model)
        if right is not None:
            right_action = _inference(ball, last_ball, right, left, right_model)
    else:
        left_action = [0, 0]
        right_action = [0, 0]
    return left_action, right_action


def _clamp(paddle, action):
    if paddle is not None:
        if paddle[0] < SCALED_PADDLE_HEIGHT:
            action = [0, 1]
        elif paddle[0] > ((GAME_BOTTOM - GAME_TOP) - SCALED_PADDLE_HEIGHT):
            action = [1, 0]
    return action


class _Env:
    """The emulator stand-in: oracle physics + oracle frame (both C)."""

    def __init__(self, seed, one_player):
        self.state = O.OrState()
        self.seed, self.one_player = seed, int(one_player)
        self.frame = np.zeros((210, 160, 3), dtype=np.uint8)
        self._fp = self.frame.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        self.L = O.lib()
        self.reset()

    def reset(self):
        self.L.or_env_reset(ctypes.byref(self.state), self.seed, self.one_player)

    def step(self, action):
        s = self.state
        self.L.or_env_step(ctypes.byref(s), int(action[4]), int(action[5]), int(action[6]), int(action[7]))
        self.L.or_render(ctypes.byref(s), self._fp)
        return self.frame, 0.0, bool(self.L.or_env_done(ctypes.byref(s))), {"score1": s.score1, "score2": s.score2}


def perform_episode(env, left_model, right_model, score_multiplier, timeout_thresh=None, win_score=None):
    """main.py:69-112.  Returns (reward, frames, score1, score2, total_frames).
    ``timeout_thresh`` / ``win_score``: config.py's TIMEOUT_THRESH / WIN_SCORE
    (None: the reference's 2000 / 3)."""
    thresh = TIMEOUT_THRESH if not timeout_thresh else timeout_thresh
    win = WIN_SCORE if not win_score else win_score
    last_score = None
    action = _blank_action()
    timeout_counter = 0.0
    total_frames = 0.0
    last_ball = None
    frames = 0
    while True:
        observation, _r, is_done, score_info = env.step(action)
        frames += 1
        if isinstance(left_model, ScoreHardcoded):
            left_model.score_info = score_info
        ball, left, right = find_stuff(observation)
        left_action, right_action = _get_actions(ball, last_ball, left, left_model, right, right_model)
        last_ball = ball
        action[RIGHT_ACTION_START:RIGHT_ACTION_END] = _clamp(right, right_action)
        action[RIGHT_ACTION_END:LEFT_ACTION_END] = _clamp(left, left_action)
        if last_score is not None:
            if last_score == score_info:
                timeout_counter += 1.0
            else:
                total_frames += timeout_counter
                timeout_counter = 0.0
        last_score = score_info
        if score_info["score1"] >= win or score_info["score2"] >= win:
            break
        if is_done:
            break
        if timeout_counter > thresh:
            break
    s1, s2 = score_info["score1"], score_info["score2"]
    if s1 == s2:
        return 0, frames, s1, s2, total_frames
    diff = s2 - s1
    reward = (diff + s2 * score_multiplier) / (total_frames / TIME_SCALER)
    return reward, frames, s1, s2, total_frames


def evaluate(nodes, genes, kinds, opp_rows, mults, opponents, base_seed=0, timeout_thresh=None, win_score=None):
    """main.py:28-66 for one genome with a fixed game schedule (kind 0 HardcodedAi,
    1 ROM CPU, 2 ScoreHardcodedAi, 3 network opponent ``opponents[opp_rows[g]]``
    with ``right_score_multiplier = mults[g]``).  Returns (fitness, rewards, frames)."""
    right = NumpyNet(nodes, genes)
    rewards, frames = [], 0
    for g in range(len(kinds)):
        k = int(kinds[g])
        left = (NumpyNet(nodes, opponents[int(opp_rows[g])]) if k == 3
                else ScoreHardcoded() if k == 2 else Hardcoded())
        env = _Env(O.game_seed(base_seed, g), k == 1)
        rew, f, _s1, _s2, _tf = perform_episode(env, left, right, float(mults[g]) if k == 3 else 1.0,
                                                timeout_thresh, win_score)
        rewards.append(rew)
        frames += f
    return sum(rewards) / float(GAMES_TO_PLAY), rewards, frames


def _worker(job):
    """One BLAS thread per worker: the pool is the parallelism (as SCOOP's
    worker processes are); an OpenBLAS pool per process would oversubscribe
    the cores (16 processes x OMP_NUM_THREADS threads on the GPU box).
    find_stuff's np.average of an absent colour warns "Mean of empty slice"
    on every hidden-ball frame, as the reference's does; the workers do not
    print it (the returned None is the reference's behaviour either way)."""
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        try:
            from threadpoolctl import threadpool_limits
        except ImportError:  # timing helper: run as is without it
            return _games(job)
        with threadpool_limits(1):
            return _games(job)


def _games(job):
    """Whole games until ``seconds`` of this worker's own time have passed
    (its clock starts when it has its job: shipping the job's genomes to a
    process is not the reference's per-frame work).  Returns (env-steps,
    games, busy seconds)."""
    nodes, genomes, kinds, opps, mults, opponents, seconds, seed = job
    np.random.seed(seed)
    t0 = time.perf_counter()
    deadline = t0 + seconds
    steps, games = 0, 0
    for i in range(genomes.shape[0]):
        right = NumpyNet(nodes, genomes[i])
        for g in range(len(kinds[i])):
            if time.perf_counter() >= deadline:
                return steps, games, time.perf_counter() - t0
            k = int(kinds[i][g])
            left = (NumpyNet(nodes, opponents[int(opps[i][g])]) if k == 3
                    else ScoreHardcoded() if k == 2 else Hardcoded())
            _rew, f, _s1, _s2, _tf = perform_episode(_Env(O.game_seed(0, g), k == 1), left, right,
                                                     float(mults[i][g]) if k == 3 else 1.0)
            steps += f
            games += 1
    return steps, games, time.perf_counter() - t0


def make_pool(workers):
    """A fork pool of idle workers.  Create it BEFORE the process touches the GPU
    (bench.py does): forked children then hold no GPU state."""
    import multiprocessing as mp
    return mp.get_context("fork").Pool(workers)


def _jobs(nodes, genomes, kinds, opps, mults, opponents, seconds, workers):
    jobs = []
    for w in range(workers):  # each worker gets only the opponent rows its games use
        ow = np.asarray(opps[w::workers])
        rows = np.unique(ow)
        jobs.append((nodes, genomes[w::workers], kinds[w::workers], np.searchsorted(rows, ow).astype(np.int32),
                     mults[w::workers], opponents[rows], seconds, w))
    return jobs


def timed_rate(nodes, genomes, kinds, opps, mults, opponents, seconds, workers=1, pool=None, solo_seconds=None):
    """env-steps/s of whole games (evaluate()'s perform_episode calls, in order)
    over ``seconds`` of each worker's time, genomes dealt round-robin to
    ``workers`` processes (as SCOOP's futures.map spreads evaluate() over
    cores, ga.py:83), all running at once: the rate is the sum of the workers'
    own rates (env-steps / busy seconds).  Returns (rate, env-steps, games,
    the longest worker's busy seconds).

    ``solo_seconds``: also run worker 0's job ALONE afterwards (one process,
    the same games from the start, nothing else running) -- the one-core
    figure on the same sample as the pooled one; then returns a 5th element
    (solo rate, solo env-steps, solo games, solo seconds, worker 0's pooled
    rate)."""
    jobs = _jobs(nodes, genomes, kinds, opps, mults, opponents, seconds, max(workers, 1))
    own = None
    if pool is None:
        own = pool = make_pool(max(workers, 1))
    try:
        res = pool.map(_worker, jobs)
        solo = None
        if solo_seconds is not None:
            j0 = jobs[0][:6] + (solo_seconds, 0)
            s_steps, s_games, s_dt = pool.apply(_worker, (j0,))
            solo = ((s_steps / s_dt if s_dt > 0 else 0.0), s_steps, s_games, s_dt,
                    (res[0][0] / res[0][2] if res[0][2] > 0 else 0.0))
    finally:
        if own is not None:
            own.close()
    steps = sum(r[0] for r in res)
    games = sum(r[1] for r in res)
    rate = sum(r[0] / r[2] for r in res if r[2] > 0)
    out = (rate, steps, games, max(r[2] for r in res))
    return out + (solo,) if solo_seconds is not None else out
