"""Host helpers of the reference's utils.py (utils.py:71-153) around the device path.

Per-frame helpers (bounds clamp, features, reward) run inside the HIP kernel;
the versions here are the host API for callers that drive single games or
build schedules.  ``pick_hall_of_famer`` makes exactly the ``random`` calls of
create_model_from_hall_of_fame (utils.py:90-101) so a batched evaluation
draws the same opponents as a sequential map of evaluate() would.
"""
import datetime
import os
import random
from copy import deepcopy

import numpy as np

from config import *  # noqa: F401,F403  (NETWORK_SHAPE etc., as the reference's utils.py:9)
from config import GAME_PLAYABLE_HEIGHT, GAME_WIDTH, SCALED_PADDLE_HEIGHT, TIME_SCALER
from numpy_nn import NeuralNetwork
from pong_amd import deap_pickle


def find_stuff(observation):
    """find_stuff (utils.py:14-19): the (row, col) centroids of the ball, left and
    right paddle colours in a 210x160x3 frame, each None when absent -- computed
    by pg_find_stuff on the device (per-channel matching as get_rect_quickly,
    utils.py:60-68).  Returns a [3, 2] float array when all three are present,
    else numpy < 1.24's object array of three entries."""
    import torch
    from pong_amd import device as _device
    dev = torch.device(DEVICE)  # noqa: F405
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if isinstance(observation, torch.Tensor):  # a DeviceEnv frame: already on the device
        frame = observation.to(device=dev, dtype=torch.uint8).contiguous()
    else:
        frame = torch.as_tensor(np.ascontiguousarray(observation, dtype=np.uint8), device=dev)
    got = _device.find_stuff(frame)[0].cpu().numpy()
    if not np.isnan(got).any():
        return got
    out = np.empty(3, dtype=object)
    out[:] = [None if np.isnan(v).any() else v for v in got]
    return out


def keep_within_game_bounds_please(paddle, action):
    """Force a paddle whose centroid row is within 16 px of a wall back toward
    the middle (utils.py:71-77); ``paddle`` is a (row, col) centroid or None."""
    if paddle is None:
        return action
    row = paddle[0]
    if row < SCALED_PADDLE_HEIGHT:
        return [0, 1]
    if row > GAME_PLAYABLE_HEIGHT - SCALED_PADDLE_HEIGHT:
        return [1, 0]
    return action


def create_model_from_genes(individual):
    return NeuralNetwork(nodes=NETWORK_SHAPE, weights=individual, bias=BIAS)  # noqa: F405


def pick_hall_of_famer(hall_of_fame):
    """(member, score multiplier) of create_model_from_hall_of_fame: shuffle the
    hall of fame's items IN PLACE (utils.py:95, as the reference does) and take
    the first member with a valid fitness; (None, 1) if there is none."""
    members = hall_of_fame.items
    if len(members) == 0:
        return None, 1
    random.shuffle(members)
    for member in members:
        if member.fitness.valid:
            return member, member.fitness.values[0]
    return None, 1


def create_model_from_hall_of_fame(hall_of_fame):
    member, multiplier = pick_hall_of_famer(hall_of_fame)
    model = None if member is None else create_model_from_genes(list(member))
    return model, multiplier


def calculate_reward(score_multiplier, total_time, my_score, enemy_score):
    """((my - enemy) + my * multiplier) / (frames / TIME_SCALER) (utils.py:104-109)."""
    return ((my_score - enemy_score) + my_score * score_multiplier) / (total_time / TIME_SCALER)


def get_random_action(all_actions):
    return all_actions[np.random.choice(all_actions.shape[0], size=None, replace=False), :]


def save_checkpoint(_population, hall_of_fame):
    """Pickle {population, hall_of_fame, rndstate, network_shape} to
    checkpoints/checkpoints/c_HH_MM_SS.pkl (utils.py:116-125 format) and
    return the path.  The pickle names DEAP's class paths
    (``deap.creator.Individual``, ``deap.creator.Fitness``,
    ``deap.tools.support.HallOfFame``) even when the in-repo restatement made
    the objects, so the reference's ``ga.load_population_from_file``
    (ga.py:41-45, plain ``pickle.load`` with real DEAP) resumes from it."""
    payload = {
        "population": _population,
        "hall_of_fame": deepcopy(hall_of_fame),
        "rndstate": random.getstate(),
        "network_shape": NETWORK_SHAPE,  # noqa: F405
    }
    os.makedirs("checkpoints/checkpoints", exist_ok=True)
    stamp = datetime.datetime.now().strftime("%H_%M_%S")
    path = os.path.join("checkpoints", "checkpoints", f"c_{stamp}.pkl")
    with open(path, "wb") as fh:
        deap_pickle.dump(payload, fh)
    return path


def calculate_gene_size():
    """Genes of NETWORK_SHAPE: sum over layers of (inputs + bias) * outputs (utils.py:128-136)."""
    shape = NETWORK_SHAPE  # noqa: F405
    extra = 1 if BIAS else 0  # noqa: F405
    return sum((shape[i] + extra) * shape[i + 1] for i in range(len(shape) - 1))


def inference(ball_location, last_ball_location, me, enemy, model):
    """Normalised [ball x, ball y, last x, last y, me y, enemy y] -> model.run (utils.py:139-153)."""
    features = [
        ball_location[1] / GAME_WIDTH,
        ball_location[0] / GAME_PLAYABLE_HEIGHT,
        last_ball_location[1] / GAME_WIDTH,
        last_ball_location[0] / GAME_PLAYABLE_HEIGHT,
        me[0] / GAME_PLAYABLE_HEIGHT,
        enemy[0] / GAME_PLAYABLE_HEIGHT,
    ]
    return model.run(features)
