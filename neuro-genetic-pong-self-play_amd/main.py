"""The reference's main.py surface (main.py:28-185) on the MI355X path.

``evaluate(individual)`` keeps its signature and meaning (average reward of
GAMES_TO_PLAY games, as a 1-tuple); ``evaluate_population(individuals)`` is
the same computation for a whole batch in one device launch
(pg_eval_population), and ``toolbox.map`` routes eaSimple's
``map(evaluate, invalid_ind)`` there.  ``main()`` is the reference's endless
eaSimple + checkpoint loop.  ``perform_episode(env, left_model, right_model,
render, score_multiplier)`` plays one game in one launch on a ``DeviceEnv``
(``make_env``) when both models are device game kinds, and frame by frame
(``perform_episode_stepwise``: the reference's own loop over ``env.step``,
``find_stuff``, ``get_actions``) for any other model with ``run`` -- e.g. the
``HumanInput`` of ``run_against_human`` (main.py:17-25), whose keys may come
from a script instead of a keyboard.  There is no viewer window: ``render``
writes GIFs under REPLAY_DIR.
"""
import numpy as np
import torch

try:
    from deap import algorithms, tools
except ImportError:
    from pong_amd.deap_compat import algorithms, tools

import ga
import utils
from config import *  # noqa: F401,F403
from ga import hall_of_fame, toolbox
from pong_amd import _lib as L
from pong_amd import runtime, schedule
from utils import pick_hall_of_famer, save_checkpoint


def _evaluator():
    # the network shape is utils' binding, as create_model_from_genes sees it (utils.py:80-87)
    return runtime.evaluator(utils.NETWORK_SHAPE, utils.BIAS, GAMES_TO_PLAY, GENOME_DTYPE,  # noqa: F405
                             PRECISION, PHYSICS_SEED, DEVICE, TIMEOUT_THRESH, WIN_SCORE)  # noqa: F405


def _fitness_tuples(fitness, status):
    for f, failed in zip(fitness, status):
        if failed:  # calculate_reward with total_frames == 0 (utils.py:106-108)
            raise ZeroDivisionError("float division by zero")
        yield (float(f),)


def evaluate_population(individuals):
    """evaluate() for every individual, in order; returns an iterator of 1-tuples.

    Hall-of-fame picks are drawn up front in the order a sequential map would
    draw them; an individual whose evaluation would raise ZeroDivisionError
    raises it when its result is reached, as a lazy map does.
    """
    individuals = list(individuals)
    n = len(individuals)
    if n == 0:
        return iter(())
    ev = _evaluator()
    genes = utils.calculate_gene_size()
    kind, opp, mult, members = schedule.reference_schedule(n, GAMES_TO_PLAY, hall_of_fame,  # noqa: F405
                                                           pick_hall_of_famer)
    dev = ev.device
    genomes = runtime.genomes_to_device(individuals, genes, ev)
    opponents = runtime.genomes_to_device(members, genes, ev) if members else None
    res, _ = ev.evaluate(genomes, torch.from_numpy(kind).to(dev), torch.from_numpy(opp).to(dev),
                         torch.from_numpy(mult).to(dev), opponents=opponents)
    return _fitness_tuples(res.fitness.cpu().numpy(), res.status.cpu().numpy())


def evaluate(individual=None, render=RENDER):  # noqa: F405
    """Average reward of the individual's GAMES_TO_PLAY games (main.py:28-66).

    ``render=True`` (render_game, main.py:115-125) writes each game as an
    animated GIF under REPLAY_DIR instead of a gym viewer window: the games are
    replayed from their action traces and rasterised on the device
    (pong_amd.replay)."""
    if render:
        return _evaluate_rendered(individual)
    return next(evaluate_population([individual]))


def _evaluate_rendered(individual):
    import os

    from pong_amd import replay
    ev = _evaluator()
    genes = utils.calculate_gene_size()
    kind, opp, mult, members = schedule.reference_schedule(1, GAMES_TO_PLAY, hall_of_fame,  # noqa: F405
                                                           pick_hall_of_famer)
    genomes = runtime.genomes_to_device([individual], genes, ev)
    opponents = runtime.genomes_to_device(members, genes, ev) if members else None
    res, frames = replay.replay(ev, genomes[0], kind[0], opp[0], mult[0], opponents=opponents)
    for g, f in enumerate(frames):
        if len(f):
            replay.write_gif(f, os.path.join(REPLAY_DIR, f"game_{g}.gif"), fps=FPS)  # noqa: F405
    return next(_fitness_tuples(res.fitness.cpu().numpy(), res.status.cpu().numpy()))


evaluate.__pong_batch__ = evaluate_population


class DeviceEnv:
    """The env ``perform_episode`` plays (the retro env of main.py:35-55): one
    game of the build's Pong -- the emulator is absent --
    in game slot ``game`` (the slot fixes the game's serves, as
    ``evaluate``'s i-th game does), two players, or ``players=1`` for the
    1-player env whose left paddle is the built-in CPU (main.py:39-40).

    ``step(action)`` (env.step, main.py:77) advances the device stepper one
    frame (pg_physics_step; right paddle = action[4:6], left = action[6:8],
    config.py) and returns (frame, 0.0, done, {'score1', 'score2'}) with the
    frame rasterised on the device (pg_render_frames, a [210, 160, 3] uint8
    device tensor); ``render('rgb_array')`` is that frame on the host."""

    def __init__(self, game=0, players=2):
        self.game, self.players = int(game), int(players)
        self.use_restricted_actions = None
        self._ph = self._frame = None
        self._reset_pending = True

    def reset(self):
        # the device state is (re)made by the next step: resetting touches no GPU
        self._reset_pending = True
        self._frame = None

    def _device_reset(self):
        from pong_amd import device as D
        from pong_amd import replay
        dev = torch.device(DEVICE)  # noqa: F405
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if self._ph is None:
            self._ph = D.Physics(1, device=dev)
        seed = replay.game_seed(PHYSICS_SEED, self.game)  # noqa: F405
        seed = seed - (1 << 64) if seed >= 1 << 63 else seed
        self._ph.reset(torch.tensor([seed], dtype=torch.int64, device=dev),
                       torch.tensor([1 if self.players == 1 else 0], dtype=torch.int32, device=dev))
        self._reset_pending = False

    def step(self, action):
        from pong_amd import device as D
        if self._ph is None or self._reset_pending:
            self._device_reset()
        a = [int(v) for v in action]
        bits = a[4] | (a[5] << 1) | (a[6] << 2) | (a[7] << 3)
        self._ph.step(torch.tensor([bits], dtype=torch.uint8, device=self._ph.device))
        self._frame = D.render_frames(self._ph.state)[0]
        s1, s2 = (int(v) for v in self._ph.state[11:13, 0].tolist())  # PG_S_SCORE1, PG_S_SCORE2
        done = s1 >= 21 or s2 >= 21  # the game's own end (Pong::done)
        return self._frame, 0.0, done, {"score1": s1, "score2": s2}

    def render(self, mode="rgb_array"):
        return None if self._frame is None else self._frame.cpu().numpy()

    def close(self):
        self._ph = self._frame = None


def make_env(game=0, players=2):
    return DeviceEnv(game, players)


_SLOT_MUL = 0xA24BAED4963EE407  # game_seed's slot multiplier (pg_device.hpp)


def _slot_seed(game):
    # game_seed(base, g) = splitmix64(base ^ M (g + 1)): a one-game launch (slot
    # 0) plays slot ``game`` of PHYSICS_SEED from the base PHYSICS_SEED ^ M (game + 1) ^ M
    m = (1 << 64) - 1
    return (PHYSICS_SEED ^ ((_SLOT_MUL * (game + 1)) & m) ^ _SLOT_MUL) & m  # noqa: F405


def perform_episode(env, left_model, right_model, render=False, score_multiplier=1):
    """One game to its end (main.py:69-112), played by the device in one
    launch (pg_eval_population, one genome, one game): returns the right
    player's reward, 0 on a drawn score, as perform_episode does.

    ``right_model`` is a ``numpy_nn.NeuralNetwork``; ``left_model`` a
    NeuralNetwork (self-play / hall-of-fame game, ``score_multiplier`` scales
    the reward, main.py:47-49), a ``HardcodedAi`` or a ``ScoreHardcodedAi``;
    on a 1-player ``env`` the left model is ignored, as the reference's
    emulator ignores the second player's buttons.  ``render`` writes the game
    as a GIF under REPLAY_DIR (no viewer window).
    """
    from dumb_ais import HardcodedAi, ScoreHardcodedAi
    from numpy_nn import NeuralNetwork
    opponents = None
    if not isinstance(right_model, NeuralNetwork):
        kind = None
    elif getattr(env, "players", 2) == 1:
        kind = L.PG_OPP_ROM_CPU
    elif isinstance(left_model, NeuralNetwork):
        kind, opponents = L.PG_OPP_NN, left_model._genes
    elif isinstance(left_model, ScoreHardcodedAi):
        kind = L.PG_OPP_SCORE
    elif isinstance(left_model, HardcodedAi):
        kind = L.PG_OPP_HARDCODED
    else:
        kind = None
    if kind is None:  # a model the kernel has no game kind for (HumanInput, any .run): frame by frame
        if not hasattr(left_model, "run") or not hasattr(right_model, "run"):
            raise TypeError("perform_episode: models need run(input_vector) -> [up, down]")
        return perform_episode_stepwise(env, left_model, right_model, render, score_multiplier)
    ev = runtime.evaluator(right_model.nodes, bool(right_model.bias), 1, "float64", PRECISION,  # noqa: F405
                           _slot_seed(getattr(env, "game", 0)), DEVICE, TIMEOUT_THRESH, WIN_SCORE)  # noqa: F405
    dev = ev.device
    kind_t = torch.tensor([[kind]], dtype=torch.int32, device=dev)
    opp_t = torch.zeros((1, 1), dtype=torch.int32, device=dev)
    mult_t = torch.tensor([[float(score_multiplier)]], dtype=torch.float64, device=dev)
    if render:
        import os

        from pong_amd import replay
        res, frames = replay.replay(ev, right_model._genes[0], kind_t[0].cpu().numpy(), opp_t[0].cpu().numpy(),
                                    mult_t[0].cpu().numpy(), opponents=opponents)
        if len(frames[0]):
            replay.write_gif(frames[0], os.path.join(REPLAY_DIR, f"episode_{getattr(env, 'game', 0)}.gif"),  # noqa: F405
                             fps=FPS)  # noqa: F405
    else:
        res, _ = ev.evaluate(right_model._genes, kind_t, opp_t, mult_t, opponents=opponents)
    if int(res.status[0]):  # calculate_reward with total_frames == 0 (utils.py:106-108)
        raise ZeroDivisionError("float division by zero")
    return float(res.rewards[0, 0])


def perform_episode_stepwise(env, left_model, right_model, render=False, score_multiplier=1):
    """perform_episode (main.py:69-112) frame by frame from the host, for models
    the kernel cannot play itself: every frame is ``env.step`` on a DeviceEnv
    (device stepper + rasteriser), ``find_stuff`` (pg_find_stuff),
    ``get_actions`` through the models' ``run`` (a NeuralNetwork's is one
    pg_forward), the bounds clamp, the timeout bookkeeping and the
    termination test, in the reference's order.  ``render`` writes the frames
    as a GIF under REPLAY_DIR.  Returns the right player's reward."""
    from dumb_ais import ScoreHardcodedAi
    if not isinstance(env, DeviceEnv):
        raise TypeError("perform_episode_stepwise plays a main.DeviceEnv (make_env)")
    last_score = None
    action = np.copy(BLANK_ACTION)  # noqa: F405
    timeout_counter = 0.0
    total_frames = 0.0
    last_ball_location = None
    shown = []
    while True:
        observation, _reward, is_done, score_info = env.step(action)
        if isinstance(left_model, ScoreHardcodedAi):
            left_model.set_score(score_info)
        ball_location, left_location, right_location = utils.find_stuff(observation)
        left_action, right_action = get_actions(ball_location, last_ball_location, left_location, left_model,
                                                right_location, right_model)
        last_ball_location = ball_location
        action[RIGHT_ACTION_START:RIGHT_ACTION_END] = utils.keep_within_game_bounds_please(  # noqa: F405
            right_location, right_action)
        action[RIGHT_ACTION_END:LEFT_ACTION_END] = utils.keep_within_game_bounds_please(  # noqa: F405
            left_location, left_action)
        timeout_counter, total_frames = calculate_timeout_and_frames(last_score, score_info, timeout_counter,
                                                                     total_frames)
        last_score = score_info
        if render:
            shown.append(env.render("rgb_array"))
        if score_info["score1"] >= WIN_SCORE or score_info["score2"] >= WIN_SCORE:  # noqa: F405
            break
        if is_done:
            break
        if timeout_counter > TIMEOUT_THRESH:  # noqa: F405
            break
    env.reset()
    if render and shown:
        import os

        from pong_amd import replay
        replay.write_gif(np.stack(shown), os.path.join(REPLAY_DIR, f"episode_{env.game}.gif"), fps=FPS)  # noqa: F405
    if score_info["score1"] == score_info["score2"]:
        return 0
    return utils.calculate_reward(score_multiplier, total_frames, score_info["score2"], score_info["score1"])


def run_against_human(individual=None, human=None, render=True):
    """main.py:17-25: the individual's network on the right, a HumanInput on
    the left, one 2-player game rendered (a GIF here, no viewer).  ``human``:
    the left model (default ``HumanInput()``, which needs pynput's keyboard);
    pass ``HumanInput(keys=...)`` to script the keys headless."""
    from human_control import HumanInput
    right_model = utils.create_model_from_genes(individual)
    left_model = human if human is not None else HumanInput()
    env = make_env(0, players=2)
    env.reset()
    return perform_episode_stepwise(env, left_model, right_model, render, 1)


def get_actions(ball_location, last_ball_location, left_location, left_model, right_location, right_model):
    """The two paddles' [up, down] for one frame (main.py:138-154): a visible
    ball and a visible paddle decide through the model (the left player sees
    the field x-flipped); a missing paddle keeps a random action; no ball, no
    move.  Each model call is one device forward (numpy_nn.NeuralNetwork.run)."""
    # both defaults drawn first, as the reference does on every frame (main.py:137-138):
    # numpy's global RNG stream stays the reference's, ball or no ball
    left_action = utils.get_random_action(ALL_ACTIONS)  # noqa: F405
    right_action = utils.get_random_action(ALL_ACTIONS)  # noqa: F405
    if ball_location is None:
        return [0, 0], [0, 0]
    last = ball_location if last_ball_location is None else last_ball_location
    if left_location is not None:
        def flip(loc):  # [row, column] with the column mirrored
            return [loc[0], GAME_WIDTH - loc[1]]  # noqa: F405
        left_action = utils.inference(flip(ball_location), flip(last), left_location, right_location, left_model)
    if right_location is not None:
        right_action = utils.inference(ball_location, last, right_location, left_location, right_model)
    return left_action, right_action


def calculate_timeout_and_frames(last_score, score_info, timeout_counter, total_frames):
    """Frames without a score change, folded into total_frames at each change (main.py:128-135)."""
    if last_score is None:
        return timeout_counter, total_frames
    if last_score == score_info:
        return timeout_counter + 1.0, total_frames
    return 0.0, total_frames + timeout_counter


def main():
    stats = tools.Statistics(lambda ind: ind.fitness.values)
    for name, fn in (("avg", np.mean), ("std", np.std), ("min", np.min), ("max", np.max)):
        stats.register(name, fn)
    while True:
        ga.population, log = algorithms.eaSimple(
            ga.population, toolbox,
            cxpb=CROSSOVER_BLEND_PROBABILITY, mutpb=GAUSSIAN_MUTATION_PROBABILITY,  # noqa: F405
            ngen=GENERATIONS_BEFORE_SAVE,  # noqa: F405
            stats=stats, halloffame=hall_of_fame, verbose=True)
        print(log)
        save_checkpoint(ga.population, hall_of_fame)


toolbox.register("evaluate", evaluate)

if __name__ == '__main__':
    main()
