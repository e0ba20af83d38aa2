"""The host-side mirror of the reference surface (config / utils / dumb_ais /
main helpers / batched map / schedule) against the reference's golden vectors.
CPU only: nothing here launches a kernel."""
import functools
import random

import numpy as np
import pytest


def test_config_surface(golden):
    import config
    ref = golden("helpers.json")["config"]
    for name, value in ref.items():
        got = getattr(config, name)
        if isinstance(got, np.ndarray):
            assert got.tolist() == value, name
        elif isinstance(got, tuple):
            assert list(got) == value, name
        else:
            assert got == value, name
    assert config.BLANK_ACTION.dtype.kind == "i" and config.ALL_ACTIONS.dtype.kind == "i"


def test_inference_features(golden):
    import utils

    class Rec:
        def run(self, x):
            self.x = x
            return [1, 0]

    for case in golden("helpers.json")["inference"]:
        r = Rec()
        utils.inference(case["ball"], case["last"], case["me"], case["enemy"], r)
        assert r.x == case["features"]  # bit-exact f64
        # the kernels' form: doubled centroids k -> (k / 2) / 160
        k = [2 * case["ball"][1], 2 * case["ball"][0], 2 * case["last"][1], 2 * case["last"][0],
             2 * case["me"][0], 2 * case["enemy"][0]]
        assert [(0.5 * v) / 160.0 for v in k] == case["features"]


def test_bounds_clamp(golden):
    import utils
    for case in golden("helpers.json")["clamp"]:
        paddle = None if case["paddle"] is None else np.array(case["paddle"])
        assert list(utils.keep_within_game_bounds_please(paddle, case["action"])) == case["out"]


def test_calculate_reward(golden):
    import utils
    for case in golden("helpers.json")["reward"]:
        got = utils.calculate_reward(case["mult"], case["total"], case["my"], case["enemy"])
        assert got == case["reward"]


def test_timeout_and_frames(golden):
    import main
    for case in golden("helpers.json")["timeout_frames"]:
        last, t, tot = None, 0.0, 0.0
        for (s1, s2), want in zip(case["seq"], case["out"]):
            info = {"score1": s1, "score2": s2}
            t, tot = main.calculate_timeout_and_frames(last, info, t, tot)
            last = info
            assert [t, tot] == want


def test_dumb_ais(golden):
    import dumb_ais
    for case in golden("helpers.json")["dumb_ais"]:
        assert dumb_ais.HardcodedAi().run(case["x"]) == case["hard"]
        sc = dumb_ais.ScoreHardcodedAi()
        sc.set_score({"score1": case["score"][0], "score2": case["score"][1]})
        assert sc.run(case["x"]) == case["score_ai"]


def test_gene_size(golden):
    import utils
    saved = utils.NETWORK_SHAPE
    try:
        for case in golden("helpers.json")["gene_size"]:
            utils.NETWORK_SHAPE = case["shape"]
            assert utils.calculate_gene_size() == case["genes"]
    finally:
        utils.NETWORK_SHAPE = saved


def test_batched_map_routes_evaluate_only():
    from pong_amd.batched import batched_map
    calls = []

    def evaluate(ind):
        raise AssertionError("per-individual path must not run")

    def batch(inds):
        calls.append(list(inds))
        return iter([(float(sum(i)),) for i in inds])

    evaluate.__pong_batch__ = batch
    wrapped = functools.partial(evaluate)
    wrapped.__dict__.update(evaluate.__dict__)
    out = list(batched_map(wrapped, [[1, 2], [3, 4]]))
    assert out == [(3.0,), (7.0,)] and calls == [[[1, 2], [3, 4]]]
    # other functions and partials with bound arguments use the builtin map
    assert list(batched_map(lambda x: x * 2, [1, 2])) == [2, 4]
    assert list(batched_map(functools.partial(lambda a, b: a + b, 10), [1, 2])) == [11, 12]


def test_zero_division_raised_lazily():
    import main
    it = main._fitness_tuples(np.array([1.0, 2.0, 3.0]), np.array([0, 1, 0]))
    assert next(it) == (1.0,)
    with pytest.raises(ZeroDivisionError):
        next(it)


def test_schedule_semantics():
    """Games 0-2 scripted with multiplier 1; later games draw a hall-of-famer
    (shuffle in place, first valid) whose fitness becomes the multiplier."""
    import utils
    from pong_amd import schedule

    class Fit:
        def __init__(self, v, valid=True):
            self.values = (v,)
            self.valid = valid

    class M(list):
        def __init__(self, g, f, valid=True):
            super().__init__(g)
            self.fitness = Fit(f, valid)

    class HoF:
        def __init__(self, items):
            self.items = items

    # empty hall of fame / None: HardcodedAi, multiplier 1, no random calls
    state = random.getstate()
    k, o, m, mem = schedule.reference_schedule(3, 6, HoF([]), utils.pick_hall_of_famer)
    assert random.getstate() == state
    assert k.tolist() == [[0, 1, 2, 0, 0, 0]] * 3 and np.all(m == 1) and mem == []
    k, o, m, mem = schedule.reference_schedule(2, 6, None, utils.pick_hall_of_famer)
    assert k.tolist() == [[0, 1, 2, 0, 0, 0]] * 2
    # only invalid members: no opponent, multiplier 1 (utils.py:92,96-100)
    hof = HoF([M([0.0], 5.0, valid=False)])
    k, o, m, mem = schedule.reference_schedule(1, 6, hof, utils.pick_hall_of_famer)
    assert k.tolist() == [[0, 1, 2, 0, 0, 0]] and np.all(m == 1)
    # valid members: same draws as the reference's create_model_from_hall_of_fame
    items = [M([float(i)], 0.25 * i - 1.0) for i in range(5)]
    hof = HoF(list(items))
    random.seed(11)
    k, o, m, mem = schedule.reference_schedule(4, 7, hof, utils.pick_hall_of_famer)
    random.seed(11)
    shadow = list(items)
    for r in range(4):
        for g in range(3, 7):
            random.shuffle(shadow)
            assert mem[o[r, g]] is shadow[0]
            assert m[r, g] == shadow[0].fitness.values[0]
    assert [id(x) for x in hof.items] == [id(x) for x in shadow]  # shuffled in place
    assert np.all(k[:, 3:] == 3) and np.all(m[:, :3] == 1)


def test_replay_game_seed_matches_oracle(oracle):
    """pong_amd.replay's host game seeds equal the physics' (or_game_seed = pg_device game_seed)."""
    from pong_amd.replay import game_seed
    for base in (0, 1, 12345, 2**63 + 7, 2**64 - 1):
        for g in range(8):
            assert game_seed(base, g) == oracle.lib().or_game_seed(base, g)


def test_human_input_key_sources():
    """human_control.HumanInput (human_control.py:26-36): run() returns the held
    [w, s] keys as [up, down]; headless, the keys come from a callable of
    (call index, input vector) or an iterable (exhausted = nothing held);
    without a key source it needs pynput's keyboard, which is absent here."""
    import human_control
    h = human_control.HumanInput(keys=lambda f, x: (f % 2, x[1] > 0.5))
    assert h.run([0, 0.9, 0, 0, 0, 0]) == [0, 1] and h.run([0, 0.1, 0, 0, 0, 0]) == [1, 0] and h.frame == 2
    h = human_control.HumanInput(keys=[(1, 0), (1, 1)])
    assert h.run() == [1, 0] and h.run() == [1, 1] and h.run() == [0, 0]
    try:
        import pynput  # noqa: F401
    except ImportError:
        with pytest.raises(RuntimeError):
            human_control.HumanInput()
