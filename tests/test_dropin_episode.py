"""The drop-in perform_episode's game slots (CPU): a one-game launch from
``main._slot_seed(g)`` plays slot g's serves, i.e. game_seed(_slot_seed(g), 0)
== game_seed(PHYSICS_SEED, g) (pg_device.hpp game_seed, oracle or_game_seed),
and the DeviceEnv surface perform_episode reads."""


def test_slot_seed_reproduces_evaluate_slots(oracle):
    import main
    for base in (main.PHYSICS_SEED, 0, 1234, (1 << 64) - 1):
        saved = main.PHYSICS_SEED
        main.PHYSICS_SEED = base
        try:
            for g in range(8):
                assert oracle.game_seed(main._slot_seed(g), 0) == oracle.game_seed(base, g)
        finally:
            main.PHYSICS_SEED = saved


def test_device_env_surface():
    import main
    env = main.make_env(3)
    assert (env.game, env.players) == (3, 2)
    assert main.make_env(1, players=1).players == 1
    env.reset()
    env.close()
