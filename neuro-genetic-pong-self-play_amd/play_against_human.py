"""The reference's play_against_human.py (play_against_human.py:1-12): the best
checkpointed individual against a human on the left paddle (w = up, s =
down), one game rendered -- a GIF under config.REPLAY_DIR here (main.run_against_human)."""
from ga import load_best_population
from main import run_against_human


def main():
    population = load_best_population()
    if population is None:
        raise SystemExit("no checkpoint under checkpoints/checkpoints/")
    individual = population[0]
    print(run_against_human(individual))


if __name__ == '__main__':
    main()
