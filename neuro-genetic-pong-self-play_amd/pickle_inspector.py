"""The reference's pickle_inspector.py (pickle_inspector.py:1-12): load the best
checkpointed population and play its best individual with rendering on --
here the games are written as GIFs under config.REPLAY_DIR (main.evaluate)."""
from ga import load_best_population
from main import evaluate


def main():
    population = load_best_population()
    if population is None:
        raise SystemExit("no checkpoint under checkpoints/checkpoints/")
    individual = population[0]
    print(evaluate(individual=individual, render=True))


if __name__ == '__main__':
    main()
