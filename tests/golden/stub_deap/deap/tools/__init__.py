from .support import HallOfFame  # noqa: F401  (deap.tools re-exports deap.tools.support)
