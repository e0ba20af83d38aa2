"""The reference's configuration surface (config.py:1-54): every name and
value is kept, so ``from config import *`` code runs unchanged.  Only the
integer dtype of the two action arrays differs in spelling: the reference's
``np.int`` (config.py:21,26) was removed from numpy 1.24 and aliased the
builtin ``int``.  The MI355X build's own knobs are at the end.
"""
import numpy as np

# --- frame colours (RGB) the pixel path matches on -----------------------
BG_COLOUR = (144, 72, 17)
BALL_COLOUR = (236, 236, 236)
LEFT_GUY_COLOUR = (213, 130, 74)
RIGHT_GUY_COLOUR = (92, 186, 92)

# --- playfield: rows GAME_TOP..GAME_BOTTOM of the 210x160 frame -----------
GAME_TOP = 34
GAME_BOTTOM = 194
GAME_PLAYABLE_HEIGHT = GAME_BOTTOM - GAME_TOP   # 160
GAME_WIDTH = 160
SCALED_PADDLE_HEIGHT = 16.0
FPS = 60

# --- the 16-button action vector: right paddle [4:6], left paddle [6:8] ---
RIGHT_ACTION_START = 4
RIGHT_ACTION_END = 6
LEFT_ACTION_END = 8
RIGHT_PLAYER_START_BUTTON = 0
LEFT_PLAYER_START_BUTTON = -1
BLANK_ACTION = np.zeros(shape=(16,), dtype=int)
for _button in (LEFT_PLAYER_START_BUTTON, RIGHT_PLAYER_START_BUTTON):
    BLANK_ACTION[_button] = 1
del _button
N_CLASSES = 2
ALL_ACTIONS = np.eye(N_CLASSES, dtype=int)

# --- episode ---------------------------------------------------------------
TIMEOUT_THRESH = 2_000
WIN_SCORE = 3
TIME_SCALER = 100.0
RENDER = False

# --- policy network --------------------------------------------------------
NETWORK_SHAPE = [6, 2, 2]
BIAS = True

# --- genetic algorithm -----------------------------------------------------
GAUSSIAN_MUTATION_MEAN = 0
GAUSSIAN_MUTATION_SIGMA = 0.9
GAUSSIAN_MUTATION_PROBABILITY = 0.9
PROBABILITY_OF_MUTATING_A_SINGLE_GENE = 0.9
CROSSOVER_BLEND_PROBABILITY = 0.9
CROSSOVER_BLEND_ALPHA = 0.9

# often changed
POPULATION_SIZE = 64
GAMES_TO_PLAY = 6
GENERATIONS_BEFORE_SAVE = 5
TOURNAMENT_SIZE = POPULATION_SIZE // 4
HALL_OF_FAME_AMOUNT = TOURNAMENT_SIZE

# --- MI355X build knobs (new; the reference has no device/precision/seed) ---
# Base seed of the Pong physics' serve randomness, per game slot (DESIGN.md "Physics").
PHYSICS_SEED = 0
# "certified": f32 hidden math whose f64 argmax is proven per decision (f64
# re-decision otherwise); "f64": numpy_nn's f64 arithmetic for every pass.
PRECISION = "certified"
# Storage type of genomes on the device; float64 keeps Python floats exact.
GENOME_DTYPE = "float64"
# "cuda" = the process's current HIP device (one process per GPU).
DEVICE = "cuda"
# evaluate(render=True) writes each replayed game here as game_<g>.gif (no viewer window).
REPLAY_DIR = "replays"
