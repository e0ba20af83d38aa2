/*
 * pong_ga.h -- C-ABI of the MI355X-native GA evaluation loop (libpong_ga.so).
 *
 * This is the drop-in boundary for the reference's hot path
 * (n00b001/neuro-genetic-pong-self-play).  Every entry point takes plain
 * pointers and sizes; all array arguments are DEVICE pointers owned by the
 * caller (the Python host passes torch tensors' data_ptr()), and every call
 * is ordered on the HIP stream passed in (NULL = the null stream).  The
 * library keeps no device allocations between calls.  Errors: the functions
 * return PG_OK (0) or a negative pg_status; pg_last_error() returns a
 * thread-local message for the last failure.  Nothing throws across the ABI.
 * Threading: one host thread per device; the caller selects the device.
 *
 * Entry point                    replaces (reference file:line)
 * ------------------------------ ---------------------------------------------
 * pg_eval_population             toolbox.map(toolbox.evaluate, invalid_ind)
 *                                (ga.py:83 futures.map, main.py:176 register):
 *                                evaluate() main.py:28-66 for a whole batch,
 *                                each game = perform_episode main.py:69-112 with
 *                                env.step main.py:77, find_stuff utils.py:14-19,
 *                                get_actions main.py:138-154, inference
 *                                utils.py:139-153, NeuralNetwork.run
 *                                numpy_nn.py:120-137, keep_within_game_bounds
 *                                utils.py:71-77, calculate_timeout_and_frames
 *                                main.py:128-135, calculate_reward utils.py:104-109
 * pg_forward                     NeuralNetwork.run numpy_nn.py:120-137 (batched)
 * pg_decide                      get_actions' model.run argmax (main.py:143-150) as the
 *                                hot kernel decides it (test / fixture entry point)
 * pg_wide_decide                 the same, as k_wide decides it (config 5 networks)
 * pg_physics_reset/pg_physics_step  env.reset()/env.step(action) main.py:56,77
 *                                (the build's SoA Pong; the emulator is absent)
 * pg_ga_select_tournament        tools.selTournament (ga.py:94; DEAP)
 * pg_ga_vary                     algorithms.varAnd with tools.cxBlend (ga.py:89)
 *                                and tools.mutGaussian (ga.py:91-92; DEAP)
 * pg_ga_schedule                 the opponent picks of evaluate() main.py:28-66 /
 *                                create_model_from_hall_of_fame utils.py:90-101
 *                                for a whole population, on device
 * pg_row_hash                    DEAP HallOfFame's similar (operator.eq on the
 *                                gene lists, ga.py:78) as a 64-bit row hash
 * pg_hof_prepare /               HallOfFame.update's device half: the candidates,
 * pg_hof_rank_classes            their hashes, the (fitness, age) ranks and
 *                                similarity classes the host scan reads
 * pg_hof_update (host)           tools.HallOfFame.update (eaSimple, main.py:165-170)
 * pg_hof_update_packed (host)    the same over the device's packed ranks and classes, O(k log k)
 * pg_gather_rows                 the new hall's genomes (HallOfFame.insert's deepcopy)
 * pg_ga_scatter_fitness /        eaSimple's bookkeeping around toolbox.map
 * pg_ga_merge_fitness            (main.py:165-170): fitness assigned to invalid_ind,
 *                                clones keep their parent's, the logbook statistics
 *                                (main.py:158-162), the hall's candidates
 * pg_ga_select_ranked            tools.selTournament (ga.py:94) with its sort inside
 * pg_ga_inherit / pg_ga_order    varAnd's clones' inherited state; the evaluation
 *                                order of invalid_ind
 * pg_hof_prepare_cand /          HallOfFame.update's device half for known
 * pg_hof_commit                  candidates; the new members' rows, hashes, fitness
 * pg_render_frames               the frame env.step returns (main.py:77; the build's
 *                                rasteriser of its SoA state in config.py colours)
 * pg_find_stuff                  find_stuff utils.py:14-19 / get_rect_quickly
 *                                utils.py:60-68, batched
 */
#ifndef PONG_GA_H
#define PONG_GA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PG_ABI_VERSION 12
#define PG_MAX_NODES 9 /* len(NETWORK_SHAPE) <= 9 */

typedef enum pg_status {
  PG_OK = 0,
  PG_ERR_INVALID = -1,     /* bad argument (message in pg_last_error) */
  PG_ERR_HIP = -2,         /* a HIP runtime call failed */
  PG_ERR_UNSUPPORTED = -3  /* shape/option not supported by this build */
} pg_status;

typedef enum pg_dtype { PG_F32 = 0, PG_F64 = 1 } pg_dtype;

/* Left-paddle opponent of one game (the genome always plays the right paddle,
 * main.py:58 right_model). */
typedef enum pg_opp_kind {
  PG_OPP_HARDCODED = 0, /* HardcodedAi in the 2-player env     main.py:50-53 */
  PG_OPP_ROM_CPU = 1,   /* 1-player env: built-in CPU opponent  main.py:39-40 */
  PG_OPP_SCORE = 2,     /* ScoreHardcodedAi                     main.py:41-42 */
  PG_OPP_NN = 3         /* NeuralNetwork of a hall-of-fame row  main.py:43-49 */
} pg_opp_kind;

typedef enum pg_precision {
  /* f32 hidden math with a certified f64 argmax: every decision whose
   * f32 error bound cannot prove the f64 argmax is recomputed in f64. */
  PG_PREC_CERTIFIED = 0,
  /* every forward in f64 (numpy_nn's arithmetic: each dot product in np.dot's own
   * order, OpenBLAS dgemv_t's partial sums, blas_dot in pg_device.hpp) */
  PG_PREC_F64 = 1
} pg_precision;

typedef enum pg_kernel {
  PG_KERNEL_AUTO = 0,      /* SPLIT when the shape and precision allow, else GENERAL */
  PG_KERNEL_GENERAL = 1,   /* one wave per game, f64, any NETWORK_SHAPE */
  PG_KERNEL_RESIDENT = 2,  /* retired (round 4): PG_ERR_UNSUPPORTED */
  PG_KERNEL_SPLIT = 3      /* [6, H<=256, 2..4]: half a lane group per paddle's network; f32 forwards with
                              a certified argmax, the failures re-decided in f64 by the wave itself
                              (8-lane groups) or by one service wave per block (other layouts) */,
  PG_KERNEL_WIDE = 4,      /* [6, H1<=512, H2<=512, 1..4]: one 512-thread workgroup per genome plays its
                              games (up to 6; more: balanced chunks of <= 6, one workgroup pass each)
                              in lockstep and streams W2 from HBM each frame
                              (numpy_nn's f64 order; AUTO picks it for H1 or H2 >= 64) */
  PG_KERNEL_STAGED = 5     /* retired (round 4): PG_ERR_UNSUPPORTED */
} pg_kernel;

/* pg_eval_args.prep: the SPLIT kernel's lane records (one per network of the
 * launch) in two halves, so a caller can prepare the genomes' records while
 * the opponents (the hall of fame) are still being decided.  Other kernels
 * have no records: PG_PREP_GENOMES does nothing there, PG_PREP_REST = ALL. */
typedef enum pg_prep {
  PG_PREP_ALL = 0,      /* prepare every record, then play */
  PG_PREP_GENOMES = 1,  /* only prepare the genomes' records into the workspace; no games are played */
  PG_PREP_REST = 2      /* the genomes' records were prepared by a PG_PREP_GENOMES call with the same
                           workspace, genomes, genome_rows, n_active and n_genomes: prepare the
                           opponents' records, then play */
} pg_prep;

/* NETWORK_SHAPE (config.py:30-32) + BIAS (config.py:34) + genome storage type. */
typedef struct pg_net {
  int32_t n_nodes;               /* len(NETWORK_SHAPE), >= 2 */
  int32_t nodes[PG_MAX_NODES];   /* nodes[0] = 6 for the game loop */
  int32_t bias;                  /* 1 = BIAS, weight rows are (in + 1) wide */
  int32_t dtype;                 /* pg_dtype of genomes and opponents */
} pg_net;

typedef struct pg_eval_args {
  /* ABI 10 (11: + timeout_thresh, win_score): sizeof(pg_eval_args) as the caller compiled it.  pg_eval_population
   * and pg_eval_workspace_bytes refuse any other value (PG_ERR_INVALID / 0
   * bytes): a binding whose struct is shorter or longer than this header's
   * would otherwise have the library read past it.  Always the first field,
   * so even a stale struct's value is read from memory the caller owns. */
  uint32_t struct_size;
  pg_net net;
  int32_t n_genomes;             /* rows of genomes evaluated by this call (>= 0) */
  int32_t n_games;               /* GAMES_TO_PLAY (config.py:46), 1..64 */
  const void *genomes;           /* [n_genomes, genome_stride] (net.dtype) */
  int64_t genome_stride;         /* elements between genome rows, >= gene count */
  const void *opponents;         /* [n_opponents, opponent_stride]: hall-of-fame genomes */
  int64_t opponent_stride;
  int32_t n_opponents;
  int32_t precision;             /* pg_precision */
  const int32_t *game_kind;      /* [n_genomes, n_games] pg_opp_kind */
  const int32_t *game_opp;       /* [n_genomes, n_games] opponent row (PG_OPP_NN) */
  const double *game_mult;       /* [n_genomes, n_games] right_score_multiplier */
  uint64_t seed;                 /* physics seed base (config.PHYSICS_SEED) */
  /* outputs, device */
  double *fitness;               /* [n_genomes]  evaluate()[0] = sum(rewards)/n_games */
  double *rewards;               /* [n_genomes, n_games] perform_episode() */
  int32_t *scores;               /* [n_genomes, n_games, 2] final score1, score2 */
  int32_t *frames;               /* [n_genomes, n_games] env.step calls */
  double *total_frames;          /* [n_genomes, n_games] main.py:73 accumulator */
  int32_t *status;               /* [n_genomes] 1 = ZeroDivisionError in calculate_reward */
  uint64_t *counters;            /* optional [16], zeroed by the call: [0] env steps stepped one frame at a time, [1] NN
                                    forwards, [2] numpy-order f64 forwards, [3] games; split kernel: [4]
                                    f32 certificate failures, [5] failures decided by the certified f64
                                    rules (plateau, gap), [6] failures decided in-wave by the f32 plateau
                                    rule; wide kernel: [7] network weight passes; split and wide
                                    kernels: [8] episode frames of periodic rallies advanced to their
                                    timeout at once; [9] hard decisions (see hard_log); split kernel:
                                    [12] serve-delay frames advanced at once (ball hidden); the
                                    episodes' frames = [0] + [8] + [12]; [10], [11], [13..15] 0 */
  uint8_t *trace;                /* optional [trace_games, trace_cap] per-frame action codes */
  int32_t trace_games;           /* games (genome-major index g = i*n_games + game) traced */
  int32_t trace_cap;
  int32_t kernel;                /* pg_kernel */
  int32_t group_lanes;           /* lanes per game of RESIDENT (4..64) / SPLIT (8..64), 0 = auto */
  void *workspace;               /* device scratch of pg_eval_workspace_bytes() bytes */
  size_t workspace_bytes;
  uint32_t *hard_log;            /* optional [hard_cap][8] records of the decisions no bound settles
                                    (fixtures for tests/golden/nn_hard_cases): split kernel, forwards the
                                    certified f64 rules hand to the numpy-order f64 forward; wide kernel,
                                    decisions whose two largest activations lie within 1e-12 (not both
                                    1.0).  Record: {row, flags, k0..k5}; flags bit 0 = row of the
                                    opponents (else genomes), bits 8..15 the decided index, bits 16..23
                                    the source (0 split, 1 wide).  counters[9] counts every such
                                    decision, also past hard_cap (requires counters). */
  int32_t hard_cap;
  const int32_t *genome_rows;    /* optional [n_genomes] device: game block i plays genomes row
                                    genome_rows[i] (NULL: row i); results stay indexed by i.  Lets the
                                    caller evaluate only eaSimple's invalid_ind (main.py:165-170)
                                    without copying rows; every index must be a valid row. */
  const int32_t *n_active;       /* optional device int32: only game blocks i < *n_active are played
                                    (n_genomes is then an upper bound; results of blocks >= *n_active,
                                    and their counters, are left untouched) -- a count computed on the
                                    device needs no host round trip before the launch. */
  int32_t prep;                  /* pg_prep (ABI 7): PG_PREP_ALL unless the records are prepared in two calls */
  int32_t horizon;               /* ABI 8, SURVEY 8(d)'s fixed-horizon measurement mode; 0 = off (evaluate()'s
                                    episodes).  T > 0 (SPLIT kernel only: [6, 33..64, 3] networks, the default
                                    8-lane groups, untraced; else PG_ERR_UNSUPPORTED): every game slot
                                    runs exactly T frames; an episode that terminates (main.py:102-107) before
                                    frame T is scored (calculate_reward) and the slot auto-resets (a fresh
                                    episode, the same networks, the serve sequence continuing), the partial
                                    last episode is dropped; no frame is advanced in closed form (counters[0]
                                    = n_games * T per genome, [8] = [12] = 0).  Outputs per game: rewards =
                                    the sum of the completed episodes' rewards in order, scores = the points
                                    of all its episodes (score1, score2), frames = T, total_frames = the
                                    completed episodes, status = any ZeroDivisionError; fitness as usual. */
  /* ABI 11: the episode limits of perform_episode (main.py:102-107), config.py's TIMEOUT_THRESH
     and WIN_SCORE; 0 = the reference's values (2000, 3).  A game ends when a score reaches
     win_score (1..21; the env's own end at 21 comes first above that) or when the no-score
     counter of calculate_timeout_and_frames (main.py:128-135) exceeds timeout_thresh
     (32..1048576: never while a served ball is still hidden, 30 frames). */
  int32_t timeout_thresh;
  int32_t win_score;
} pg_eval_args;

/* Trace byte: right_code | left_code << 2 | ball_visible << 4, where a code is
 * 0 = [0,0], 1 = [1,0] (up), 2 = [0,1] (down): the action written into
 * action[4:6] / action[6:8] after that frame (main.py:91-92). */

typedef struct pg_forward_args {
  pg_net net;
  int32_t n;                     /* forward passes */
  const void *genomes;           /* [*, genome_stride] (net.dtype) */
  int64_t genome_stride;
  const int32_t *genome_index;   /* [n] genome row of pass i; NULL = row i */
  const double *x;               /* [n, nodes[0]] inputs */
  int32_t precision;             /* pg_precision */
  int32_t *index;                /* [n] np.argmax of the output activations */
  double *act;                   /* optional [n, nodes[last]] output activations */
  uint64_t *counters;            /* optional [4]: [2] += passes re-decided in f64 (others unused) */
  double *z_all;                 /* optional, PG_PREC_F64 only: [n, sum(nodes[1:])] every layer's
                                    pre-activations np.dot(w, column) (numpy_nn.py:127), layer by layer */
  double *h_all;                 /* optional, PG_PREC_F64 only: the same layout, the activations */
} pg_forward_args;

/* The split kernel's decision for given inputs: pass i is network row
 * genome_index[i] (i if NULL) on the doubled-centroid features k[i][0..5]
 * (utils.inference's inputs are k / 320; main.py:143-150).  It runs the very
 * cascade k_service runs in a game -- the f32 pass and its certificate, the
 * in-wave plateau rule, the f64 plateau and certified rules,
 * and last the numpy-order f64 forward -- so fixtures of hard inputs pin the
 * hot kernel's decisions.  [6, H <= 256, 2..4] networks. */
typedef struct pg_decide_args {
  pg_net net;
  int32_t n;
  const void *genomes;           /* [*, genome_stride] (net.dtype) */
  int64_t genome_stride;
  const int32_t *genome_index;   /* [n] or NULL */
  const int32_t *k;              /* [n, 6] doubled centroids, each in [0, 320] */
  int32_t *index;                /* out [n] np.argmax of NeuralNetwork.run's activations */
  int32_t *stage;                /* optional out [n]: 0 f32 certificate, 1 in-wave plateau rule,
                                    2 certified f64 rules, 3 numpy-order f64 forward,
                                    4 the f32 rules under the frame's own bound (H in 33..64,
                                    the layout whose k_service decides in the game wave) */
} pg_decide_args;

/* The wide kernel's decision for given inputs: k_wide itself (the evaluation
 * kernel of [6, H1 <= 512, H2 <= 512, 1..4] networks, BASELINE config 5) runs
 * one frame of network row genome_index[i] (i if NULL) on the doubled
 * centroids k[i][0..5] -- its layer path and argmax exactly as in a game
 * (get_actions main.py:143-150, NeuralNetwork.run numpy_nn.py:120-137), so the
 * near-tie fixtures k_wide logs (pg_eval_args.hard_log) pin k_wide itself. */
typedef struct pg_wide_decide_args {
  pg_net net;
  int32_t n;
  const void *genomes;           /* [*, genome_stride] (net.dtype) */
  int64_t genome_stride;
  const int32_t *genome_index;   /* [n] or NULL */
  const int32_t *k;              /* [n, 6] doubled centroids, each in [0, 320] */
  int32_t *index;                /* out [n] np.argmax of NeuralNetwork.run's activations */
  double *act;                   /* optional out [n, nodes[3]] the output activations */
  void *workspace;               /* device, pg_wide_decide_workspace_bytes */
  size_t workspace_bytes;
} pg_wide_decide_args;

/* Struct-of-arrays game state: int32 [PG_STATE_FIELDS, n], field f of game i
 * at state[f * n + i]; 64 bytes per game. */
enum {
  PG_S_BALL_X = 0, PG_S_BALL_Y, PG_S_BALL_VX, PG_S_BALL_VY, PG_S_BALL_VISIBLE,
  PG_S_SERVE_TIMER, PG_S_SERVE_DIR, PG_S_HITS, PG_S_POINT, PG_S_LEFT_Y, PG_S_RIGHT_Y,
  PG_S_SCORE1, PG_S_SCORE2, PG_S_ONE_PLAYER, PG_S_SEED_LO, PG_S_SEED_HI,
  PG_STATE_FIELDS
};

/* GA step on device (DEAP semantics, counter-based RNG): see pg_ga_vary. */
typedef struct pg_ga_args {
  int32_t n;                     /* population size */
  int64_t genes;                 /* genes per genome */
  int32_t dtype;                 /* pg_dtype of both genome buffers */
  const void *parents;           /* [n_parents, stride] current population */
  int64_t stride;
  int32_t n_parents;
  const int32_t *chosen;         /* [n] parent row of offspring slot i (selection) */
  void *offspring;               /* [n, stride] output */
  uint8_t *invalid;              /* [n] 1 = fitness invalidated (varied) */
  double cxpb, mutpb;            /* CROSSOVER_BLEND_PROBABILITY, GAUSSIAN_MUTATION_PROBABILITY */
  double alpha;                  /* CROSSOVER_BLEND_ALPHA */
  double mu, sigma, indpb;       /* GAUSSIAN_MUTATION_MEAN/SIGMA, PROBABILITY_OF_MUTATING_A_SINGLE_GENE */
  uint64_t seed;                 /* RNG key: (seed, generation) */
  uint64_t generation;
  /* ABI 9: [(n + 1) / 2] or NULL.  Non-NULL: only the pairs (2j, 2j + 1) with
   * pair_mask[j] != 0 are written to offspring (invalid[] is written for every
   * row either way).  Every offspring row is a pure function of its pair's
   * parent rows and the (seed, generation) keys, so rows varied in separate
   * calls equal one full call's: a rank of a sharded run varies its shard
   * first and, once the fitness all-gather has named them, the hall-of-fame
   * candidates and the next selection's parents. */
  const uint8_t *pair_mask;
  /* ABI 10: or a compact list of the pairs to vary -- pair_list[0 .. *pair_count)
   * (device) -- so a completion that varies a few thousand of P / 2 pairs
   * launches that many waves, not one per pair.  pair_cap only sizes the grid
   * (min(pair_cap, pairs, 8192) waves, which stride over the list: since ABI
   * 12 every listed pair is written whatever pair_cap >= 1 is, so a caller
   * that knows the count only on the device passes an upper bound).  Only the listed pairs' rows and invalid flags are written (pair_mask
   * is then ignored); pg_ga_list_pairs turns a mask into such a list. */
  const int32_t *pair_list;
  const int32_t *pair_count;
  int32_t pair_cap;
} pg_ga_args;

typedef struct pg_select_args {
  int32_t n_pop;                 /* individuals to choose from */
  int32_t k;                     /* picks (len(population)) */
  int32_t tournsize;             /* TOURNAMENT_SIZE (config.py:49) */
  const double *fitness;         /* [n_pop] */
  int32_t *chosen;               /* [k] output: row of the winner of tournament j */
  uint64_t seed;
  uint64_t generation;
} pg_select_args;

/* Per-game opponents of a population (evaluate(), main.py:28-66). */
typedef enum pg_schedule_mode {
  /* games 0, 1, 2: HardcodedAi, the ROM CPU, ScoreHardcodedAi; games >= 3: a
   * uniformly random hall-of-fame member (create_model_from_hall_of_fame
   * utils.py:90-101 shuffles and takes the first valid one) whose fitness is
   * the right_score_multiplier; HardcodedAi with multiplier 1 if n_hof = 0 */
  PG_SCHED_REFERENCE = 0,
  /* every game against hall-of-fame row ((row_offset + i) * n_games + g) mod n_hof */
  PG_SCHED_SELFPLAY = 1
} pg_schedule_mode;
/* PG_SCHED_SELFPLAY with hof_slices K > 1 (ABI 10): the hall is K interleaved
 * slices (slice b = members b, b + K, b + 2K, ... of [0, n_hof)), and the
 * genomes of global row block b' = row / block_rows play slice b = b' mod K:
 * game g of row r against slice member ((r * n_games + g) mod |slice b|), i.e.
 * hall row that * K + b (slice_local: the index within the slice, for a caller
 * that passes the slice itself as the opponents -- a rank whose shard is one
 * block needs only its slice's lane records).  Every slice spans
 * the whole fitness order, so the blocks face statistically equal opponents. */

typedef struct pg_schedule_args {
  int32_t mode;                  /* pg_schedule_mode */
  int32_t n;                     /* rows */
  int32_t n_games;
  int64_t row_offset;            /* global index of row 0 (a rank's shard) */
  int32_t n_hof;                 /* valid hall-of-fame members: opponent rows [0, n_hof) */
  const double *hof_fitness;     /* [n_hof] device: a pick's right_score_multiplier */
  uint64_t seed;                 /* picks keyed by (seed, generation, global row, game) */
  uint64_t generation;
  int32_t *kind;                 /* out [n, n_games] device, pg_opp_kind */
  int32_t *opp;                  /* out [n, n_games] device */
  double *mult;                  /* out [n, n_games] device */
  const int32_t *rows;           /* optional [n] device: global row of entry i (NULL: row_offset + i) */
  int32_t hof_slices;            /* ABI 10, PG_SCHED_SELFPLAY: K slices of the hall (0 or 1: one, as before) */
  int32_t block_rows;            /* rows per genome block (K > 1: >= 1) */
  int32_t slice_local;           /* 1: opp = index within the block's slice; 0: hall row */
} pg_schedule_args;

/* HallOfFame.update (DEAP) over host arrays.  Members are in HallOfFame.items
 * order (best first; among equal fitness the newest first); "similar" is the
 * equality of pg_row_hash values (or of any other class labels: when every
 * label lies in [0, hof_n + pop_n), e.g. dense ids from a device-side unique,
 * counts are kept in a direct-indexed array).  Sequential semantics: an individual enters
 * iff the hall is not full or its fitness beats the worst member strictly,
 * and no member is similar; a full hall drops its last (worst, oldest among
 * equals) member; an empty hall first takes population[0].  Fitness must not
 * be NaN.  O(hof_n + pop_n) given the ranks: while the hall is full its worst
 * member only moves up the (fitness, age) order. */
typedef struct pg_hof_args {
  int32_t maxsize;               /* HALL_OF_FAME_AMOUNT (config.py:50) */
  int32_t hof_n;                 /* current members */
  const double *hof_fitness;     /* [hof_n] host */
  const uint64_t *hof_hash;      /* [hof_n] host */
  int32_t pop_n;
  const double *pop_fitness;     /* [pop_n] host, population order */
  const uint64_t *pop_hash;      /* [pop_n] host */
  const int32_t *rank;           /* optional [hof_n + pop_n] host: each entry's position in the ascending
                                    order of (fitness, age) -- old member j is entry j, aged so that
                                    member hof_n - 1 is the oldest; population row i is entry hof_n + i,
                                    newer than every member and than rows < i.  NULL: sorted here. */
  int32_t *new_n;                /* out: members after the update */
  int32_t *new_src;              /* out [maxsize]: member j's source: j' < hof_n = old member j',
                                    hof_n + i = population row i */
  double *new_fitness;           /* out [maxsize] */
} pg_hof_args;

/* pg_hof_update over the device's packing (pg_hof_rank_classes /
 * pg_hof_prepare_cand: packed[e] = rank | class << 32 for the hof_n members in
 * items order and the k candidates in population order, then the candidates'
 * fitness bits), host arrays.  The same rule and result as pg_hof_update, in
 * O(k log k + new_n): the members are in items order, so the worst remaining
 * member is always the last not yet evicted, and a member class (the first
 * member of its hash) is present exactly while that member is; only the
 * members at the hall's tail and the candidates are visited, and the output
 * is filled by ranges.  Falls back to the full scan when the members' ranks
 * are not descending. */
typedef struct pg_hof_packed_args {
  int32_t maxsize;               /* HALL_OF_FAME_AMOUNT */
  int32_t hof_n;                 /* current members */
  const double *hof_fitness;     /* [hof_n] host, items order */
  int32_t k;                     /* candidates */
  const int64_t *packed;         /* [hof_n + 2k] host */
  int32_t *new_n;                /* out */
  int32_t *new_src;              /* out [maxsize]: j' < hof_n old member j', hof_n + c candidate c */
  double *new_fitness;           /* out [maxsize] */
  /* ABI 12, the hall kept in place: member j's row lives in storage slot
   * slot[j].  slot_in [hof_n] (NULL: slot j = j) the members' slots; slot_out
   * (NULL: not computed) [maxsize] out: a kept member keeps its slot, an
   * entering candidate takes a slot an evicted member freed (in items order
   * of the evicted) or, while the hall grows, slot hof_n, hof_n + 1, ...;
   * the slots in use are always [0, new_n). */
  const int32_t *slot_in;
  int32_t *slot_out;
} pg_hof_packed_args;
int32_t pg_hof_update_packed(const pg_hof_packed_args *args);

/* Device half of the hall-of-fame update (pg_hof_rank_classes): for the old
 * members (items order) and k candidate rows, each entry's pg_hof_args.rank and
 * a dense similarity class of the row hashes, packed as
 * packed[e] = rank[e] | class[e] << 32 for e < hof_n + k (members first), then
 * packed[hof_n + k + j] = the bits of candidate j's fitness.  All pointers are
 * device memory on the stream's device; workspace >=
 * pg_hof_rank_classes_workspace_bytes(hof_n + k). */
typedef struct pg_hof_rank_args {
  int32_t hof_n;
  const double *hof_fitness;     /* [hof_n] device, items order */
  const uint64_t *hof_hash;      /* [hof_n] device */
  int32_t k;
  const double *cand_fitness;    /* [k] device, population order */
  const uint64_t *cand_hash;     /* [k] device */
  int64_t *packed;               /* out [hof_n + 2k] device */
  void *workspace;
  size_t workspace_bytes;
} pg_hof_rank_args;

/* The whole device half of the hall-of-fame update (pg_hof_prepare): the
 * candidates (every row, or with filter the rows whose fitness is strictly
 * above worst -- a full hall's admission rule), their row hashes, and the
 * pg_hof_rank_classes packing of members + candidates.  One host sync (the
 * candidate count, written to *k).  Device pointers on the stream's device;
 * workspace >= pg_hof_prepare_workspace_bytes(hof_n, pop_n). */
typedef struct pg_hof_prepare_args {
  const double *fitness;         /* [pop_n] device, population order */
  int32_t pop_n;
  int32_t filter;                /* 1: candidates are fitness > worst; 0: every row */
  double worst;
  const void *rows;              /* [pop_n, stride] device, dtype */
  int64_t stride;
  int64_t genes;
  int32_t dtype;
  int32_t hof_n;
  const double *hof_fitness;     /* [hof_n] device, items order */
  const uint64_t *hof_hash;      /* [hof_n] device */
  int32_t *k;                    /* out (host): number of candidates */
  int64_t *cand;                 /* out [pop_n] device: candidate rows, population order */
  uint64_t *hashes;              /* out [hof_n + pop_n] device: members', then candidates' hashes */
  int64_t *packed;               /* out [hof_n + 2 pop_n] device: as pg_hof_rank_classes (n = hof_n + k) */
  void *workspace;
  size_t workspace_bytes;
} pg_hof_prepare_args;

const char *pg_version(void);
int32_t pg_abi_version(void);
/* Build options of this library (0: no optional features; the retired layouts
 * PG_KERNEL_RESIDENT / PG_KERNEL_STAGED are never compiled in). */
int32_t pg_build_flags(void);
const char *pg_last_error(void);
/* Number of visible HIP devices (>= 0), or a negative pg_status. */
int32_t pg_device_count(void);
size_t pg_eval_workspace_bytes(const pg_eval_args *args);
int32_t pg_gene_count(const pg_net *net);

int32_t pg_eval_population(const pg_eval_args *args, void *stream);
int32_t pg_forward(const pg_forward_args *args, void *stream);
int32_t pg_decide(const pg_decide_args *args, void *stream);
size_t pg_wide_decide_workspace_bytes(const pg_wide_decide_args *args);
int32_t pg_wide_decide(const pg_wide_decide_args *args, void *stream);
int32_t pg_physics_reset(int32_t *state, int32_t n, const uint64_t *seeds,
                         const int32_t *one_player, void *stream);
/* actions [n]: bit0 right up, bit1 right down, bit2 left up, bit3 left down */
int32_t pg_physics_step(int32_t *state, int32_t n, const uint8_t *actions, void *stream);
int32_t pg_ga_select_tournament(const pg_select_args *args, void *stream);
/* selTournament for large tournsize by rank sampling: the winner of a
 * tournament of t draws with replacement has ascending rank floor(n V^(1/t))
 * (V uniform), ties resolved uniformly -- the same distribution as the
 * draw-by-draw tournament.  sorted_fitness ascending, order[r] = row of rank r. */
int32_t pg_ga_select_tournament_ranked(const pg_select_args *args, const double *sorted_fitness,
                                       const int32_t *order, void *stream);
int32_t pg_ga_vary(const pg_ga_args *args, void *stream);
/* pair_mask[rows[i] >> 1] = 1 for i < n_rows, except pairs in [skip_lo, skip_hi)
 * and pairs j with exclude[j] != 0 (exclude [n_pairs] or NULL; mask [n_pairs];
 * rows outside [0, 2 n_pairs) are skipped). */
int32_t pg_ga_mark_pairs(uint8_t *pair_mask, int32_t n_pairs, const int32_t *rows, int32_t n_rows,
                         int32_t skip_lo, int32_t skip_hi, const uint8_t *exclude, void *stream);
/* list[0 .. *count) = the pairs j with pair_mask[j] != 0, in no particular order
 * (*count set by the call; list [n_pairs] or at least as long as the marks). */
int32_t pg_ga_list_pairs(const uint8_t *pair_mask, int32_t n_pairs, int32_t *list, int32_t *count, void *stream);
int32_t pg_ga_schedule(const pg_schedule_args *args, void *stream);
/* hash[i] = 64-bit hash of the genes of row index[i] (row i if index is NULL):
 * f32/f64 bit patterns, -0.0 as 0.0, so equal gene lists hash equal. */
int32_t pg_row_hash(const void *rows, int64_t stride, const int32_t *index, int32_t n, int64_t genes,
                    int32_t dtype, uint64_t *hash, void *stream);
/* Host only (no device memory, no GPU needed). */
int32_t pg_hof_update(const pg_hof_args *args);
size_t pg_hof_rank_classes_workspace_bytes(int32_t n);
int32_t pg_hof_rank_classes(const pg_hof_rank_args *args, void *stream);
size_t pg_hof_prepare_workspace_bytes(int32_t hof_n, int32_t pop_n);
int32_t pg_hof_prepare(const pg_hof_prepare_args *args, void *stream);
/* ---- one eaSimple generation around the evaluation (DeviceGA; DEAP's eaSimple,
 * main.py:165-170, operators ga.py:89-94).  Device pointers on the stream's
 * device; each call is stream-ordered and syncs nothing. ---- */

/* The evaluation's results in the shard's row order (toolbox.map's results
 * assigned to invalid_ind, eaSimple): entry i (< *n_active, or every entry
 * when n_active is NULL) played population row rows[i] (NULL: row_lo + i):
 * shard_fitness[rows[i] - row_lo] = fitness[i] and, when lineage is given,
 * lineage[rows[i]] = max over games of frames[i][g] (the evaluation order's
 * prediction); shard rows no entry played read 0.  rows must be a permutation
 * of the shard's rows. */
typedef struct pg_scatter_args {
  int32_t n;                     /* entries = shard rows */
  int32_t n_games;
  int32_t row_lo;                /* the shard's first population row */
  const double *fitness;         /* [n] k_fitness' results */
  const int32_t *frames;         /* [n, n_games] */
  const int32_t *rows;           /* [n] or NULL */
  const int32_t *n_active;       /* [1] device or NULL */
  double *shard_fitness;         /* out [n] */
  float *lineage;                /* in/out [row_lo + n] or NULL */
} pg_scatter_args;
int32_t pg_ga_scatter_fitness(const pg_scatter_args *args, void *stream);

/* The generation's fitness: new_fitness[i] = invalid[i] ? fitness[i] :
 * inherited[i] (varAnd's clones keep their parent's fitness; invalid NULL:
 * every row evaluated), the logbook statistics of main.py:158-162 and the
 * hall-of-fame candidates -- rows with new_fitness > worst (filter: a full
 * hall admits only those, HallOfFame.update) or every row -- in ascending row
 * order.  summary[8] = {any NaN (calculate_reward's ZeroDivisionError,
 * utils.py:106-108), mean, std (ddof 0), min, max over the non-NaN values,
 * nevals (rows evaluated), k (candidates), 0}; every reduction in a fixed
 * order (reproducible).  new_fitness may alias fitness. */
typedef struct pg_merge_args {
  int32_t pop_n;
  const double *fitness;         /* [pop_n] evaluated fitness (gathered over ranks) */
  const uint8_t *invalid;        /* [pop_n] or NULL */
  const double *inherited;       /* [pop_n] (read where invalid[i] == 0) */
  double *new_fitness;           /* out [pop_n] */
  int32_t filter;
  double worst;
  int32_t *cand;                 /* out [pop_n]: the first k entries */
  double *cand_fitness;          /* out [pop_n] */
  double *summary;               /* out [8] device */
  void *workspace;               /* >= pg_ga_merge_workspace_bytes(pop_n) */
  size_t workspace_bytes;
} pg_merge_args;
size_t pg_ga_merge_workspace_bytes(int32_t pop_n);
int32_t pg_ga_merge_fitness(const pg_merge_args *args, void *stream);

/* pg_ga_select_tournament_ranked with its stable fitness sort inside (one call). */
size_t pg_ga_select_workspace_bytes(int32_t n_pop);
int32_t pg_ga_select_ranked(const pg_select_args *args, void *workspace, size_t workspace_bytes, void *stream);

/* What offspring slot i inherits from its parent chosen[i] (varAnd clones the
 * chosen individuals): inherited[i] = fitness[chosen[i]] and lineage_out[i] =
 * lineage_in[chosen[i]]; either output may be NULL. */
int32_t pg_ga_inherit(const int32_t *chosen, int32_t n, const double *fitness, double *inherited,
                      const float *lineage_in, float *lineage_out, void *stream);

/* A shard's evaluation order (which rows toolbox.map(evaluate, invalid_ind)
 * plays, main.py:165-170, and in what order): rows[0, *count) = the shard's
 * invalid rows (invalid NULL: all), by_length: the longest lineage[row] first,
 * ties by row; then the valid rows (clones) by row.  invalid and lineage are
 * indexed by population row. */
size_t pg_ga_order_workspace_bytes(int32_t n);
int32_t pg_ga_order(int32_t n, int32_t row_lo, const uint8_t *invalid, const float *lineage, int32_t by_length,
                    int32_t *rows, int32_t *count, void *workspace, size_t workspace_bytes, void *stream);

/* HallOfFame.update's scan input for k known candidates (pg_ga_merge_fitness'
 * cand list): their pg_row_hash values, and the packing of pg_hof_rank_classes
 * -- ranks from a sort of the candidates alone plus binary searches into the
 * members' items order, dense classes (a member's: the first member of equal
 * hash; a candidate's: that member, else hof_n + the first candidate of equal
 * hash) from two hash tables. */
typedef struct pg_hof_cand_args {
  int32_t hof_n;
  const double *hof_fitness;     /* [hof_n] items order (descending) */
  const uint64_t *hof_hash;      /* [hof_n] */
  int32_t k;
  const int32_t *cand;           /* [k] population rows, ascending */
  const double *cand_fitness;    /* [k] */
  const void *rows;              /* [*, stride] population rows, dtype */
  int64_t stride;
  int64_t genes;
  int32_t dtype;
  uint64_t *cand_hash;           /* out [k] */
  int64_t *packed;               /* out [hof_n + 2k] */
  void *workspace;               /* >= pg_hof_prepare_cand_workspace_bytes(hof_n, k) */
  size_t workspace_bytes;
} pg_hof_cand_args;
size_t pg_hof_prepare_cand_workspace_bytes(int32_t hof_n, int32_t k);
int32_t pg_hof_prepare_cand(const pg_hof_cand_args *args, void *stream);

/* The new hall (HallOfFame.insert's deepcopy of each entrant): member j from
 * pg_hof_update's new_src[j] = src[j]: old member src[j] < n_old (rows
 * old_rows, hash old_hash) or candidate c = src[j] - n_old (population row
 * cand[c], hash cand_hash[c]); new_fitness[j] = fitness_in[j].  Outputs
 * disjoint from the inputs. */
typedef struct pg_hof_commit_args {
  void *dst;
  int64_t dst_stride;
  const void *old_rows;
  int64_t old_stride;
  const void *rows;
  int64_t rows_stride;
  const int32_t *cand;
  const int32_t *src;            /* [m] device */
  int32_t n_old;
  int32_t m;
  int64_t genes;
  int32_t dtype;
  const uint64_t *old_hash;
  const uint64_t *cand_hash;
  uint64_t *new_hash;            /* out [m] */
  const double *fitness_in;      /* [m] device */
  double *new_fitness;           /* out [m] */
  /* ABI 12: dst_slot [m] device (NULL: member j's row is dst row j).  Non-NULL:
   * the hall in place -- dst is the hall's storage, member j's row is dst row
   * dst_slot[j] (pg_hof_packed_args.slot_out), and only entering candidates'
   * rows are written (a kept member's row is already in its slot; old_rows is
   * not read).  Hashes and fitness are written by position as without it. */
  const int32_t *dst_slot;
} pg_hof_commit_args;
int32_t pg_hof_commit(const pg_hof_commit_args *args, void *stream);

/* dst row j = old_rows[src[j]] if src[j] < n_old, else rows[index[src[j] - n_old]]
 * (index NULL: rows[src[j] - n_old]) -- pg_hof_update's new_src applied in one
 * pass; strides in elements, dst disjoint from both sources. */
int32_t pg_gather_rows(void *dst, int64_t dst_stride, const void *old_rows, int64_t old_stride, const void *rows,
                       int64_t rows_stride, const int64_t *index, const int32_t *src, int32_t n_old, int32_t n,
                       int64_t genes, int32_t dtype, void *stream);
/* frames [n, 210, 160, 3] uint8 (16-byte aligned) from the SoA state [PG_STATE_FIELDS, n]:
 * background, the walls above/below the playfield, both paddles, the ball if visible. */
int32_t pg_render_frames(const int32_t *state, int32_t n, uint8_t *frames, void *stream);
/* out [n, 3, 2] f64: find_stuff's (row, col) centroids of the ball, left and right
 * colours in the crop rows 34..193, matched per channel as get_rect_quickly does;
 * NaN for None.  frame_stride in bytes (>= 100800, multiple of 16). */
int32_t pg_find_stuff(const uint8_t *frames, int64_t frame_stride, int32_t n, double *out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PONG_GA_H */
