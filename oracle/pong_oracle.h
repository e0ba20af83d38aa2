/*
 * pong_oracle.h -- CPU ORACLE for the GA evaluation loop.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path may include, link
 * or call this code: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU baseline.
 *
 * It is a plain-C restatement of the reference's per-genome evaluation
 * (n00b001/neuro-genetic-pong-self-play):
 *   - NeuralNetwork.run            numpy_nn.py:120-137  (f64, sigmoid = 1/(1+e**-x) numpy_nn.py:22-23;
 *                                  np.dot in OpenBLAS dgemv_t's order, or_blas_dot)
 *   - populate_weights layout      numpy_nn.py:52-69
 *   - inference features           utils.py:139-153
 *   - get_actions                  main.py:138-154
 *   - keep_within_game_bounds      utils.py:71-77
 *   - calculate_timeout_and_frames main.py:128-135
 *   - perform_episode loop         main.py:69-112
 *   - calculate_reward             utils.py:104-109
 *   - evaluate (6-game average)    main.py:28-66
 *   - HardcodedAi / ScoreHardcodedAi dumb_ais.py:1-25
 * plus the build's own integer Pong physics (the reference steps the gym-retro
 * Atari emulator, main.py:77, which is third-party and absent; see DESIGN.md
 * "Physics").  The policy side is pinned against golden vectors generated from
 * the real reference code (tests/golden/make_golden.py); the physics is pinned
 * only by this restatement (parity for the emulator itself is unpinned).
 */
#ifndef PONG_ORACLE_H
#define PONG_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- geometry of the cropped 160x160 playfield (obs.npy, rows 34..193) ---- */
#define OR_FIELD_W 160
#define OR_FIELD_H 160
#define OR_PADDLE_H 16
#define OR_PADDLE_W 4
#define OR_LEFT_PADDLE_X 16
#define OR_RIGHT_PADDLE_X 140
#define OR_BALL_H 4
#define OR_BALL_W 2
#define OR_PADDLE_Y_MIN (-8)
#define OR_PADDLE_Y_MAX 152
#define OR_PADDLE_SPEED 3
#define OR_CPU_SPEED 2
#define OR_SERVE_DELAY 30
#define OR_BALL_VX0 2
#define OR_BALL_VX_MAX 4
#define OR_DONE_SCORE 21

/* ---- episode constants (config.py) ---- */
#define OR_WIN_SCORE 3          /* config.py:53 */
#define OR_TIMEOUT_THRESH 2000  /* config.py:28 */
/* The episode limits every later or_play_* call uses (perform_episode's
 * termination, main.py:102-107; pg_eval_args.timeout_thresh / win_score):
 * 0 restores the reference's values above.  Not thread-safe: set it before
 * the calls, not during a parallel evaluation. */
void or_set_limits(int timeout_thresh, int win_score);

/* opponent kinds for the LEFT paddle (the genome always plays the right paddle) */
enum {
  OR_OPP_HARDCODED = 0, /* HardcodedAi, 2-player env            main.py:52-53 */
  OR_OPP_ROM_CPU = 1,   /* 1-player env, built-in CPU on the left main.py:39-40 */
  OR_OPP_SCORE = 2,     /* ScoreHardcodedAi                      main.py:41-42 */
  OR_OPP_NN = 3         /* NeuralNetwork from the hall of fame   main.py:43-49 */
};

typedef struct {
  int ball_x, ball_y, ball_vx, ball_vy;
  int ball_visible, serve_timer, serve_dir, hits, point;
  int lpy, rpy;
  int score1, score2;
  int one_player;
  uint64_t seed;
} or_pong_state;

typedef struct {
  int n_nodes;        /* len(NETWORK_SHAPE) */
  const int *nodes;   /* NETWORK_SHAPE; nodes[0] must be 6 for the game loop */
  int bias;           /* BIAS */
} or_net;

typedef struct {
  int score1, score2;
  int frames;           /* env.step calls made */
  double total_frames;  /* main.py:73,133 accumulator */
  double reward;        /* perform_episode return value */
  int zero_division;    /* 1 if the reference would raise ZeroDivisionError */
  int slow_decisions;   /* unused by the oracle (kept for struct symmetry) */
} or_game_result;

uint64_t or_splitmix64(uint64_t x);
uint64_t or_game_seed(uint64_t base_seed, int game_index);

void or_env_reset(or_pong_state *s, uint64_t game_seed, int one_player);
/* One env.step(action): right paddle [up,down] = action[4:6], left = action[6:8]. */
void or_env_step(or_pong_state *s, int r_up, int r_dn, int l_up, int l_dn);
int or_env_done(const or_pong_state *s);

int or_gene_count(const or_net *net);
/* numpy_nn.NeuralNetwork.run: returns argmax index; writes the final-layer
 * activations (len nodes[last]) into out_act if non-NULL. */
/* np.dot(W, x) for a C-contiguous [n, m] float64 W, in the operation order of
 * numpy's OpenBLAS dgemv_t (x86-64 AVX2/FMA kernel); see pong_oracle.c. */
double or_blas_dot(const double *a, const double *x, int m, int j, int n);
void or_blas_gemv(const double *w, int n, int m, const double *x, double *y);
int or_nn_run(const double *genes, const or_net *net, const double *x, double *out_act);

/* One perform_episode.  genes: right-paddle genome; opp_genes: left genome for
 * OR_OPP_NN.  trace (optional): per frame one byte = right_code | left_code<<2
 * | visible<<4, codes 0=[0,0] 1=[1,0] 2=[0,1]. */
void or_play_game(const double *genes, const or_net *net, int opp_kind,
                  const double *opp_genes, double mult, uint64_t game_seed,
                  or_game_result *out, uint8_t *trace, int trace_cap);

/* One game slot: horizon <= 0 is or_play_game; horizon T > 0 the fixed-horizon
 * measurement mode of pg_eval_args.horizon (T frames, auto-reset, see there). */
void or_play_slot(const double *genes, const or_net *net, int opp_kind, const double *opp_genes, double mult,
                  uint64_t game_seed, int horizon, or_game_result *out, uint8_t *trace, int trace_cap);

/* A whole population: games per genome = n_games; kind/opp/mult are
 * [n, n_games]; opponents[opp_index * stride ...]; fitness = evaluate().
 * n_threads <= 0 means serial.  Returns 0, or the 1-based index of the first
 * genome whose evaluation would raise ZeroDivisionError (outputs still filled). */
int or_eval_population(int n, int n_games, const double *genomes, int64_t stride,
                       const double *opponents, int64_t opp_stride,
                       const int32_t *kind, const int32_t *opp_index,
                       const double *mult, const or_net *net, uint64_t base_seed,
                       double *fitness, double *rewards, int32_t *scores,
                       int32_t *frames, double *total_frames, int32_t *status,
                       int n_threads);
/* The same with every game slot in the fixed-horizon mode (horizon > 0). */
int or_eval_population_h(int n, int n_games, const double *genomes, int64_t stride,
                         const double *opponents, int64_t opp_stride,
                         const int32_t *kind, const int32_t *opp_index,
                         const double *mult, const or_net *net, uint64_t base_seed, int horizon,
                         double *fitness, double *rewards, int32_t *scores,
                         int32_t *frames, double *total_frames, int32_t *status,
                         int n_threads);

/* ---- pixel path (utils.py:14-19, 60-68; the build's frame of its state) ---- */
#define OR_FRAME_BYTES (210 * 160 * 3)
/* The 210x160x3 frame of a state in config.py colours: background, walls at
 * rows 24..33 and 194..209, both paddles clipped to the playfield, the ball. */
void or_render(const or_pong_state *s, uint8_t *frame);
/* find_stuff: out[0..5] = ball, left, right (row, col) centroids over the crop
 * rows 34..193, matched per channel (get_rect_quickly); NaN for None. */
void or_find_stuff(const uint8_t *frame, double *out);

#ifdef __cplusplus
}
#endif
#endif
