// pg_eval.hpp -- what the evaluation kernels of libpong_ga.so share across
// translation units (pong_ga.hip: the small-network kernels and the C-ABI;
// pg_wide.hip: the streaming kernel for wide two-hidden-layer networks).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pong_ga.h"
#include "pg_device.hpp"

namespace pg {

// Record a failure for pg_last_error() and return code (defined in pong_ga.hip).
int32_t fail(int32_t code, const char *fmt, ...);

#define PG_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(PG_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(e_));        \
  } while (0)

// ------------------------------------------------------- kernel params ----
struct EvalParams {
  const void *genomes;
  const void *opponents;
  const int32_t *rows;  // optional [n_genomes]: block i of games plays genome row rows[i] (NULL: row i)
  const int32_t *n_active;  // optional device count: only blocks i < min(*n_active, n_genomes) are played
  const int32_t *kind;
  const int32_t *opp;
  const double *mult;
  double *rewards;
  int32_t *scores;
  int32_t *frames;
  double *total_frames;
  int32_t *status_game;  // [n*games] scratch: zero-division per game
  uint64_t *counters;
  uint8_t *trace;
  uint32_t *hard_log;    // optional [hard_cap][8] (pg_eval_args.hard_log)
  int hard_cap;
  unsigned int *work;    // dynamic game counter (workspace)
  int64_t gstride, ostride;
  uint64_t seed;
  int n_genomes, n_games, total, n_opponents;
  int trace_games, trace_cap;
  int nodes[PG_MAX_NODES];
  int n_nodes, bias, max_width;
  float *recs;         // split kernel: lane records (k_prep_records), [n_genomes + n_opponents][L/2][rec_floats]
  int horizon;         // pg_eval_args.horizon: fixed-horizon measurement mode (T frames per game slot), 0 = off
  int timeout_thresh;  // pg_eval_args.timeout_thresh: TIMEOUT_THRESH (kTimeoutThresh unless set)
  int win_score;       // pg_eval_args.win_score: WIN_SCORE (kWinScore unless set)
  int prep;            // pg_prep: which records k_prep_records writes; it also zeroes the work header and
                       // the counters when its launch precedes the games (PG_PREP_ALL / PG_PREP_REST)
  void *wide_scratch;  // k_wide: the blocks' tile-major W2 copies (workspace)
  int wide_w3_resident;  // k_wide: every network's W3 kept in LDS for the genome's games
  // k_wide probe (pg_wide_decide, n_games = 1): block i runs one frame of
  // genome i on the doubled centroids wide_probe_k[i][0..5] instead of a game
  const int32_t *wide_probe_k;
  int32_t *wide_probe_index;  // out [n_genomes] np.argmax
  double *wide_probe_act;     // optional out [n_genomes, nodes[3]]
};

// Genome blocks / games this launch plays (pg_eval_args.n_active).  Made
// wave-uniform explicitly: as a per-lane load result the loop bound of the
// game loops became a vector compare, which cost k_service 14 % (11.0 vs
// 12.7 ms per launch, tools/runs/r2_b6.sh).
__device__ inline int active_genomes(const EvalParams &p) {
  if (!p.n_active) return p.n_genomes;
  const int a = __builtin_amdgcn_readfirstlane(*p.n_active);
  return a < 0 ? 0 : (a < p.n_genomes ? a : p.n_genomes);
}
__device__ inline int active_total(const EvalParams &p) {
  return p.n_active ? active_genomes(p) * p.n_games : p.total;
}

// Genome row played by block i of games (pg_eval_args.genome_rows).
__device__ inline int genome_row(const EvalParams &p, int i) { return p.rows ? p.rows[i] : i; }

// Results of one finished game: perform_episode's return value and the
// bookkeeping around it (main.py:108-112, utils.py:104-109).
// (S: Pong or PongK; only the scores are read)
template <class S>
__device__ inline double episode_reward(const S &st, int total, double mult, int &zero_div) {
  zero_div = 0;
  if (st.s1 == st.s2) return 0.0;  // main.py:109-110
  const double tf = (double)total;
  if (tf == 0.0) {
    zero_div = 1;
    return __builtin_nan("");
  }
  // ((my - enemy) + my * mult) / (total_frames / 100.0), no contraction
  const double diff = (double)(st.s2 - st.s1);
  const double bonus = __dmul_rn((double)st.s2, mult);
  return __dadd_rn(diff, bonus) / (tf / 100.0);
}

template <class S>
__device__ inline void finish_game(const EvalParams &p, int w, const S &st, int frames, int total) {
  int zero_div;
  const double reward = episode_reward(st, total, p.mult[w], zero_div);
  p.rewards[w] = reward;
  p.scores[2 * w] = st.s1;
  p.scores[2 * w + 1] = st.s2;
  p.frames[w] = frames;
  p.total_frames[w] = (double)total;
  p.status_game[w] = zero_div;
}

// Features of utils.inference (utils.py:139-153) in f64 from doubled
// centroids k: value = (k / 2) / 160, exactly the reference's rounding.
__device__ inline double feat64(int k) { return __dmul_rn(0.5, (double)k) / 160.0; }
__device__ inline double feat64_flip(int k) { return (160.0 - __dmul_rn(0.5, (double)k)) / 160.0; }


int num_cus();

// Append one hard-decision record (pg_eval_args.hard_log); counters[9] counts them all.
__device__ inline void log_hard_raw(uint32_t *hard_log, uint64_t *counters, int hard_cap, int row, int is_opp, int idx,
                                    int source, const int k[6]) {
  if (!hard_log || !counters) return;
  const unsigned long long r = atomicAdd((unsigned long long *)&counters[9], 1ull);
  if (r >= (unsigned long long)hard_cap) return;
  uint32_t *rec = hard_log + r * 8;
  rec[0] = (uint32_t)row;
  rec[1] = (uint32_t)(is_opp & 1) | ((uint32_t)(idx & 255) << 8) | ((uint32_t)(source & 255) << 16);
  for (int i = 0; i < 6; ++i) rec[2 + i] = (uint32_t)k[i];
}
__device__ inline void log_hard(const EvalParams &p, int row, int is_opp, int idx, int source, const int k[6]) {
  log_hard_raw(p.hard_log, p.counters, p.hard_cap, row, is_opp, idx, source, k);
}

// pg_decide's parameters (k_decide, pg_decide.hip: k_service's cascade on given inputs)
struct DecideParams {
  const void *genomes;
  const int32_t *gidx;
  const int32_t *k;
  int32_t *index;
  int32_t *stage;
  int64_t gstride;
  int n, H, b;
};
// k_decide for the split layout of L lanes per game (pg_decide.hip; its own
// translation unit, on the default machine scheduler: the iterative-ILP one
// pong_ga.hip uses for k_service crashes the register allocator on k_decide)
int32_t launch_decide(const DecideParams &p, int L, int O, bool f64, size_t lds, hipStream_t s);

// [6, H1, H2, O] networks (two hidden layers, H1, H2 <= 512, O in 2..4,
// n_games <= 8) on the weight-streaming kernel k_wide (pg_wide.hip).
bool wide_shape_ok(const pg_net &n, int n_games);
size_t wide_workspace_bytes(const pg_eval_args *a);
int32_t launch_wide(const EvalParams &p, int dtype, void *scratch, hipStream_t s);


}  // namespace pg
