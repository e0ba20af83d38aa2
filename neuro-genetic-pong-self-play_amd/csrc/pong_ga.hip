// pong_ga.hip -- MI355X (gfx950) kernels and the C-ABI of libpong_ga.so.
//
// The hot path: evaluate() (main.py:28-66) for a whole population in one
// launch.  Every game (perform_episode, main.py:69-112) runs to termination
// inside the kernel: the Pong state and both networks' weights stay in
// registers for the whole episode, so HBM is touched once per game (weights
// in, results out) instead of once per frame.  See DESIGN.md.
//
//   k_service<L,U,O,WT>   [6, H<=256, O] networks (pg_service.hpp): an aligned
//                         group of L lanes plays one game, half a group per
//                         paddle's network in VGPRs; f32 math with a certified
//                         f64 argmax, the failures re-decided in f64 by the
//                         wave itself (8-lane groups) or a service wave.
//   k_general<WT>         any NETWORK_SHAPE, one wave per game, f64 numpy_nn
//                         arithmetic with activations staged in LDS.
//   k_fitness             sum(all_rewards) / GAMES_TO_PLAY in the reference order.
//   k_forward_*           NeuralNetwork.run batched (parity entry point).
//   k_physics_*           the SoA Pong stepper on its own.
//   k_select / k_vary     DEAP selTournament / varAnd(cxBlend, mutGaussian).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <algorithm>
#include <memory>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/pong_ga.h"
#include "pg_device.hpp"
#include "pg_eval.hpp"
#include "pg_f64math.h"
#include "pg_cascade.hpp"
#include "pg_service.hpp"

#ifndef PG_VERSION_STRING
#define PG_VERSION_STRING "pong_ga 0.1.0 (gfx950)"
#endif

namespace pg {

// --------------------------------------------------------------- errors ----
static thread_local std::string g_last_error;

int32_t fail(int32_t code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}


// ===================================================== general (f64) path ==
// One forward pass of NeuralNetwork.run (numpy_nn.py:120-137) by one wave, in
// f64 with numpy's operation order per unit (np.dot's BLAS order over
// [inputs..., 1], blas_dot); cur holds the input vector (with the trailing 1 if
// bias).  Returns the argmax index; cur/nxt are LDS buffers of max_width + 1
// doubles.  With z_all/h_all (pg_forward's diagnostics) every layer's
// pre-activations and activations are stored there as well.
template <typename WT>
__device__ int forward_f64_wave(const WT *__restrict__ w, const int *nodes, int n_nodes, int b,
                                double *&cur, double *&nxt, int lane, double *z_all = nullptr,
                                double *h_all = nullptr) {
  long off = 0;
  int zo = 0;
  for (int l = 0; l + 1 < n_nodes; ++l) {
    const int nin = nodes[l], nout = nodes[l + 1], cols = nin + b;
    for (int j = lane; j < nout; j += 64) {
      const WT *row = w + off + (long)j * cols;
      const double *cv = cur;
      const double z = blas_dot([&](int i) { return (double)row[i]; }, [&](int i) { return cv[i]; }, cols,
                                blas_kind(j, nout));
      nxt[j] = sigmoid_f64(z);
      if (z_all) z_all[zo + j] = z;
      if (h_all) h_all[zo + j] = nxt[j];
    }
    zo += nout;
    if (b && lane == 0) nxt[nout] = 1.0;
    wave_lds_sync();
    off += (long)cols * nout;
    double *t = cur;
    cur = nxt;
    nxt = t;
  }
  const int n_out = nodes[n_nodes - 1];
  int best = 0;  // np.argmax: the first NaN if any, else the first maximum
  for (int j = 1; j < n_out && !__builtin_isnan(cur[best]); ++j)
    if (__builtin_isnan(cur[j]) || cur[j] > cur[best]) best = j;
  return best;
}

template <typename WT>
__global__ __launch_bounds__(64) void k_general(EvalParams p) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x;
  const int W = p.max_width + 1;
  double *bufA = lds, *bufB = lds + W;
  const WT *genomes = (const WT *)p.genomes;
  const WT *opponents = (const WT *)p.opponents;
  uint64_t c_steps = 0, c_fwd = 0, c_games = 0;
  const int games_total = active_total(p);
  for (;;) {
    int w = 0;
    if (lane == 0) w = (int)atomicAdd(p.work, 1u);
    w = __builtin_amdgcn_readfirstlane(w);
    if (w >= games_total) break;
    const int i = w / p.n_games, g = w % p.n_games;
    const int kind = p.kind[w];
    const WT *gr = genomes + (long)genome_row(p, i) * p.gstride;
    const WT *gl = (kind == kOppNN) ? opponents + (long)p.opp[w] * p.ostride : gr;
    Pong st;
    st.reset(game_seed(p.seed, g), kind == kOppRomCpu);
    int act_r = 0, act_l = 0, timeout = 0, total = 0, frames = 0;
    for (;;) {
      const int s1b = st.s1, s2b = st.s2;
      const int pvis = st.vis, pbx2 = 2 * st.bx + kBallW - 1, pby2 = 2 * st.by + kBallH - 1;
      st.step(act_r, act_l);
      frames += 1;
      const int vis = st.vis;
      const int bx2 = 2 * st.bx + kBallW - 1, by2 = 2 * st.by + kBallH - 1;
      const int lc2 = paddle_c2(st.lpy), rc2 = paddle_c2(st.rpy);
      int left = 0, right = 0;
      if (vis) {  // get_actions main.py:143-150
        const int lbx2 = pvis ? pbx2 : bx2, lby2 = pvis ? pby2 : by2;
        if (kind == kOppNN) {
          double *cur = bufA, *nxt = bufB;
          if (lane == 0) {
            cur[0] = feat64_flip(bx2); cur[1] = feat64(by2); cur[2] = feat64_flip(lbx2);
            cur[3] = feat64(lby2); cur[4] = feat64(lc2); cur[5] = feat64(rc2);
            if (p.bias) cur[6] = 1.0;
          }
          wave_lds_sync();
          left = index_to_code(forward_f64_wave(gl, p.nodes, p.n_nodes, p.bias, cur, nxt, lane));
          wave_lds_sync();
          c_fwd += 1;
        } else if (kind == kOppScore) {
          left = (st.s1 <= st.s2) ? hardcoded(by2, lc2) : 0;
        } else {
          left = hardcoded(by2, lc2);
        }
        double *cur = bufA, *nxt = bufB;
        if (lane == 0) {
          cur[0] = feat64(bx2); cur[1] = feat64(by2); cur[2] = feat64(lbx2);
          cur[3] = feat64(lby2); cur[4] = feat64(rc2); cur[5] = feat64(lc2);
          if (p.bias) cur[6] = 1.0;
        }
        wave_lds_sync();
        right = index_to_code(forward_f64_wave(gr, p.nodes, p.n_nodes, p.bias, cur, nxt, lane));
        wave_lds_sync();
        c_fwd += 1;
      }
      act_l = clamp_action(lc2, left);
      act_r = clamp_action(rc2, right);
      if (p.trace && w < p.trace_games && frames <= p.trace_cap && lane == 0)
        p.trace[(long)w * p.trace_cap + frames - 1] = (uint8_t)(act_r | (act_l << 2) | (vis << 4));
      if (frames > 1) {  // calculate_timeout_and_frames main.py:128-135
        if (st.s1 == s1b && st.s2 == s2b) {
          timeout += 1;
        } else {
          total += timeout;
          timeout = 0;
        }
      }
      if (st.s1 >= p.win_score || st.s2 >= p.win_score || st.done() || timeout > p.timeout_thresh) break;
    }
    c_steps += frames;
    c_games += 1;
    if (lane == 0) finish_game(p, w, st, frames, total);
  }
  if (p.counters && lane == 0 && c_games) {
    atomicAdd((unsigned long long *)&p.counters[0], (unsigned long long)c_steps);
    atomicAdd((unsigned long long *)&p.counters[1], (unsigned long long)c_fwd);
    atomicAdd((unsigned long long *)&p.counters[3], (unsigned long long)c_games);
  }
}

// ------------------------------------------------------------- fitness ----
// evaluate()'s return: sum(all_rewards) (left to right from int 0) / float(GAMES_TO_PLAY).
__global__ void k_fitness(const double *rewards, const int32_t *status_game, int n, const int32_t *n_active,
                          int games, double *fitness, int32_t *status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (n_active && i >= *n_active)) return;  // rows not played keep their contents
  double s = 0.0;
  int err = 0;
  for (int g = 0; g < games; ++g) {
    s = __dadd_rn(s, rewards[(long)i * games + g]);
    err |= status_game[(long)i * games + g];
  }
  fitness[i] = s / (double)games;
  if (status) status[i] = err;
}

// ============================================================ forward ====
struct FwdParams {
  const void *genomes;
  const int32_t *gidx;
  const double *x;
  int32_t *index;
  double *act;
  double *z_all, *h_all;  // optional [n, sum(nodes[1:])]: every layer's pre-activations / activations
  uint64_t *counters;
  int64_t gstride;
  int n;
  int nodes[PG_MAX_NODES];
  int n_nodes, bias, max_width, n_units;
};

template <typename WT>
__global__ __launch_bounds__(64) void k_forward_general(FwdParams p) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x;
  const int W = p.max_width + 1;
  const int n_in = p.nodes[0], n_out = p.nodes[p.n_nodes - 1];
  for (int t = blockIdx.x; t < p.n; t += gridDim.x) {
    const long row = p.gidx ? p.gidx[t] : t;
    const WT *gw = (const WT *)p.genomes + row * p.gstride;
    double *cur = lds, *nxt = lds + W;
    for (int i = lane; i < n_in; i += 64) cur[i] = p.x[(long)t * n_in + i];
    if (p.bias && lane == 0) cur[n_in] = 1.0;
    wave_lds_sync();
    const int idx = forward_f64_wave(gw, p.nodes, p.n_nodes, p.bias, cur, nxt, lane,
                                     p.z_all ? p.z_all + (long)t * p.n_units : nullptr,
                                     p.h_all ? p.h_all + (long)t * p.n_units : nullptr);
    if (lane == 0) p.index[t] = idx;
    if (p.act)
      for (int j = lane; j < n_out; j += 64) p.act[(long)t * n_out + j] = cur[j];
    wave_lds_sync();
  }
}

template <int L, int U, int O, typename WT>
__global__ __launch_bounds__(256) void k_forward_resident(FwdParams p) {
  constexpr int GPB = 256 / L;
  const int H = p.nodes[1], b = p.bias;
  extern __shared__ double lds_all[];
  const int lig = threadIdx.x & (L - 1);
  const int grp = threadIdx.x / L;
  double *lds = lds_all + grp * f64_lds_doubles(H, O);
  uint32_t slow = 0;
  for (int t = blockIdx.x * GPB + grp; t < p.n; t += gridDim.x * GPB) {
    const long row = p.gidx ? p.gidx[t] : t;
    const WT *gw = (const WT *)p.genomes + row * p.gstride;
    Net<U, O> net;
    load_net<L, U, O, WT>(net, gw, H, b, lig);
    float x[6], acc[O], z[O];
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = (float)p.x[(long)t * 6 + i];
    partial_f32<U, O>(net, x, acc);
#pragma unroll
    for (int o = 0; o < O; ++o) z[o] = group_sum<L>(acc[o]) + net.c[o];
    int idx = certify<O>(z, net.e);
    if (idx >= 0 && p.act) {
      // activations are reported within 2e-6: |S(z) - S(z_hat)| <= e * S'(max(|z_hat| - e, 0))
      bool tight = true;
#pragma unroll
      for (int o = 0; o < O; ++o) {
        const float tt = fmaxf(fabsf(z[o]) - net.e, 0.f);
        const float sp = __expf(-tt) / ((1.f + __expf(-tt)) * (1.f + __expf(-tt)));
        tight = tight && (net.e * sp <= 2e-6f);
      }
      if (!tight) idx = -1;
    }
    if (idx < 0) {
      // arbitrary f64 inputs here: the group's f64 pass on them directly
      double xd[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) xd[i] = p.x[(long)t * 6 + i];
      idx = forward_f64_group<L, U, O, WT>(gw, H, b, (const double *)xd, lds, lig);
      if (p.act && lig < O) p.act[(long)t * O + lig] = lds[f64_out_offset(H, O) + lig];
      wave_lds_sync();
      slow += (lig == 0);
    } else if (p.act && lig < O) {
      float zz = z[0];
#pragma unroll
      for (int o = 1; o < O; ++o) zz = (lig == o) ? z[o] : zz;
      p.act[(long)t * O + lig] = sigmoid_f64((double)zz);
    }
    if (lig == 0) p.index[t] = idx;
  }
  if (p.counters && slow) atomicAdd((unsigned long long *)&p.counters[2], (unsigned long long)slow);
}

// ============================================================ physics ====
__global__ void k_physics_reset(int32_t *s, int n, const uint64_t *seeds, const int32_t *one_player) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Pong st;
  st.reset(seeds ? seeds[i] : 0ull, one_player ? one_player[i] : 0);
  const int f[PG_STATE_FIELDS] = {st.bx, st.by, st.vx, st.vy, st.vis, st.timer, st.dir, st.hits,
                                  st.point, st.lpy, st.rpy, st.s1, st.s2, st.one_player,
                                  (int)(uint32_t)st.seed, (int)(uint32_t)(st.seed >> 32)};
#pragma unroll
  for (int k = 0; k < PG_STATE_FIELDS; ++k) s[(long)k * n + i] = f[k];
}

__global__ void k_physics_step(int32_t *s, int n, const uint8_t *actions) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Pong st;
  st.bx = s[0L * n + i]; st.by = s[1L * n + i]; st.vx = s[2L * n + i]; st.vy = s[3L * n + i];
  st.vis = s[4L * n + i]; st.timer = s[5L * n + i]; st.dir = s[6L * n + i]; st.hits = s[7L * n + i];
  st.point = s[8L * n + i]; st.lpy = s[9L * n + i]; st.rpy = s[10L * n + i];
  st.s1 = s[11L * n + i]; st.s2 = s[12L * n + i]; st.one_player = s[13L * n + i];
  st.seed = (uint64_t)(uint32_t)s[14L * n + i] | ((uint64_t)(uint32_t)s[15L * n + i] << 32);
  const int a = actions[i];
  st.step(a & 3, (a >> 2) & 3);
  s[0L * n + i] = st.bx; s[1L * n + i] = st.by; s[2L * n + i] = st.vx; s[3L * n + i] = st.vy;
  s[4L * n + i] = st.vis; s[5L * n + i] = st.timer; s[6L * n + i] = st.dir; s[7L * n + i] = st.hits;
  s[8L * n + i] = st.point; s[9L * n + i] = st.lpy; s[10L * n + i] = st.rpy;
  s[11L * n + i] = st.s1; s[12L * n + i] = st.s2;
}

// ================================================================ GA =====
// Counter-based uniform double in [0,1): splitmix64 of (seed, generation,
// stream, a, b).  DEAP draws from Python's Mersenne Twister; the device GA
// matches its distributions, not its stream (DESIGN.md "GA").
__device__ __forceinline__ double u01(uint64_t seed, uint64_t gen, uint64_t stream, uint64_t a,
                                      uint64_t b) {
  uint64_t k = splitmix64(seed + 0x9E3779B97F4A7C15ull * (gen + 1));
  k = splitmix64(k ^ (stream * 0xD6E8FEB86659FD93ull + a));
  k = splitmix64(k ^ b);
  return (double)(k >> 11) * 0x1.0p-53;
}

// tools.selTournament: for each pick, tournsize aspirants drawn with
// replacement (selRandom = random.choice), the first maximum wins (max()).
__global__ void k_select(pg_select_args a) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.k) return;
  int best = -1;
  double bf = 0.0;
  for (int t = 0; t < a.tournsize; ++t) {
    const int idx = (int)(u01(a.seed, a.generation, 1, (uint64_t)j, (uint64_t)t) * (double)a.n_pop);
    const double f = a.fitness[idx];
    if (best < 0 || f > bf) {
      best = idx;
      bf = f;
    }
  }
  a.chosen[j] = best;
}

// selTournament by rank sampling (see pong_ga.h): P(winner rank <= r) = ((r+1)/n)^t.
__global__ void k_select_ranked(pg_select_args a, const double *sorted, const int32_t *order) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.k) return;
  const int n = a.n_pop;
  const double v = u01(a.seed, a.generation, 8, (uint64_t)j, 0);
  int r = (int)((double)n * exp(log(v) / (double)a.tournsize));
  r = r < 0 ? 0 : (r > n - 1 ? n - 1 : r);
  const double f = sorted[r];
  int lo = 0, hi = n;  // tie group [first, last) of value f
  int a0 = 0, b0 = r;
  while (a0 < b0) { const int m = (a0 + b0) >> 1; if (sorted[m] < f) a0 = m + 1; else b0 = m; }
  lo = a0;
  a0 = r; b0 = n;
  while (a0 < b0) { const int m = (a0 + b0) >> 1; if (sorted[m] <= f) a0 = m + 1; else b0 = m; }
  hi = a0;
  const int pick = lo + (int)(u01(a.seed, a.generation, 9, (uint64_t)j, 0) * (double)(hi - lo));
  a.chosen[j] = order[pick < hi ? pick : hi - 1];
}

// algorithms.varAnd: clone the chosen parents, cxBlend consecutive pairs
// (i-1, i) w.p. cxpb, then mutGaussian each individual w.p. mutpb.
//   cxBlend:     gamma = (1 + 2 alpha) U - alpha; x1' = (1-gamma) x1 + gamma x2; x2' = gamma x1 + (1-gamma) x2
//   mutGaussian: w.p. indpb per gene, x += N(mu, sigma)
// Counter-based randoms: a key per (generation, stream, pair or individual),
// then one splitmix64 per gene.  The two individuals of a pair share one
// Box-Muller draw (r cos t, r sin t), in f32 (the noise is added in f64).
__device__ __forceinline__ uint64_t rng_key(uint64_t seed, uint64_t gen, uint64_t stream, uint64_t a) {
  const uint64_t k = splitmix64(seed + 0x9E3779B97F4A7C15ull * (gen + 1));
  return splitmix64(k ^ (stream * 0xD6E8FEB86659FD93ull + a));
}
__device__ __forceinline__ double rng_u01(uint64_t key, uint64_t b) {
  return (double)(splitmix64(key ^ b) >> 11) * 0x1.0p-53;
}

// One wave per pair: the pair's draws (crossover, mutation, the keys of its
// per-gene streams) are wave-uniform scalar work done once, then the wave
// sweeps the genes 128 at a time (two coalesced 512-B pieces per parent row,
// all four loads issued before the arithmetic).
template <typename WT>
__device__ __forceinline__ void vary_pair(const pg_ga_args &a, int pair);

template <typename WT>
__global__ __launch_bounds__(256) void k_vary(pg_ga_args a) {
  const int wave = (int)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (a.pair_list) {  // a compact list of the pairs to write (pong_ga.h): the grid strides over it
    const int count = __builtin_amdgcn_readfirstlane(*a.pair_count);
    const int waves = (int)gridDim.x * 4;
#pragma unroll 1
    for (int w = wave; w < count; w += waves) vary_pair<WT>(a, __builtin_amdgcn_readfirstlane(a.pair_list[w]));
    return;
  }
  vary_pair<WT>(a, wave);
}

template <typename WT>
__device__ __forceinline__ void vary_pair(const pg_ga_args &a, int pair) {
  const int pairs = (a.n + 1) / 2;
  if (pair >= pairs) return;
  const int lane = threadIdx.x & 63;
  const int i0 = 2 * pair, i1 = 2 * pair + 1;
  const bool has1 = i1 < a.n;
  const bool cx = has1 && rng_u01(rng_key(a.seed, a.generation, 2, (uint64_t)pair), 0) < a.cxpb;
  const bool mut0 = rng_u01(rng_key(a.seed, a.generation, 4, (uint64_t)i0), 0) < a.mutpb;
  const bool mut1 = has1 && rng_u01(rng_key(a.seed, a.generation, 4, (uint64_t)i1), 0) < a.mutpb;
  if (lane == 0) {
    a.invalid[i0] = (uint8_t)(cx || mut0);
    if (has1) a.invalid[i1] = (uint8_t)(cx || mut1);
  }
  if (!a.pair_list && a.pair_mask && !a.pair_mask[pair]) return;  // a pair this call does not write (pong_ga.h)
  const uint64_t k3 = rng_key(a.seed, a.generation, 3, (uint64_t)pair);
  const uint64_t k5 = rng_key(a.seed, a.generation, 5, (uint64_t)pair);
  const uint64_t k6 = rng_key(a.seed, a.generation, 6, (uint64_t)pair);
  const WT *p1 = (const WT *)a.parents + (long)a.chosen[i0] * a.stride;
  const WT *p2 = (const WT *)a.parents + (long)(has1 ? a.chosen[i1] : a.chosen[i0]) * a.stride;
  WT *o1 = (WT *)a.offspring + (long)i0 * a.stride;
  WT *o2 = (WT *)a.offspring + (long)i1 * a.stride;
  const auto one = [&](long gene, double x1, double x2) {
    if (cx) {
      const double u = rng_u01(k3, (uint64_t)gene);
      const double gamma = __dadd_rn(__dmul_rn(1.0 + 2.0 * a.alpha, u), -a.alpha);
      const double y1 = __dadd_rn(__dmul_rn(1.0 - gamma, x1), __dmul_rn(gamma, x2));
      const double y2 = __dadd_rn(__dmul_rn(gamma, x1), __dmul_rn(1.0 - gamma, x2));
      x1 = y1;
      x2 = y2;
    }
    // one 64-bit draw decides both individuals' indpb hits (32 bits each),
    // one more feeds the shared Box-Muller pair (24 bits per uniform)
    const uint64_t hb = splitmix64(k5 ^ (uint64_t)gene);
    const bool h0 = mut0 && (double)(uint32_t)hb * 0x1.0p-32 < a.indpb;
    const bool h1 = mut1 && (double)(uint32_t)(hb >> 32) * 0x1.0p-32 < a.indpb;
    if (h0 || h1) {
      const uint64_t nb = splitmix64(k6 ^ (uint64_t)gene);
      const float u1 = 1.0f - (float)(nb >> 40) * 0x1.0p-24f;  // (0, 1]
      const float u2 = (float)((nb >> 8) & 0xFFFFFFu) * 0x1.0p-24f;
      const float r = sqrtf(-2.0f * logf(u1));
      float sn, cs;
      sincosf(6.2831853f * u2, &sn, &cs);
      if (h0) x1 = __dadd_rn(x1, __dadd_rn(a.mu, __dmul_rn(a.sigma, (double)(r * cs))));
      if (h1) x2 = __dadd_rn(x2, __dadd_rn(a.mu, __dmul_rn(a.sigma, (double)(r * sn))));
    }
    o1[gene] = (WT)x1;
    if (has1) o2[gene] = (WT)x2;
  };
  // kVaryChunk 128-gene pieces of both parents requested before any arithmetic
  // (a [6,64,3] genome, 454 genes, is one chunk): more loads in flight per wave
  constexpr int kVaryChunk = 4;
  for (long g0 = 0; g0 < a.genes; g0 += 128 * kVaryChunk) {
    double x[kVaryChunk][2][2];
#pragma unroll
    for (int c = 0; c < kVaryChunk; ++c) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const long g = g0 + c * 128 + h * 64 + lane;
        const bool v = g < a.genes;
        x[c][h][0] = v ? (double)p1[g] : 0.0;
        x[c][h][1] = v && has1 ? (double)p2[g] : 0.0;
      }
    }
#pragma unroll
    for (int c = 0; c < kVaryChunk; ++c) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const long g = g0 + c * 128 + h * 64 + lane;
        if (g < a.genes) one(g, x[c][h][0], x[c][h][1]);
      }
    }
  }
}

__global__ void k_mark_pairs(uint8_t *mask, int n_pairs, const int32_t *rows, int n_rows, int skip_lo, int skip_hi,
                             const uint8_t *exclude) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows) return;
  const int r = rows[i];
  if (r < 0 || r >= 2 * n_pairs) return;
  const int j = r >> 1;
  if ((j < skip_lo || j >= skip_hi) && !(exclude && exclude[j])) mask[j] = 1;
}

// pg_ga_list_pairs: the marked pairs appended to a list (order irrelevant).
__global__ void k_list_pairs(const uint8_t *mask, int n_pairs, int32_t *list, int32_t *count) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n_pairs && mask[j]) list[atomicAdd(count, 1)] = j;
}

// Opponent schedule of evaluate() (main.py:28-66) for rows [0, n).
__global__ void k_schedule(pg_schedule_args a) {
  const long w = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= (long)a.n * a.n_games) return;
  const long i = w / a.n_games;
  const int g = (int)(w % a.n_games);
  const long row = a.rows ? (long)a.rows[i] : a.row_offset + i;
  int kind = kOppHard, opp = 0;
  double mult = 1.0;
  if (a.mode == PG_SCHED_SELFPLAY) {
    if (a.n_hof > 0) {
      kind = kOppNN;
      const int K = a.hof_slices > 1 && a.n_hof >= a.hof_slices ? a.hof_slices : 1;
      if (K == 1) {
        opp = (int)((row * a.n_games + g) % a.n_hof);
      } else {  // the block's interleaved slice of the hall (pong_ga.h)
        const int b = (int)((row / a.block_rows) % K);
        const long m = (a.n_hof - b + K - 1) / K;
        const int k = (int)((row * a.n_games + g) % m);
        opp = a.slice_local ? k : k * K + b;
      }
    }
  } else if (g < 3) {
    kind = g == 0 ? kOppHard : (g == 1 ? kOppRomCpu : kOppScore);
    // right_score_multiplier is 1 until the first pick (main.py:32)
  } else if (a.n_hof > 0) {
    kind = kOppNN;
    opp = (int)(u01(a.seed, a.generation, 10, (uint64_t)row, (uint64_t)g) * (double)a.n_hof);
    opp = opp < a.n_hof ? opp : a.n_hof - 1;
    mult = a.hof_fitness[opp];
  }
  a.kind[w] = kind;
  a.opp[w] = opp;
  a.mult[w] = mult;
}

// pg_gather_rows: one workgroup per destination row.
template <typename WT>
__global__ __launch_bounds__(256) void k_gather_rows(WT *dst, int64_t dst_stride, const WT *old_rows, int64_t old_stride,
                                                     const WT *rows, int64_t rows_stride, const int64_t *index,
                                                     const int32_t *src, int n_old, int64_t genes) {
  const int j = blockIdx.x;
  const int s = src[j];
  const WT *from = s < n_old ? old_rows + (long)s * old_stride
                             : rows + (index ? index[s - n_old] : (long)(s - n_old)) * rows_stride;
  WT *to = dst + (long)j * dst_stride;
  for (int64_t g = threadIdx.x; g < genes; g += 256) to[g] = from[g];
}

// 64-bit content hash of each row: an order-independent sum of mixed
// (index, bit pattern) terms, so the block reduction order cannot matter.
template <typename WT>
__global__ __launch_bounds__(256) void k_row_hash(const WT *rows, int64_t stride, const int32_t *index, int n,
                                                  int64_t genes, uint64_t *out) {
  __shared__ uint64_t part[4];
  const int r = blockIdx.x;
  if (r >= n) return;
  const WT *row = rows + (long)(index ? index[r] : r) * stride;
  uint64_t h = 0;
  for (int64_t j = threadIdx.x; j < genes; j += 256) {
    uint64_t bits;
    if constexpr (sizeof(WT) == 8) {
      const double v = row[j];
      bits = v == 0.0 ? 0ull : (uint64_t)__double_as_longlong(v);
    } else {
      const float v = row[j];
      bits = v == 0.0f ? 0ull : (uint64_t)__float_as_uint(v);
    }
    h += splitmix64(bits ^ ((uint64_t)j * 0x9E3779B97F4A7C15ull));
  }
  for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) out[r] = splitmix64(part[0] + part[1] + part[2] + part[3] + (uint64_t)genes);
}

// ====================================================== host dispatch ====
static int gene_count(const pg_net &n) {
  const int b = n.bias ? 1 : 0;
  long t = 0;
  for (int i = 0; i + 1 < n.n_nodes; ++i) t += (long)(n.nodes[i] + b) * n.nodes[i + 1];
  return t > 0x7fffffff ? -1 : (int)t;
}

static int32_t check_net(const pg_net &n, bool game) {
  if (n.n_nodes < 2 || n.n_nodes > PG_MAX_NODES)
    return fail(PG_ERR_INVALID, "net.n_nodes=%d must be in [2, %d]", n.n_nodes, PG_MAX_NODES);
  for (int i = 0; i < n.n_nodes; ++i)
    if (n.nodes[i] < 1 || n.nodes[i] > 65536)
      return fail(PG_ERR_INVALID, "net.nodes[%d]=%d out of range", i, n.nodes[i]);
  if (game && n.nodes[0] != 6)
    return fail(PG_ERR_INVALID, "the game feeds 6 inputs (utils.py:146-152); nodes[0]=%d", n.nodes[0]);
  if (n.dtype != PG_F32 && n.dtype != PG_F64) return fail(PG_ERR_INVALID, "net.dtype=%d", n.dtype);
  if (gene_count(n) < 0) return fail(PG_ERR_INVALID, "network too large");
  return PG_OK;
}

static int max_width(const pg_net &n) {
  int m = 0;
  for (int i = 0; i < n.n_nodes; ++i) m = n.nodes[i] > m ? n.nodes[i] : m;
  return m;
}

static int g_num_cus = 0;
int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      g_num_cus = prop.multiProcessorCount;
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

// Resident kernel table: (L, U) chosen from the hidden width H.
struct ResidentChoice {
  int L, U;
};
static ResidentChoice choose_resident(int H, int requested_L) {
  static const ResidentChoice table[] = {{4, 1}, {8, 1}, {16, 1}, {32, 1}, {16, 4}, {32, 4}, {64, 4}};
  static const ResidentChoice all[] = {{4, 1}, {8, 1}, {16, 1}, {32, 1}, {64, 1}, {16, 2}, {32, 2},
                                       {64, 2}, {16, 4}, {32, 4}, {64, 4}};
  if (requested_L > 0) {
    for (const auto &c : all)
      if (c.L == requested_L && c.L * c.U >= H) return c;
    return {0, 0};
  }
  for (const auto &c : table)
    if (c.L * c.U >= H) return c;
  return {0, 0};
}


// split layout for hidden width H: L lanes per game (L/2 per network).  Fewer
// lanes per game means more games per wave, so the replicated scalar work of
// a frame (physics, bookkeeping, the certificate) is shared by fewer lanes;
// L = 8 holds up to 16 units per lane (H <= 64) in 256 VGPRs (measured
// fastest for [6,64,3]: profiles/r01/sweep_lanes.log).
static int choose_split_lanes(int H) {
  if (H <= 64) return 8;
  if (H <= 128) return 32;
  return 64;
}

template <typename WT>
static int32_t launch_service_any(const EvalParams &p, int L, int O, hipStream_t s) {
  const int H = p.nodes[1];
  // the bench layout here (H in (32, 64] with L = 8: U = 16 is the smallest
  // that holds it); every other (L, U) in pg_service_more.hip
#ifdef PG_DEV_MIN
  const bool here = L == 8 && H <= 64;
#else
  const bool here = L == 8 && H > 32 && H <= 64;
#endif
  // (only O = 3 here: the iterative scheduler's register allocator crashes
  // ROCm 7.2's compiler on the O = 2 / 4 instances, built in pg_service_more.hip)
  if (here && O == 3) return launch_service<8, 16, 3, WT, true>(p, s);
#ifdef PG_DEV_MIN  // variant builds for experiments (tools/build_variant.sh): the bench layout only
  return fail(PG_ERR_UNSUPPORTED, "no service kernel for L=%d H=%d O=%d", L, H, O);
#else
  return launch_service_more(p, L, O, sizeof(WT) == 8, s);
#endif
}


template <int L, int U, int O, typename WT>
static int32_t launch_fwd_resident(const FwdParams &p, hipStream_t s) {
  constexpr int GPB = 256 / L;
  const size_t lds = (size_t)GPB * f64_lds_doubles(p.nodes[1], O) * sizeof(double);
  const int want = (p.n + GPB - 1) / GPB;
  const int cap = num_cus() * 8;
  const int grid = want < cap ? want : cap;
  if (grid <= 0) return PG_OK;
  hipLaunchKernelGGL((k_forward_resident<L, U, O, WT>), dim3(grid), dim3(256), lds, s, p);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

template <typename WT>
static int32_t launch_fwd_resident_any(const FwdParams &p, ResidentChoice c, int O, hipStream_t s) {
#define PG_FRES(LL, UU)                                                  \
  if (c.L == LL && c.U == UU) {                                          \
    if (O == 2) return launch_fwd_resident<LL, UU, 2, WT>(p, s);         \
    if (O == 3) return launch_fwd_resident<LL, UU, 3, WT>(p, s);         \
    if (O == 4) return launch_fwd_resident<LL, UU, 4, WT>(p, s);         \
  }
#ifndef PG_DEV_MIN
  PG_FRES(4, 1) PG_FRES(8, 1) PG_FRES(16, 1) PG_FRES(32, 1) PG_FRES(64, 1)
  PG_FRES(16, 2) PG_FRES(32, 2) PG_FRES(64, 2) PG_FRES(16, 4) PG_FRES(32, 4) PG_FRES(64, 4)
#endif
#undef PG_FRES
  return fail(PG_ERR_UNSUPPORTED, "no resident forward kernel for L=%d U=%d O=%d", c.L, c.U, O);
}

static bool resident_shape_ok(const pg_net &n) {
  return n.n_nodes == 3 && n.nodes[0] == 6 && n.nodes[1] <= 256 && n.nodes[2] >= 2 && n.nodes[2] <= 4;
}

}  // namespace pg

using namespace pg;

// ================================================================ C-ABI ===
extern "C" {

const char *pg_version(void) { return PG_VERSION_STRING; }
int32_t pg_abi_version(void) { return PG_ABI_VERSION; }
int32_t pg_build_flags(void) { return 0; }
const char *pg_last_error(void) { return g_last_error.c_str(); }

int32_t pg_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return fail(PG_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
  return n;
}

// [0, 256): dynamic game counter; then one int32 per game (zero-division
// flags); for the staged kernel, then its prepared lane records
static size_t eval_base_workspace(const pg_eval_args *a) {
  const size_t games = a ? (size_t)(a->n_genomes > 0 ? a->n_genomes : 0) * (size_t)(a->n_games > 0 ? a->n_games : 0) : 0;
  return 256 + ((games * sizeof(int32_t) + 255) / 256) * 256;
}

// the kernel pg_eval_population runs for a (PG_KERNEL_AUTO resolved)
static int resolve_kernel(const pg_eval_args *a) {
  if (a->kernel != PG_KERNEL_AUTO) return a->kernel;
  if (resident_shape_ok(a->net) && a->precision == PG_PREC_CERTIFIED) return PG_KERNEL_SPLIT;
  if (wide_shape_ok(a->net, a->n_games) && (a->net.nodes[1] >= 64 || a->net.nodes[2] >= 64)) return PG_KERNEL_WIDE;
  return PG_KERNEL_GENERAL;
}

// the split kernel's lane records (k_prep_records), after the base workspace
static size_t split_records_bytes(const pg_eval_args *a) {
  if (!resident_shape_ok(a->net) || a->n_genomes <= 0) return 0;
  const int H = a->net.nodes[1];
  const int L = a->group_lanes > 0 ? a->group_lanes : choose_split_lanes(H);
  const int U = (L == 8 && H <= 64) ? 16 : service_units(L, H);  // >= what any build instantiates
  if (U <= 0) return 0;
  return (service_records_bytes(a->n_genomes, a->opponents ? a->n_opponents : 0, L, U, a->net.nodes[2]) + 255) /
         256 * 256;
}

// ABI 10: the caller's struct must be this header's (pg_eval_args.struct_size)
static int32_t check_struct_size(const pg_eval_args *a) {
  if (a->struct_size != sizeof(pg_eval_args))
    return fail(PG_ERR_INVALID, "pg_eval_args.struct_size=%u, this library's struct is %zu bytes (ABI %d)",
                a->struct_size, sizeof(pg_eval_args), PG_ABI_VERSION);
  return PG_OK;
}

size_t pg_eval_workspace_bytes(const pg_eval_args *a) {
  if (a && check_struct_size(a) != PG_OK) return 0;
  size_t n = eval_base_workspace(a);
  if (!a) return n;
  const int kernel = resolve_kernel(a);
  if (kernel == PG_KERNEL_SPLIT) n += split_records_bytes(a);
  if (kernel == PG_KERNEL_WIDE && wide_shape_ok(a->net, a->n_games)) n += (wide_workspace_bytes(a) + 255) / 256 * 256;
  return n;
}

int32_t pg_gene_count(const pg_net *net) {
  if (!net) return fail(PG_ERR_INVALID, "net is NULL");
  int32_t rc = check_net(*net, false);
  if (rc != PG_OK) return rc;
  return gene_count(*net);
}

int32_t pg_eval_population(const pg_eval_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  int32_t rc = check_struct_size(a);
  if (rc != PG_OK) return rc;
  rc = check_net(a->net, true);
  if (rc != PG_OK) return rc;
  if (a->n_genomes < 0) return fail(PG_ERR_INVALID, "n_genomes=%d < 0", a->n_genomes);
  if (a->n_games < 1 || a->n_games > 64) return fail(PG_ERR_INVALID, "n_games=%d not in [1, 64]", a->n_games);
  if (a->horizon < 0) return fail(PG_ERR_INVALID, "horizon=%d < 0", a->horizon);
  if (a->timeout_thresh != 0 && (a->timeout_thresh < 32 || a->timeout_thresh > (1 << 20)))
    return fail(PG_ERR_INVALID, "timeout_thresh=%d not 0 or in [32, 1048576]", a->timeout_thresh);
  if (a->win_score < 0) return fail(PG_ERR_INVALID, "win_score=%d < 0", a->win_score);
  if (a->n_genomes == 0) {  // nothing to play (e.g. an empty shard); the counters still read zero
    if (a->counters) PG_HIP(hipMemsetAsync(a->counters, 0, 16 * sizeof(uint64_t), (hipStream_t)stream));
    return PG_OK;
  }
  const long total = (long)a->n_genomes * a->n_games;
  if (total > 0x7fffffffL) return fail(PG_ERR_INVALID, "too many games (%ld)", total);
  const int G = gene_count(a->net);
  if (!a->genomes || a->genome_stride < G)
    return fail(PG_ERR_INVALID, "genomes NULL or genome_stride=%lld < gene count %d", (long long)a->genome_stride, G);
  if (!a->game_kind || !a->game_opp || !a->game_mult || !a->fitness || !a->rewards || !a->scores ||
      !a->frames || !a->total_frames || !a->status)
    return fail(PG_ERR_INVALID, "a required per-game array is NULL");
  if (a->n_opponents > 0 && (!a->opponents || a->opponent_stride < G))
    return fail(PG_ERR_INVALID, "opponents NULL or opponent_stride < gene count");
  if (a->precision != PG_PREC_CERTIFIED && a->precision != PG_PREC_F64)
    return fail(PG_ERR_INVALID, "precision=%d", a->precision);
  if (a->trace && (a->trace_games < 0 || a->trace_cap < 1))
    return fail(PG_ERR_INVALID, "trace needs trace_games >= 0 and trace_cap >= 1");
  if (a->prep < PG_PREP_ALL || a->prep > PG_PREP_REST) return fail(PG_ERR_INVALID, "prep=%d", a->prep);
  if (a->horizon > 0 && a->trace) return fail(PG_ERR_INVALID, "horizon mode runs untraced (trace must be NULL)");
  if (a->horizon > 0 && resolve_kernel(a) != PG_KERNEL_SPLIT)
    return fail(PG_ERR_UNSUPPORTED, "horizon mode runs on the SPLIT kernel ([6, H<=64, 3], certified)");
  const size_t need = pg_eval_workspace_bytes(a);
  if (!a->workspace || a->workspace_bytes < need)
    return fail(PG_ERR_INVALID, "workspace of %zu bytes required (got %zu)", need, a->workspace_bytes);

  hipStream_t s = (hipStream_t)stream;
  EvalParams p;
  memset(&p, 0, sizeof(p));
  p.genomes = a->genomes;
  p.opponents = a->opponents ? a->opponents : a->genomes;
  p.kind = a->game_kind;
  p.opp = a->game_opp;
  p.mult = a->game_mult;
  p.rewards = a->rewards;
  p.scores = a->scores;
  p.frames = a->frames;
  p.total_frames = a->total_frames;
  p.counters = a->counters;
  p.trace = a->trace;
  p.trace_games = a->trace ? a->trace_games : 0;
  p.trace_cap = a->trace_cap;
  p.hard_log = a->hard_cap > 0 ? a->hard_log : nullptr;
  p.hard_cap = a->hard_cap;
  p.work = (unsigned int *)a->workspace;
  p.status_game = (int32_t *)((char *)a->workspace + 256);
  p.gstride = a->genome_stride;
  p.ostride = a->opponent_stride;
  p.n_opponents = a->opponents ? a->n_opponents : 0;
  p.rows = a->genome_rows;
  p.n_active = a->n_active;
  p.seed = a->seed;
  p.n_genomes = a->n_genomes;
  p.n_games = a->n_games;
  p.total = (int)total;
  for (int i = 0; i < a->net.n_nodes; ++i) p.nodes[i] = a->net.nodes[i];
  p.n_nodes = a->net.n_nodes;
  p.bias = a->net.bias ? 1 : 0;
  p.max_width = max_width(a->net);

  p.prep = a->prep;
  p.horizon = a->horizon;
  p.timeout_thresh = a->timeout_thresh > 0 ? a->timeout_thresh : kTimeoutThresh;
  // above the env's own end (a score of 21, Pong::done) WIN_SCORE changes nothing
  p.win_score = a->win_score > 0 ? (a->win_score < kDoneScore ? a->win_score : kDoneScore) : kWinScore;
  const int kernel = resolve_kernel(a);
  if (kernel != PG_KERNEL_SPLIT) {
    if (a->prep == PG_PREP_GENOMES) return PG_OK;  // no records outside the split kernel
    p.prep = PG_PREP_ALL;
    PG_HIP(hipMemsetAsync(a->workspace, 0, 256, s));
    if (a->counters) PG_HIP(hipMemsetAsync(a->counters, 0, 16 * sizeof(uint64_t), s));
  }  // the split kernel's k_prep_records zeroes the work header and the counters itself
  const bool res_ok = resident_shape_ok(a->net);
  const bool wide_ok = wide_shape_ok(a->net, a->n_games);
  if (kernel == PG_KERNEL_WIDE) {
    if (!wide_ok)
      return fail(PG_ERR_UNSUPPORTED, "wide kernel needs NETWORK_SHAPE [6, H1<=512, H2<=512, 1..4] and n_games <= 8");
    rc = launch_wide(p, a->net.dtype, (char *)a->workspace + eval_base_workspace(a), s);
    if (rc != PG_OK) return rc;
  } else if (kernel == PG_KERNEL_SPLIT) {
    if (!res_ok) return fail(PG_ERR_UNSUPPORTED, "split kernel needs NETWORK_SHAPE [6, H<=256, 2..4]");
    if (a->precision != PG_PREC_CERTIFIED) return fail(PG_ERR_UNSUPPORTED, "split kernel is the certified-precision path");
    const int H = a->net.nodes[1];
    const int L = a->group_lanes > 0 ? a->group_lanes : choose_split_lanes(H);
    p.recs = (float *)((char *)a->workspace + eval_base_workspace(a));
    rc = a->net.dtype == PG_F64 ? launch_service_any<double>(p, L, a->net.nodes[2], s)
                                : launch_service_any<float>(p, L, a->net.nodes[2], s);
    if (rc != PG_OK) return rc;
    if (a->prep == PG_PREP_GENOMES) return PG_OK;  // records only: no games, no fitness
  } else if (kernel == PG_KERNEL_RESIDENT || kernel == PG_KERNEL_STAGED) {
    // retired layouts (correct, measured slower than SPLIT; removed in round 4)
    return fail(PG_ERR_UNSUPPORTED, "the %s kernel was retired (DESIGN 4.1b-c); use SPLIT",
                kernel == PG_KERNEL_RESIDENT ? "resident" : "staged");
  } else if (kernel == PG_KERNEL_GENERAL) {
    const size_t lds = 2 * (size_t)(p.max_width + 1) * sizeof(double);
    if (lds > 160 * 1024) return fail(PG_ERR_UNSUPPORTED, "layer width %d too large for LDS", p.max_width);
    const int cap = num_cus() * 16;
    const int grid = total < cap ? (int)total : cap;
    if (a->net.dtype == PG_F64)
      hipLaunchKernelGGL(k_general<double>, dim3(grid), dim3(64), lds, s, p);
    else
      hipLaunchKernelGGL(k_general<float>, dim3(grid), dim3(64), lds, s, p);
    PG_HIP(hipGetLastError());
  } else {
    return fail(PG_ERR_INVALID, "kernel=%d", a->kernel);
  }
  hipLaunchKernelGGL(k_fitness, dim3((a->n_genomes + 255) / 256), dim3(256), 0, s, a->rewards,
                     p.status_game, a->n_genomes, a->n_active, a->n_games, a->fitness, a->status);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_forward(const pg_forward_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  int32_t rc = check_net(a->net, false);
  if (rc != PG_OK) return rc;
  if (a->n < 0) return fail(PG_ERR_INVALID, "n=%d < 0", a->n);
  if (a->n == 0) return PG_OK;
  const int G = gene_count(a->net);
  if (!a->genomes || a->genome_stride < G || !a->x || !a->index)
    return fail(PG_ERR_INVALID, "genomes/x/index NULL or genome_stride < gene count %d", G);
  hipStream_t s = (hipStream_t)stream;
  FwdParams p;
  memset(&p, 0, sizeof(p));
  p.genomes = a->genomes;
  p.gidx = a->genome_index;
  p.x = a->x;
  p.index = a->index;
  p.act = a->act;
  p.z_all = a->z_all;
  p.h_all = a->h_all;
  p.counters = a->counters;
  p.gstride = a->genome_stride;
  p.n = a->n;
  for (int i = 0; i < a->net.n_nodes; ++i) p.nodes[i] = a->net.nodes[i];
  for (int i = 1; i < a->net.n_nodes; ++i) p.n_units += a->net.nodes[i];
  if ((a->z_all || a->h_all) && a->precision != PG_PREC_F64)
    return fail(PG_ERR_INVALID, "z_all/h_all need precision PG_PREC_F64");
  p.n_nodes = a->net.n_nodes;
  p.bias = a->net.bias ? 1 : 0;
  p.max_width = max_width(a->net);
  if (a->precision == PG_PREC_CERTIFIED && resident_shape_ok(a->net)) {
    const ResidentChoice c = choose_resident(a->net.nodes[1], 0);
    return a->net.dtype == PG_F64 ? launch_fwd_resident_any<double>(p, c, a->net.nodes[2], s)
                                  : launch_fwd_resident_any<float>(p, c, a->net.nodes[2], s);
  }
  if (a->precision != PG_PREC_CERTIFIED && a->precision != PG_PREC_F64)
    return fail(PG_ERR_INVALID, "precision=%d", a->precision);
  const size_t lds = 2 * (size_t)(p.max_width + 1) * sizeof(double);
  if (lds > 160 * 1024) return fail(PG_ERR_UNSUPPORTED, "layer width %d too large for LDS", p.max_width);
  const int cap = num_cus() * 16;
  const int grid = a->n < cap ? a->n : cap;
  if (a->net.dtype == PG_F64)
    hipLaunchKernelGGL(k_forward_general<double>, dim3(grid), dim3(64), lds, s, p);
  else
    hipLaunchKernelGGL(k_forward_general<float>, dim3(grid), dim3(64), lds, s, p);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_decide(const pg_decide_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  int32_t rc = check_net(a->net, false);
  if (rc != PG_OK) return rc;
  if (!resident_shape_ok(a->net)) return fail(PG_ERR_UNSUPPORTED, "pg_decide: the split kernel's shapes only");
  if (a->n < 0) return fail(PG_ERR_INVALID, "n=%d < 0", a->n);
  if (a->n == 0) return PG_OK;
  const int G = gene_count(a->net);
  if (!a->genomes || a->genome_stride < G || !a->k || !a->index)
    return fail(PG_ERR_INVALID, "genomes/k/index NULL or genome_stride < gene count %d", G);
  DecideParams p;
  memset(&p, 0, sizeof(p));
  p.genomes = a->genomes;
  p.gidx = a->genome_index;
  p.k = a->k;
  p.index = a->index;
  p.stage = a->stage;
  p.gstride = a->genome_stride;
  p.n = a->n;
  p.H = a->net.nodes[1];
  p.b = a->net.bias ? 1 : 0;
  const int H = p.H, O = a->net.nodes[2];
  const int L = choose_split_lanes(H);
  const size_t lds = (size_t)f64_lds_doubles(H, O) * sizeof(double);
  return launch_decide(p, L, O, a->net.dtype == PG_F64, lds, (hipStream_t)stream);
}

// pg_wide_decide runs k_wide as a one-game evaluation of n genomes: the
// evaluation's sizes for its workspace (a game counter, then the blocks' W2 copies)
static pg_eval_args wide_decide_eval(const pg_wide_decide_args *a) {
  pg_eval_args e;
  memset(&e, 0, sizeof(e));
  e.struct_size = sizeof(e);
  e.net = a->net;
  e.n_genomes = a->n;
  e.n_games = 1;
  return e;
}

size_t pg_wide_decide_workspace_bytes(const pg_wide_decide_args *a) {
  if (!a || a->n <= 0 || !wide_shape_ok(a->net, 1)) return 256;
  const pg_eval_args e = wide_decide_eval(a);
  return 256 + (wide_workspace_bytes(&e) + 255) / 256 * 256;
}

int32_t pg_wide_decide(const pg_wide_decide_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  int32_t rc = check_net(a->net, false);
  if (rc != PG_OK) return rc;
  if (!wide_shape_ok(a->net, 1))
    return fail(PG_ERR_UNSUPPORTED, "pg_wide_decide: the wide kernel's shapes [6, H1<=512, H2<=512, 1..4] only");
  if (a->n < 0) return fail(PG_ERR_INVALID, "n=%d < 0", a->n);
  if (a->n == 0) return PG_OK;
  const int G = gene_count(a->net);
  if (!a->genomes || a->genome_stride < G || !a->k || !a->index)
    return fail(PG_ERR_INVALID, "genomes/k/index NULL or genome_stride < gene count %d", G);
  const size_t need = pg_wide_decide_workspace_bytes(a);
  if (!a->workspace || a->workspace_bytes < need)
    return fail(PG_ERR_INVALID, "workspace of %zu bytes required (got %zu)", need, a->workspace_bytes);
  hipStream_t s = (hipStream_t)stream;
  EvalParams p;
  memset(&p, 0, sizeof(p));
  p.genomes = a->genomes;
  p.opponents = a->genomes;
  p.rows = a->genome_index;
  p.work = (unsigned int *)a->workspace;
  p.gstride = a->genome_stride;
  p.ostride = a->genome_stride;
  p.n_genomes = a->n;
  p.n_games = 1;
  p.total = a->n;
  for (int i = 0; i < a->net.n_nodes; ++i) p.nodes[i] = a->net.nodes[i];
  p.n_nodes = a->net.n_nodes;
  p.bias = a->net.bias ? 1 : 0;
  p.max_width = max_width(a->net);
  p.wide_probe_k = a->k;
  p.wide_probe_index = a->index;
  p.wide_probe_act = a->act;
  PG_HIP(hipMemsetAsync(a->workspace, 0, 256, s));
  return launch_wide(p, a->net.dtype, (char *)a->workspace + 256, s);
}

int32_t pg_physics_reset(int32_t *state, int32_t n, const uint64_t *seeds, const int32_t *one_player,
                         void *stream) {
  if (n < 0 || (n > 0 && !state)) return fail(PG_ERR_INVALID, "state NULL or n < 0");
  if (n == 0) return PG_OK;
  hipLaunchKernelGGL(k_physics_reset, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, state, n,
                     seeds, one_player);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_physics_step(int32_t *state, int32_t n, const uint8_t *actions, void *stream) {
  if (n < 0 || (n > 0 && (!state || !actions))) return fail(PG_ERR_INVALID, "state/actions NULL or n < 0");
  if (n == 0) return PG_OK;
  hipLaunchKernelGGL(k_physics_step, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, state, n,
                     actions);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_ga_select_tournament(const pg_select_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  if (a->k < 0 || a->n_pop < 1 || a->tournsize < 1 || !a->fitness || !a->chosen)
    return fail(PG_ERR_INVALID, "selTournament needs k >= 0, n_pop >= 1, tournsize >= 1 and buffers");
  if (a->k == 0) return PG_OK;
  hipLaunchKernelGGL(k_select, dim3((a->k + 255) / 256), dim3(256), 0, (hipStream_t)stream, *a);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_ga_select_tournament_ranked(const pg_select_args *a, const double *sorted_fitness,
                                       const int32_t *order, void *stream) {
  if (!a || !sorted_fitness || !order) return fail(PG_ERR_INVALID, "args/sorted_fitness/order is NULL");
  if (a->k < 0 || a->n_pop < 1 || a->tournsize < 1 || !a->chosen)
    return fail(PG_ERR_INVALID, "selTournament needs k >= 0, n_pop >= 1, tournsize >= 1 and buffers");
  if (a->k == 0) return PG_OK;
  hipLaunchKernelGGL(k_select_ranked, dim3((a->k + 255) / 256), dim3(256), 0, (hipStream_t)stream, *a,
                     sorted_fitness, order);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_ga_vary(const pg_ga_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  if (a->n < 0 || a->genes < 1 || a->stride < a->genes || !a->parents || !a->chosen || !a->offspring ||
      !a->invalid || (a->dtype != PG_F32 && a->dtype != PG_F64))
    return fail(PG_ERR_INVALID, "varAnd: bad sizes or NULL buffers");
  if (a->n == 0) return PG_OK;
  const int pairs = (a->n + 1) / 2;
  if (a->pair_list && (!a->pair_count || a->pair_cap < 0)) return fail(PG_ERR_INVALID, "varAnd: pair_list needs pair_count and pair_cap >= 0");
  // list mode: the grid strides over the listed pairs, so pair_cap (an upper
  // bound of the count, which the device holds) only sizes the grid
  constexpr int kListWaves = 8192;
  int waves = a->pair_list ? (a->pair_cap < pairs ? a->pair_cap : pairs) : pairs;
  if (a->pair_list && waves > kListWaves) waves = kListWaves;
  if (waves == 0) return PG_OK;
  const dim3 grid((unsigned)((waves + 3) / 4));  // one wave per pair
  if (a->dtype == PG_F64)
    hipLaunchKernelGGL(k_vary<double>, grid, dim3(256), 0, (hipStream_t)stream, *a);
  else
    hipLaunchKernelGGL(k_vary<float>, grid, dim3(256), 0, (hipStream_t)stream, *a);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_ga_list_pairs(const uint8_t *mask, int32_t n_pairs, int32_t *list, int32_t *count, void *stream) {
  if (n_pairs < 0 || !count || (n_pairs && (!mask || !list))) return fail(PG_ERR_INVALID, "list_pairs: bad sizes or NULL buffers");
  PG_HIP(hipMemsetAsync(count, 0, sizeof(int32_t), (hipStream_t)stream));
  if (n_pairs == 0) return PG_OK;
  hipLaunchKernelGGL(k_list_pairs, dim3((unsigned)((n_pairs + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mask,
                     n_pairs, list, count);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_ga_mark_pairs(uint8_t *mask, int32_t n_pairs, const int32_t *rows, int32_t n_rows, int32_t skip_lo,
                         int32_t skip_hi, const uint8_t *exclude, void *stream) {
  if (n_pairs < 0 || n_rows < 0 || (n_rows && (!mask || !rows)))
    return fail(PG_ERR_INVALID, "mark_pairs: bad sizes or NULL buffers");
  if (n_rows == 0) return PG_OK;
  hipLaunchKernelGGL(k_mark_pairs, dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mask,
                     n_pairs, rows, n_rows, skip_lo, skip_hi, exclude);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_ga_schedule(const pg_schedule_args *a, void *stream) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  if (a->n < 0 || a->n_games < 1 || a->n_hof < 0 || a->row_offset < 0 ||
      (a->mode != PG_SCHED_REFERENCE && a->mode != PG_SCHED_SELFPLAY))
    return fail(PG_ERR_INVALID, "schedule: bad sizes or mode");
  if (a->n == 0) return PG_OK;
  if (!a->kind || !a->opp || !a->mult || (a->mode == PG_SCHED_REFERENCE && a->n_hof > 0 && !a->hof_fitness))
    return fail(PG_ERR_INVALID, "schedule: NULL output or hof_fitness");
  const long total = (long)a->n * a->n_games;
  if (a->hof_slices > 1 && a->block_rows < 1) return fail(PG_ERR_INVALID, "schedule: hof_slices > 1 needs block_rows >= 1");
  hipLaunchKernelGGL(k_schedule, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *a);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_gather_rows(void *dst, int64_t dst_stride, const void *old_rows, int64_t old_stride, const void *rows,
                       int64_t rows_stride, const int64_t *index, const int32_t *src, int32_t n_old, int32_t n,
                       int64_t genes, int32_t dtype, void *stream) {
  if (n < 0 || n_old < 0 || genes < 1 || (dtype != PG_F32 && dtype != PG_F64) ||
      (n > 0 && (!dst || !src || (n_old > 0 && !old_rows) || dst_stride < genes || old_stride < genes ||
                 rows_stride < genes)))
    return fail(PG_ERR_INVALID, "gather_rows: bad sizes, dtype or NULL buffers");
  if (n == 0) return PG_OK;
  if (dtype == PG_F64)
    hipLaunchKernelGGL(k_gather_rows<double>, dim3(n), dim3(256), 0, (hipStream_t)stream, (double *)dst, dst_stride,
                       (const double *)old_rows, old_stride, (const double *)rows, rows_stride, index, src, n_old,
                       genes);
  else
    hipLaunchKernelGGL(k_gather_rows<float>, dim3(n), dim3(256), 0, (hipStream_t)stream, (float *)dst, dst_stride,
                       (const float *)old_rows, old_stride, (const float *)rows, rows_stride, index, src, n_old,
                       genes);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_row_hash(const void *rows, int64_t stride, const int32_t *index, int32_t n, int64_t genes,
                    int32_t dtype, uint64_t *hash, void *stream) {
  if (n < 0 || genes < 0 || (n > 0 && (!rows || !hash || stride < genes)) || (dtype != PG_F32 && dtype != PG_F64))
    return fail(PG_ERR_INVALID, "row_hash: bad sizes, dtype or NULL buffers");
  if (n == 0) return PG_OK;
  if (dtype == PG_F64)
    hipLaunchKernelGGL(k_row_hash<double>, dim3(n), dim3(256), 0, (hipStream_t)stream, (const double *)rows, stride,
                       index, n, genes, hash);
  else
    hipLaunchKernelGGL(k_row_hash<float>, dim3(n), dim3(256), 0, (hipStream_t)stream, (const float *)rows, stride,
                       index, n, genes, hash);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t pg_hof_update(const pg_hof_args *a) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  if (a->maxsize < 0 || a->hof_n < 0 || a->hof_n > a->maxsize || a->pop_n < 0 || !a->new_n ||
      (a->maxsize > 0 && (!a->new_src || !a->new_fitness)) || (a->hof_n > 0 && (!a->hof_fitness || !a->hof_hash)) ||
      (a->pop_n > 0 && (!a->pop_fitness || !a->pop_hash)))
    return fail(PG_ERR_INVALID, "hof_update: bad sizes or NULL buffers");
  // Entries e < hof_n are the old members (items order), entries hof_n + i the
  // population.  Rank = position in ascending (fitness, age) order, age as
  // HallOfFame.keys orders equal fitness: later insertions rank higher.  The
  // hall is a presence bitmap over ranks; its worst member is the lowest
  // present rank, which only moves up while the hall is full (an entrant
  // beats the worst strictly), so each removal is an amortised O(1) scan.
  const int hn = a->hof_n, pn = a->pop_n, n = hn + pn;
  auto fit_of = [&](int e) { return e < hn ? a->hof_fitness[e] : a->pop_fitness[e - hn]; };
  auto hash_of = [&](int e) { return e < hn ? a->hof_hash[e] : a->pop_hash[e - hn]; };
  auto age_of = [&](int e) { return e < hn ? (hn - 1 - e) : e; };  // old member hn-1 is the oldest
  std::vector<int32_t> rank_v, by_rank((size_t)n);
  const int32_t *rank = a->rank;
  if (!rank) {
    std::vector<int32_t> order((size_t)n);
    for (int e = 0; e < n; ++e) order[e] = e;
    std::sort(order.begin(), order.end(), [&](int x, int y) {
      const double fx = fit_of(x), fy = fit_of(y);
      return fx < fy || (fx == fy && age_of(x) < age_of(y));
    });
    rank_v.resize((size_t)n);
    for (int r = 0; r < n; ++r) rank_v[order[r]] = r;
    rank = rank_v.data();
  }
  for (int e = 0; e < n; ++e) {
    if (rank[e] < 0 || rank[e] >= n) return fail(PG_ERR_INVALID, "hof_update: rank[%d]=%d out of range", e, rank[e]);
    by_rank[rank[e]] = e;
  }
  std::vector<uint64_t> present(((size_t)n + 63) / 64, 0);
  // Similarity classes: when every hash is a dense class id in [0, n) (DeviceGA
  // passes torch.unique's inverse), counts are a direct-indexed array; else a
  // flat open-addressing table keyed by the 64-bit row hash.
  bool dense = true;
  for (int e = 0; e < n && dense; ++e) dense = (uint64_t)hash_of(e) < (uint64_t)n;
  std::vector<int32_t> dense_count(dense ? (size_t)n : 0, 0);
  size_t cap = 1;
  if (!dense)
    while (cap < 2 * (size_t)n + 16) cap <<= 1;
  struct Slot {
    uint64_t key;
    int32_t count, used;
  };
  std::vector<Slot> table(dense ? 0 : cap, Slot{0, 0, 0});
  auto count_of = [&](uint64_t key) -> int32_t & {
    if (dense) return dense_count[key];
    size_t i = (size_t)(key * 0x9E3779B97F4A7C15ull) & (cap - 1);
    while (table[i].used && table[i].key != key) i = (i + 1) & (cap - 1);
    if (!table[i].used) table[i] = Slot{key, 0, 1};
    return table[i].count;
  };
  int size = 0, worst = n;  // lowest present rank (n: none)
  auto add = [&](int e) {
    const int r = rank[e];
    present[r >> 6] |= 1ull << (r & 63);
    count_of(hash_of(e)) += 1;
    size += 1;
    worst = r < worst ? r : worst;
  };
  for (int e = 0; e < hn; ++e) add(e);
  for (int i = 0; i < pn; ++i) {
    if (size == 0 && a->maxsize != 0) {  // DEAP: an empty hall takes population[0]
      add(hn);
      continue;
    }
    if (a->maxsize == 0) continue;
    const double f = a->pop_fitness[i];
    if (size >= a->maxsize && !(f > fit_of(by_rank[worst]))) continue;  // ind.fitness > self[-1].fitness
    if (count_of(a->pop_hash[i]) > 0) continue;                        // similar to a member
    if (size >= a->maxsize) {  // remove(-1): the worst, oldest among equal fitness
      present[worst >> 6] &= ~(1ull << (worst & 63));
      count_of(hash_of(by_rank[worst])) -= 1;
      size -= 1;
      size_t wd = (size_t)worst >> 6;
      uint64_t bits = present[wd] & (~0ull << (worst & 63));
      while (!bits && ++wd < present.size()) bits = present[wd];
      worst = bits ? (int)(wd * 64 + __builtin_ctzll(bits)) : n;
    }
    add(hn + i);
  }
  // items order: best first, newest first among equal fitness = descending rank
  int j = 0;
  for (size_t wd = present.size(); wd-- > 0;) {
    uint64_t bits = present[wd];
    while (bits) {
      const int hi = 63 - __builtin_clzll(bits);
      bits &= ~(1ull << hi);
      const int e = by_rank[wd * 64 + hi];
      a->new_src[j] = e;
      a->new_fitness[j] = fit_of(e);
      ++j;
    }
  }
  *a->new_n = j;
  return PG_OK;
}

namespace {
// The hall in place (pg_hof_packed_args.slot_out), for the general scan's
// result: kept members keep their slots; entering candidates take the freed
// slots -- those of the members not kept, in items order, then hof_n,
// hof_n + 1, ... -- in output order (the packed scan does the same inline).
int32_t assign_slots(int hn, int new_n, const int32_t *slot_in, const int32_t *src, int32_t *slot_out) {
  const auto slot_of = [&](int e) { return slot_in ? slot_in[e] : e; };
  std::vector<int32_t> freed;
  std::vector<uint8_t> kept((size_t)hn, 0);
  for (int j = 0; j < new_n; ++j)
    if (src[j] < hn) kept[src[j]] = 1;
  for (int e = 0; e < hn; ++e)
    if (!kept[e]) freed.push_back(slot_of(e));
  size_t next = 0;
  int grow = hn;
  for (int j = 0; j < new_n; ++j) {
    if (src[j] < hn) {
      slot_out[j] = slot_of(src[j]);
    } else if (next < freed.size()) {
      slot_out[j] = freed[next++];
    } else {
      slot_out[j] = grow++;
    }
  }
  if (grow > new_n) return fail(PG_ERR_INVALID, "hof_update_packed: slots beyond the new hall (%d > %d)", grow, new_n);
  return PG_OK;
}
}  // namespace

int32_t pg_hof_update_packed(const pg_hof_packed_args *a) {
  if (!a) return fail(PG_ERR_INVALID, "args is NULL");
  const int hn = a->hof_n, k = a->k;
  if (a->maxsize < 0 || hn < 0 || hn > a->maxsize || k < 0 || !a->new_n || (a->maxsize > 0 && (!a->new_src || !a->new_fitness)) ||
      (hn > 0 && !a->hof_fitness) || (hn + k > 0 && !a->packed))
    return fail(PG_ERR_INVALID, "hof_update_packed: bad sizes or NULL buffers");
  if (a->slot_in && hn > 0) {  // (a min/max pass the compiler vectorises: the scan is on the generation's path)
    int32_t lo = a->slot_in[0], hi = a->slot_in[0];
    for (int e = 1; e < hn; ++e) {
      lo = a->slot_in[e] < lo ? a->slot_in[e] : lo;
      hi = a->slot_in[e] > hi ? a->slot_in[e] : hi;
    }
    if (lo < 0 || hi >= hn) return fail(PG_ERR_INVALID, "hof_update_packed: slot_in outside [0, hof_n) (%d..%d)", lo, hi);
  }
  const int64_t *pk = a->packed;
  const int n = hn + k;
  auto rank_of = [&](int e) { return (int32_t)(uint32_t)pk[e]; };
  auto class_of = [&](int e) { return (int32_t)(pk[e] >> 32); };
  auto cand_fit = [&](int c) {
    double f;
    std::memcpy(&f, &pk[n + c], sizeof(double));
    return f;
  };
  // the general scan: the packing decoded (an empty hall's first entrant, or
  // members whose ranks are not descending)
  const auto general = [&]() -> int32_t {
    std::vector<int32_t> rank((size_t)n);
    std::vector<uint64_t> hh((size_t)hn), ph((size_t)k);
    std::vector<double> pf((size_t)k);
    for (int e = 0; e < n; ++e) {
      rank[e] = rank_of(e);
      if (e < hn) hh[e] = (uint64_t)class_of(e);
      else ph[e - hn] = (uint64_t)class_of(e);
    }
    for (int c = 0; c < k; ++c) pf[c] = cand_fit(c);
    pg_hof_args g;
    g.maxsize = a->maxsize;
    g.hof_n = hn;
    g.hof_fitness = a->hof_fitness;
    g.hof_hash = hh.data();
    g.pop_n = k;
    g.pop_fitness = pf.data();
    g.pop_hash = ph.data();
    g.rank = rank.data();
    g.new_n = a->new_n;
    g.new_src = a->new_src;
    g.new_fitness = a->new_fitness;
    const int32_t rc = pg_hof_update(&g);
    if (rc != PG_OK || !a->slot_out) return rc;
    return assign_slots(hn, *a->new_n, a->slot_in, a->new_src, a->slot_out);
  };
  if (a->maxsize == 0) {
    *a->new_n = 0;
    return PG_OK;
  }
  if (hn == 0) return general();
  for (int e = 1; e < hn; ++e)
    if (rank_of(e) >= rank_of(e - 1)) return general();  // members not in items order
  for (int c = 0; c < k; ++c)
    if (class_of(hn + c) < 0 || class_of(hn + c) >= n) return fail(PG_ERR_INVALID, "hof_update_packed: class out of range");
  // accepted candidates present in the hall: a bitmap over the entries'
  // ranks (cmin = its lowest set bit) and rank -> candidate; their classes'
  // counts (candidate classes are >= hn)
  std::vector<uint64_t> cbits(((size_t)n + 63) / 64, 0);
  std::unique_ptr<int32_t[]> cand_at(new int32_t[(size_t)n]);  // read only where a bit is set
  int cmin = n;
  std::vector<int32_t> ccount((size_t)k, 0);
  // accepted candidates whose class is a member's (their row equals a member
  // evicted before them): rare, so a small map instead of an array of hof_n
  std::unordered_map<int32_t, int32_t> mcount;
  int p = hn - 1;  // members 0..p present: eviction takes the tail first
  int size = hn;
  for (int c = 0; c < k; ++c) {
    const double f = cand_fit(c);
    const int cls = class_of(hn + c);
    // the worst present entry: the tail member or the lowest-ranked accepted candidate
    const bool cand_worst = cmin < n && (p < 0 || cmin < rank_of(p));
    if (size >= a->maxsize) {  // ind.fitness > self[-1].fitness
      const double fw = cand_worst ? cand_fit(cand_at[cmin]) : a->hof_fitness[p];
      if (!(f > fw)) continue;
    }
    if (cls < hn ? (cls <= p || mcount.count(cls) > 0) : ccount[cls - hn] > 0) continue;  // similar to a present entry
    if (size >= a->maxsize) {  // remove(-1)
      if (cand_worst) {
        const int wc = class_of(hn + cand_at[cmin]);
        if (wc >= hn) {
          ccount[wc - hn] -= 1;
        } else if (--mcount[wc] == 0) {
          mcount.erase(wc);
        }
        cbits[(size_t)cmin >> 6] &= ~(1ull << (cmin & 63));
        size_t wd = (size_t)cmin >> 6;
        uint64_t bits = cbits[wd];
        while (!bits && ++wd < cbits.size()) bits = cbits[wd];
        cmin = bits ? (int)(wd * 64 + __builtin_ctzll(bits)) : n;
      } else {
        p -= 1;
      }
      size -= 1;
    }
    const int r = rank_of(hn + c);
    cbits[(size_t)r >> 6] |= 1ull << (r & 63);
    cand_at[r] = c;
    cmin = r < cmin ? r : cmin;
    if (cls >= hn) ccount[cls - hn] += 1;
    else mcount[cls] += 1;
    size += 1;
  }
  // items order: members 0..p (descending rank) merged with the present
  // candidates by descending rank (the bitmap walked down), member runs
  // copied as ranges
  // (slot_out: a member run keeps its slots; a candidate takes the next freed
  // slot -- the evicted tail p+1..hn-1's, then hn, hn + 1, ...)
  int32_t *so = a->slot_out;
  int freed = p + 1, grow = hn;
  const auto member_run = [&](int j0, int from, int to) {
    for (int e = from; e < to; ++e) a->new_src[j0 + e - from] = e;
    std::memcpy(a->new_fitness + j0, a->hof_fitness + from, sizeof(double) * (size_t)(to - from));
    if (so) {
      if (a->slot_in) std::memcpy(so + j0, a->slot_in + from, sizeof(int32_t) * (size_t)(to - from));
      else
        for (int e = from; e < to; ++e) so[j0 + e - from] = e;
    }
  };
  int j = 0, m = 0;  // output position, next member
  for (size_t wd = cbits.size(); wd-- > 0;) {
    uint64_t bits = cbits[wd];
    while (bits) {
      const int hi = 63 - __builtin_clzll(bits);
      bits &= ~(1ull << hi);
      const int r = (int)(wd * 64 + hi), c = cand_at[r];
      int lo = m;  // the members ranked above this candidate
      while (lo <= p && rank_of(lo) > r) ++lo;
      member_run(j, m, lo);
      j += lo - m;
      m = lo;
      a->new_src[j] = hn + c;
      a->new_fitness[j] = cand_fit(c);
      if (so) so[j] = freed < hn ? (a->slot_in ? a->slot_in[freed++] : freed++) : grow++;
      ++j;
    }
  }
  if (p + 1 > m) member_run(j, m, p + 1);
  j += p + 1 > m ? p + 1 - m : 0;
  *a->new_n = j;
  if (so && grow > j) return fail(PG_ERR_INVALID, "hof_update_packed: slots beyond the new hall (%d > %d)", grow, j);
  return PG_OK;
}

}  // extern "C"
