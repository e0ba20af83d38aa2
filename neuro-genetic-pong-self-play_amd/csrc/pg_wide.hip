// pg_wide.hip -- k_wide: evaluate() (main.py:28-66) for wide two-hidden-layer
// networks [6, H1, H2, O] (BASELINE config 5: [6, 512, 512, 3], 267 779 genes).
//
// A wide network does not fit in registers (1 MB of f32 weights), so its
// weights are STREAMED from HBM every frame.  One 512-thread workgroup per CU
// plays all n_games (6) games of one genome in lockstep, so the genome's W2
// (the 512 x 513 matrix that is 98 % of the genes) is read once per frame for
// all six games; each NN opponent's W2 is read once per frame for its game.
// Per frame:
//   A  wave 0, one lane per game: physics step, centroids, features, the
//      scripted left paddles; the set of networks that must run this frame
//      (ball visible: get_actions main.py:143-153) goes to LDS.
//   B  layer 1, thread j = hidden unit j, every needed column.
//   C  layer 2: W2 tiles of 512 rows x K columns (128 B per row) pass
//      HBM -> registers -> LDS (two tiles in flight per block), thread t owns
//      row t and accumulates its dot product in np.dot's order (four partial
//      sums k mod 4, blas_dot); the genome's tile serves its six games' columns.
//   D  layer 3: one thread per (column, output).
//   E  wave 0: argmax, clamp, bookkeeping, termination, results.
// Every dot product is np.dot's own operation sequence (numpy_nn.py:126-129:
// W . [h; 1] through OpenBLAS dgemv_t, pg_device.hpp blas_dot) with the same
// sigmoid as k_general, so k_wide and k_general agree bit for bit; the
// streamed weights are exact (f32 or f64 genomes, widened to f64).
#include <hip/hip_runtime.h>

#include "pg_eval.hpp"

namespace pg {

constexpr int kWideThreads = 512;  // = max H2: one W2 row per thread
constexpr int kWideMaxGames = 8;

// W2 tile: 128 B of each of the 512 rows, at a 144 B pitch in LDS (16 lanes'
// ds_read_b128 of their own rows hit 16 distinct 16-B bank groups).
constexpr int kTileRowBytes = 128, kTilePitch = 144;
#ifndef PG_WIDE_DEPTH
#define PG_WIDE_DEPTH 2
#endif
constexpr int kDepth = PG_WIDE_DEPTH;  // register sets in the W2 tile ring (2 and 3 measured equal)

// LDS carve (bytes): feats [NC][8] f64 | outputs [NC][4] f64 | control |
// opponent rows | rally keys | h1 [C2][NC] f64 | tile [512][144 B], reused for
// h2 [C3][NC] f64 after layer 2.
constexpr int kOffOut = 1024, kOffCtl = 1536, kOffOrow = 1920, kOffRally = 2048, kOffH1 = 2304;
__host__ __device__ constexpr int align16(int v) { return (v + 15) & ~15; }

__host__ __device__ inline int wide_lds_bytes(int NC, int H1, int H2, int b) {
  const int h1 = align16((H1 + b) * NC * 8);
  const int tile = kWideThreads * kTilePitch;
  const int h2 = align16((H2 + b) * NC * 8);
  return kOffH1 + h1 + (tile > h2 ? tile : h2);
}

// numpy's sigmoid, out of line: one copy of the libm pow instead of one per
// unrolled column keeps the layer loops' register pressure low
__device__ __noinline__ double sigmoid_f64_call(double z) { return sigmoid_f64(z); }

// index of the q-th set bit of m (q < popcount(m))
__device__ __forceinline__ int nth_set_bit(unsigned m, int q) {
  for (int i = 0; i < q; ++i) m &= m - 1;
  return __builtin_ctz(m);
}

// np.argmax over O activations: the first NaN if any, else the first maximum
__device__ __forceinline__ int argmax_np(const double *v, int O) {
  int best = 0;
  for (int j = 1; j < O && !__builtin_isnan(v[best]); ++j)
    if (__builtin_isnan(v[j]) || v[j] > v[best]) best = j;
  return best;
}

// A decision no bound settles (pg_eval_args.hard_log): the two largest
// activations within 1e-12 of each other, not both saturated at 1.0.
__device__ __forceinline__ bool near_tie(const double *v, int O) {
  double t1 = -1.0, t2 = -1.0;
  for (int j = 0; j < O; ++j) {
    const double x = v[j];
    if (x > t1) { t2 = t1; t1 = x; } else if (x > t2) { t2 = x; }
  }
  return t1 - t2 <= 1e-12 && !(t2 == 1.0);
}
__device__ __noinline__ void log_wide(const EvalParams &p, int row, int is_opp, int idx, const double *x) {
  int k[6];
  for (int i = 0; i < 6; ++i) k[i] = (int)rint(x[i] * 320.0);  // the doubled centroids back from k/320
  log_hard(p, row, is_opp, idx, 1, k);
}

// Diagnostic build (-DPG_WIDE_STAMPS): thread 0 adds the shader-clock cycles
// between the frame's phase boundaries into counters[4..6] (A+E+B, C, D).
#ifdef PG_WIDE_STAMPS
#define PG_STAMP(i)                                                        \
  do {                                                                     \
    if (t == 0) {                                                          \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();                  \
      stamp_acc[(i) == 0 ? 0 : (i) == 1 ? 0 : (i) == 2 ? 1 : 2] += now_ - stamp_last; \
      stamp_last = now_;                                                   \
    }                                                                      \
  } while (0)
#else
#define PG_STAMP(i) \
  do {              \
  } while (0)
#endif

template <int NG, typename WT>
__global__ __launch_bounds__(kWideThreads) void k_wide(EvalParams p) {
#ifdef PG_WIDE_STAMPS
  uint64_t stamp_acc[3] = {0, 0, 0}, stamp_last = __builtin_amdgcn_s_memtime();
#endif
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  constexpr int NC = 2 * NG;  // columns: right (genome) of game c = c, left (opponent) of game c = NG + c
  constexpr int K = kTileRowBytes / (int)sizeof(WT);
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int b = p.bias;
  const int H1 = p.nodes[1], H2 = p.nodes[2], O = p.nodes[3];
  const int C1 = 6 + b, C2 = H1 + b, C3 = H2 + b;
  const long W1n = (long)H1 * C1, W2n = (long)H2 * C2;
  const int T = (C2 + K - 1) / K;  // tiles per W2

  double *feat = (double *)lds_raw;              // [NC][8]
  double *outv = (double *)(lds_raw + kOffOut);  // [NC][4]
  int *ctl = (int *)(lds_raw + kOffCtl);         // [0] genome; frame-parity halves at [8..] and [40..]
  long long *orow = (long long *)(lds_raw + kOffOrow);  // [NG] opponent row offsets (elements)
  uint64_t *rkey = (uint64_t *)(lds_raw + kOffRally);    // [NG] Brent's saved rally key per game
  int *rat = (int *)(lds_raw + kOffRally + 64), *rspan = (int *)(lds_raw + kOffRally + 96);
  double *h1 = (double *)(lds_raw + kOffH1);            // [C2][NC]
  unsigned char *tile = lds_raw + kOffH1 + align16(C2 * NC * 8);
  double *h2 = (double *)tile;  // [C3][NC], after layer 2

  const WT *genomes = (const WT *)p.genomes;
  const WT *opponents = (const WT *)p.opponents;
  const int n_games = p.n_games;
  uint64_t c_steps = 0, c_fwd = 0, c_games = 0, c_streams = 0, c_skip = 0;
  const int n_genomes_active = active_genomes(p);

  for (;;) {  // genomes, one per workgroup at a time
    if (t == 0) ctl[0] = (int)atomicAdd(p.work, 1u);
    __syncthreads();
    const int gi = ctl[0];
    if (gi >= n_genomes_active) break;
    const int grow = genome_row(p, gi);
    const WT *gbase = genomes + (long)grow * p.gstride;

    // game state: wave 0, lane g < n_games
    Pong st;
    int act_r = 0, act_l = 0, timeout = 0, total = 0, frames = 0, kind = 0, w = 0;
    bool active = false;
    if (wid == 0 && lane < n_games) {
      w = gi * n_games + lane;
      kind = p.kind[w];
      orow[lane] = kind == kOppNN ? (long long)p.opp[w] * p.ostride : 0;
      st.reset(game_seed(p.seed, lane), kind == kOppRomCpu);
      active = true;
    }
    for (int fno = 0;; ++fno) {  // frames, all games in lockstep
      int *cf = ctl + 8 + (fno & 1) * 32;  // [0] column mask, [1] any active, [2] nets, [3..] net ids
      // ---- A: env.step + find_stuff + inference features (main.py:77-87)
      int s1b = 0, s2b = 0, vis = 0, lc2 = 0, rc2 = 0, left = 0;
      if (wid == 0) {
        if (active) {
          s1b = st.s1;
          s2b = st.s2;
          const int pvis = st.vis, pbx2 = 2 * st.bx + kBallW - 1, pby2 = 2 * st.by + kBallH - 1;
          st.step(act_r, act_l);
          frames += 1;
          vis = st.vis;
          const int bx2 = 2 * st.bx + kBallW - 1, by2 = 2 * st.by + kBallH - 1;
          lc2 = paddle_c2(st.lpy);
          rc2 = paddle_c2(st.rpy);
          if (vis) {  // get_actions main.py:143-150
            const int lbx2 = pvis ? pbx2 : bx2, lby2 = pvis ? pby2 : by2;
            double *fr = feat + lane * 8;
            fr[0] = feat64(bx2); fr[1] = feat64(by2); fr[2] = feat64(lbx2);
            fr[3] = feat64(lby2); fr[4] = feat64(rc2); fr[5] = feat64(lc2); fr[6] = 1.0;
            if (kind == kOppNN) {
              double *fl = feat + (NG + lane) * 8;
              fl[0] = feat64_flip(bx2); fl[1] = feat64(by2); fl[2] = feat64_flip(lbx2);
              fl[3] = feat64(lby2); fl[4] = feat64(lc2); fl[5] = feat64(rc2); fl[6] = 1.0;
            } else if (kind == kOppScore) {
              left = (st.s1 <= st.s2) ? hardcoded(by2, lc2) : 0;
            } else {
              left = hardcoded(by2, lc2);
            }
          }
        }
        const uint64_t rb = __ballot(active && vis);
        const uint64_t lb = __ballot(active && vis && kind == kOppNN);
        const uint64_t ab = __ballot(active);
        if (lane == 0) {
          cf[0] = (int)((unsigned)rb | ((unsigned)lb << NG));
          cf[1] = ab != 0;
          int nn = 0;
          if (rb) cf[3 + nn++] = 0;
          for (int c = 0; c < NG; ++c)
            if ((lb >> c) & 1) cf[3 + nn++] = 1 + c;
          cf[2] = nn;
        }
      }
      __syncthreads();
      PG_STAMP(0);
      const unsigned mask = (unsigned)cf[0];
      if (!cf[1]) break;
      const int n_nets = cf[2];
      c_streams += n_nets;  // uniform: every thread counts, thread 0 reports

      if (mask) {
        // ---- B: layer 1, h1 = S(W1 . [x; 1]) per needed column (numpy_nn.py:126-129)
        for (int j = t; j < H1; j += kWideThreads) {
          if (mask & ((1u << NG) - 1)) {
            const WT *row = gbase + (long)j * C1;
            double wv[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) wv[i] = (i < C1) ? (double)row[i] : 0.0;
#pragma unroll
            for (int c = 0; c < NG; ++c) {
              if (!((mask >> c) & 1)) continue;
              const double *x = feat + c * 8;
              h1[j * NC + c] = sigmoid_f64_call(blas_dot6(wv, x, b));
            }
          }
#pragma unroll
          for (int c = 0; c < NG; ++c) {
            if (!((mask >> (NG + c)) & 1)) continue;
            const WT *row = opponents + orow[c] + (long)j * C1;
            const double *x = feat + (NG + c) * 8;
            double wo[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) wo[i] = (i < C1) ? (double)row[i] : 0.0;
            h1[j * NC + NG + c] = sigmoid_f64_call(blas_dot6(wo, x, b));
          }
        }
        if (b && t < NC) h1[H1 * NC + t] = 1.0;
        __syncthreads();
        PG_STAMP(1);

        // ---- C: layer 2, W2 streamed in tiles; thread t accumulates row t.
        // A tile is 128 B of every row (K = 128 / sizeof(WT) columns); lane
        // t loads 16 B pieces (chunk t % 8 of rows t / 8 + 64 it), so each
        // wave-instruction reads 8 rows x 128 B.  Tiles pass through a ring
        // of kDepth register sets: while tile s is multiplied out of LDS,
        // tiles s+1 .. s+kDepth are in flight.
        // Row sums in np.dot's order (pg_device.hpp blas_dot; C2 <= 513 is one
        // block): four partial sums k mod 4 over k < m2 (kind 0: fused
        // multiply-add; kind 1: two sums k mod 2; kind 2: rounded products),
        // the m3 = C2 & 3 trailing weights kept for the tail after the last tile.
        const int kind2 = blas_kind(t, H2);
        const int m3 = C2 & 3, m2 = C2 - m3;
        double zg[NG][4];  // the genome's partial sums (per game)
        double zp[4];      // the current opponent network's partial sums
        double zop[NG];    // finished opponents' row sums (written once per network pass)
        double tw[3] = {0.0, 0.0, 0.0};  // the current network's tail weights
        double tg[3] = {0.0, 0.0, 0.0};  // the genome's tail weights
#pragma unroll
        for (int c = 0; c < NG; ++c) {
          zop[c] = 0.0;
#pragma unroll
          for (int l = 0; l < 4; ++l) zg[c][l] = 0.0;
        }
#pragma unroll
        for (int l = 0; l < 4; ++l) zp[l] = 0.0;
        const int S = n_nets * T;
        const int lane_off = (t >> 3) * C2 * (int)sizeof(WT) + (t & 7) * 16;
        const int w2_bytes = H2 * C2 * (int)sizeof(WT);
        // Steps s >= S load through an empty descriptor (no memory traffic), so
        // every issue is unconditional and the waits stay counted.
        // Tile s+kDepth's loads are spread over tile s's arithmetic (one
        // 16-B piece per piece of work): a wave whose loads cannot all be
        // accepted at once keeps computing instead of stalling at the issue.
        struct Src {
          __amdgpu_buffer_rsrc_t rsrc;
          int k0;
        };
        auto source = [&](int s) -> Src {
          const bool valid = s < S;
          const int net = valid ? __builtin_amdgcn_readfirstlane(cf[3 + s / T]) : 0;
          const int k0 = valid ? (s % T) * K : 0;
          const WT *base = (net == 0 ? gbase : opponents + orow[net - 1]) + W1n;
          const uint64_t ad = (uint64_t)base;
          const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ad);
          const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(ad >> 32));
          return {__builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                                    valid ? w2_bytes : 0, 0x00020000),
                  k0};
        };
        auto load = [&](const Src &src, int it) -> uint4 {
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(
              src.rsrc, lane_off, (src.k0 + it * 64 * C2) * (int)sizeof(WT), 0);
          return make_uint4(v[0], v[1], v[2], v[3]);
        };
        auto store = [&](const uint4 (&r)[8]) {
#pragma unroll
          for (int it = 0; it < 8; ++it)
            *(uint4 *)((unsigned char *)tile + (it * 64 + (t >> 3)) * kTilePitch + (t & 7) * 16) = r[it];
        };
        // one weight wk at row position kk (kk % 4 == l) into partial sums a
        auto accum = [&](double (&a)[4], int l, double wk, double h) {
          if (kind2 == 0) {
            a[l] = fma(wk, h, a[l]);
          } else {
            const double pr = __dmul_rn(wk, h);
            if (kind2 == 1) {
              if (l & 1) a[1] = __dadd_rn(a[1], pr); else a[0] = __dadd_rn(a[0], pr);
            } else {
              a[l] = __dadd_rn(a[l], pr);
            }
          }
        };
        // multiply tile s (in LDS) into the row sums and load tile sn into r
        auto compute = [&](int s, uint4 (&r)[8], int sn) {
          const Src src = source(sn);
          bool work = s < S && t < H2;
#ifdef PG_WIDE_NOCOMPUTE
          work = false;  // diagnostic build: streaming only
#endif
          if (!work) {
#pragma unroll
            for (int q = 0; q < 8; ++q) r[q] = load(src, q);
            return;
          }
          const int net = cf[3 + s / T], tl = s % T, k0 = tl * K;
          const int kn = min(K, C2 - k0);
          const bool full = k0 + K <= m2;  // the whole tile is inside the block (no tail, no end)
          const unsigned char *tr = (const unsigned char *)tile + t * kTilePitch;
          constexpr int E = 16 / (int)sizeof(WT);  // weights per 16-B piece
          if (net == 0) {
            if (full && kind2 == 0) {  // the hot case: every element a fused multiply-add
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                const uint4 v = *(const uint4 *)(tr + q * 16);
                r[q] = load(src, q);
                WT wq[E];
                __builtin_memcpy(wq, &v, 16);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                  const int k = q * E + e;
                  const double wk = (double)wq[e];
                  const double *hp = h1 + (k0 + k) * NC;
#pragma unroll
                  for (int c = 0; c < NG; ++c) zg[c][k & 3] = fma(wk, hp[c], zg[c][k & 3]);
                }
              }
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                const uint4 v = *(const uint4 *)(tr + q * 16);
                r[q] = load(src, q);
                WT wq[E];
                __builtin_memcpy(wq, &v, 16);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                  const int k = q * E + e, kk = k0 + k;
                  if (k < kn) {
                    const double wk = (double)wq[e];
                    if (kk < m2) {
                      const double *hp = h1 + kk * NC;
#pragma unroll
                      for (int c = 0; c < NG; ++c) accum(zg[c], k & 3, wk, hp[c]);
                    } else {
#pragma unroll
                      for (int i = 0; i < 3; ++i) tg[i] = (kk - m2 == i) ? wk : tg[i];
                    }
                  }
                }
              }
            }
          } else {
            const double *hp = h1 + NG + net - 1;
            if (tl == 0) {
#pragma unroll
              for (int l = 0; l < 4; ++l) zp[l] = 0.0;
            }
            if (full && kind2 == 0) {
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                const uint4 v = *(const uint4 *)(tr + q * 16);
                r[q] = load(src, q);
                WT wq[E];
                __builtin_memcpy(wq, &v, 16);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                  const int k = q * E + e;
                  zp[k & 3] = fma((double)wq[e], hp[(k0 + k) * NC], zp[k & 3]);
                }
              }
            } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const uint4 v = *(const uint4 *)(tr + q * 16);
              r[q] = load(src, q);
              WT wq[E];
              __builtin_memcpy(wq, &v, 16);
#pragma unroll
              for (int e = 0; e < E; ++e) {
                const int k = q * E + e, kk = k0 + k;
                if (k < kn) {
                  const double wk = (double)wq[e];
                  if (kk < m2) {
                    accum(zp, k & 3, wk, hp[kk * NC]);
                  } else {
#pragma unroll
                    for (int i = 0; i < 3; ++i) tw[i] = (kk - m2 == i) ? wk : tw[i];
                  }
                }
              }
            }
            }
            if (tl == T - 1) {  // once per network pass: the block sum and the tail
              const double y = __dadd_rn(0.0, __dadd_rn(__dadd_rn(zp[0], zp[2]), __dadd_rn(zp[1], zp[3])));
              zop[net - 1] =
                  blas_tail([&](int i) { return tw[i - m2]; }, [&](int i) { return hp[i * NC]; }, m2, m3, y);
            }
          }
        };

        // ring: before step s, LDS holds tile s, set s % kDepth is free and
        // sets (s+1 .. s+kDepth-1) % kDepth hold tiles in flight
        uint4 R[kDepth][8];
#pragma unroll
        for (int d = 0; d < kDepth; ++d) {
          const Src src = source(d);
#pragma unroll
          for (int q = 0; q < 8; ++q) R[d][q] = load(src, q);
        }
        store(R[0]);
        __syncthreads();
        for (int s = 0; s < S; s += kDepth) {
#pragma unroll
          for (int d = 0; d < kDepth; ++d) {
            compute(s + d, R[d], s + d + kDepth);
            __syncthreads();
            store(R[(d + 1) % kDepth]);  // tile s+d+1
            __syncthreads();
          }
        }
        // every tile read is behind the last barrier: h2 may overwrite the tile
        if (t < H2) {
          double zgf[NG];
#pragma unroll
          for (int c = 0; c < NG; ++c) {
            const double y = __dadd_rn(0.0, __dadd_rn(__dadd_rn(zg[c][0], zg[c][2]), __dadd_rn(zg[c][1], zg[c][3])));
            zgf[c] = blas_tail([&](int i) { return tg[i - m2]; }, [&](int i) { return h1[i * NC + c]; }, m2, m3, y);
          }
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            const double zc = c < NG ? zgf[c] : zop[c - NG];
            h2[t * NC + c] = ((mask >> c) & 1) ? sigmoid_f64_call(zc) : 0.0;
          }
        }
        if (b && t < NC) h2[H2 * NC + t] = 1.0;
        __syncthreads();
        PG_STAMP(2);

        // ---- D: layer 3 + output sigmoid, one thread per (needed column, output).
        // The needed networks' W3 rows are first staged into the h1 region
        // (dead after layer 2) by all threads with coalesced loads, as many
        // networks at a time as fit, so the sequential sums read only LDS.
        {
          WT *w3s = (WT *)h1;
          const int per_net = O * C3;
          const int cap = (C2 * NC * 8) / (per_net * (int)sizeof(WT));
          const unsigned rbits = mask & ((1u << NG) - 1);
          for (int g0 = 0; g0 < n_nets; g0 += cap) {
            const int gn = min(cap, n_nets - g0);
            // kW3Batch loads in flight per thread before any LDS store (a
            // load-then-store loop waits out one HBM round trip per element)
            constexpr int kW3Batch = 8;
            for (int i0 = t; i0 < gn * per_net; i0 += kW3Batch * kWideThreads) {
              WT val[kW3Batch];
#pragma unroll
              for (int q = 0; q < kW3Batch; ++q) {
                const int i = i0 + q * kWideThreads;
                const int ii = i < gn * per_net ? i : i0;
                const int slot = ii / per_net, net = cf[3 + g0 + slot];
                const WT *v = (net == 0 ? gbase : opponents + orow[net - 1]) + W1n + W2n;
                val[q] = v[ii - slot * per_net];
              }
#pragma unroll
              for (int q = 0; q < kW3Batch; ++q)
                if (i0 + q * kWideThreads < gn * per_net) w3s[i0 + q * kWideThreads] = val[q];
            }
            __syncthreads();
            const int nchain = __builtin_popcount(mask) * O;
            if (t < nchain) {
              const int o = t % O, c = nth_set_bit(mask, t / O);
              // position of this column's network in the frame's network list
              const int pos = c < NG ? 0 : (rbits ? 1 : 0) + __builtin_popcount((mask >> NG) & ((1u << (c - NG)) - 1));
              if (pos >= g0 && pos < g0 + gn) {
                const WT *v = w3s + (pos - g0) * per_net + o * C3;
                const double *hp = h2 + c;
                const double zz = blas_dot([&](int j) { return (double)v[j]; }, [&](int j) { return hp[j * NC]; },
                                           C3, blas_kind(o, O));
                outv[c * 4 + o] = sigmoid_f64_call(zz);
              }
            }
            __syncthreads();
          }
        }
        PG_STAMP(3);
      }

      // ---- E: actions, clamp, bookkeeping (main.py:88-107, 128-135)
      if (wid == 0 && active) {
        int right = 0;
        if (vis) {
          const int ir = argmax_np(outv + lane * 4, O);
          right = index_to_code(ir);
          if (p.hard_log && near_tie(outv + lane * 4, O)) log_wide(p, grow, 0, ir, feat + lane * 8);
          if (kind == kOppNN) {
            const int il = argmax_np(outv + (NG + lane) * 4, O);
            left = index_to_code(il);
            if (p.hard_log && near_tie(outv + (NG + lane) * 4, O)) log_wide(p, p.opp[w], 1, il, feat + (NG + lane) * 8);
          }
          c_fwd += 1 + (kind == kOppNN ? 1 : 0);
        }
        act_l = clamp_action(lc2, left);
        act_r = clamp_action(rc2, right);
        if (p.trace && w < p.trace_games && frames <= p.trace_cap)
          p.trace[(long)w * p.trace_cap + frames - 1] = (uint8_t)(act_r | (act_l << 2) | (vis << 4));
        if (frames > 1) {
          if (st.s1 == s1b && st.s2 == s2b) {
            timeout += 1;
          } else {
            total += timeout;
            timeout = 0;
          }
        }
#ifndef PG_NO_RALLY_SKIP
        // a periodic rally ends at the timeout with nothing else changed (pg_device.hpp rally_key)
        if (timeout >= kRallyStart && timeout <= kTimeoutThresh && (timeout & (kRallyStride - 1)) == 0 &&
        !p.trace) {
          const uint64_t key = rally_key(st, act_r, act_l);
          if (timeout == kRallyStart) {
            rkey[lane] = key;
            rat[lane] = timeout;
            rspan[lane] = kRallyStart;
          } else if (rkey[lane] == key) {
            const int rest = kTimeoutThresh + 1 - timeout;
            frames += rest;
            c_skip += rest;
            timeout = kTimeoutThresh + 1;
          } else if (timeout - rat[lane] == rspan[lane]) {
            rkey[lane] = key;
            rat[lane] = timeout;
            rspan[lane] *= 2;
          }
        }
#endif
        if (st.s1 >= kWinScore || st.s2 >= kWinScore || st.done() || timeout > kTimeoutThresh) {
          finish_game(p, w, st, frames, total);
          active = false;
          c_steps += frames;
          c_games += 1;
        }
      }
    }
  }
  if (p.counters && wid == 0 && c_games) {
    atomicAdd((unsigned long long *)&p.counters[0], (unsigned long long)(c_steps - c_skip));
    if (c_skip) atomicAdd((unsigned long long *)&p.counters[8], (unsigned long long)c_skip);
    atomicAdd((unsigned long long *)&p.counters[1], (unsigned long long)c_fwd);
    atomicAdd((unsigned long long *)&p.counters[3], (unsigned long long)c_games);
  }
#ifdef PG_WIDE_STAMPS
  if (p.counters && t == 0)
    for (int i = 0; i < 3; ++i) atomicAdd((unsigned long long *)&p.counters[4 + i], (unsigned long long)stamp_acc[i]);
#endif
  if (p.counters && t == 0 && c_streams)  // network passes: each streams W1, W2, W3 of one network once
    atomicAdd((unsigned long long *)&p.counters[7], (unsigned long long)c_streams);
}

bool wide_shape_ok(const pg_net &n, int n_games) {
  return n.n_nodes == 4 && n.nodes[0] == 6 && n.nodes[1] >= 1 && n.nodes[1] <= kWideThreads &&
         n.nodes[2] >= 1 && n.nodes[2] <= kWideThreads && n.nodes[3] >= 1 && n.nodes[3] <= 4 &&
         n_games >= 1 && n_games <= kWideMaxGames;
}

template <int NG, typename WT>
static int32_t launch_wide_t(const EvalParams &p, hipStream_t s) {
  const int lds = wide_lds_bytes(2 * NG, p.nodes[1], p.nodes[2], p.bias);
  if (lds > 160 * 1024) return fail(PG_ERR_UNSUPPORTED, "k_wide needs %d bytes of LDS", lds);
  // above 64 KB of dynamic LDS; an older runtime that rejects the attribute launches anyway
  (void)hipFuncSetAttribute((const void *)k_wide<NG, WT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  (void)hipGetLastError();
  const int cap = num_cus();
  const int grid = p.n_genomes < cap ? p.n_genomes : cap;
  if (grid <= 0) return PG_OK;
  hipLaunchKernelGGL((k_wide<NG, WT>), dim3(grid), dim3(kWideThreads), (size_t)lds, s, p);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t launch_wide(const EvalParams &p, int dtype, hipStream_t s) {
  if (p.n_games <= 6)
    return dtype == PG_F64 ? launch_wide_t<6, double>(p, s) : launch_wide_t<6, float>(p, s);
  return dtype == PG_F64 ? launch_wide_t<8, double>(p, s) : launch_wide_t<8, float>(p, s);
}

}  // namespace pg
