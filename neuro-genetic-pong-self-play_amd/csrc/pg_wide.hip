// pg_wide.hip -- k_wide: evaluate() (main.py:28-66) for wide two-hidden-layer
// networks [6, H1, H2, O] (BASELINE config 5: [6, 512, 512, 3], 267 779 genes).
//
// A wide network does not fit in registers (1 MB of f32 weights), so its
// weights are STREAMED from HBM every frame.  One 512-thread workgroup per CU
// plays all n_games (6) games of one genome in lockstep, so the genome's W2
// (the 512 x 513 matrix that is 98 % of the genes) is read once per frame for
// all six games; each NN opponent's W2 is read once per frame for its game.
// (More than six games per genome: balanced chunks of at most six, one work
// item each.)
// Per frame:
//   A  wave 0, one lane per game: physics step, centroids, features, the
//      scripted left paddles; the set of networks that must run this frame
//      (ball visible: get_actions main.py:143-153) goes to LDS.
//   B  layer 1, thread j = hidden unit j, every needed column.
//   C  layer 2: thread t owns row t of W2 and accumulates its dot product in
//      np.dot's order (four partial sums k mod 4, blas_dot).  Each network's
//      W2 was re-laid TILE-MAJOR into the block's scratch when the genome
//      started (K columns x every row per tile, 16-B pieces row-interleaved),
//      so a wave's load is 1 KB contiguous and line-aligned and goes straight
//      to registers: no LDS staging, no barrier inside the layer; the
//      genome's tile serves its six games' columns.
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
constexpr int kWideMaxGames = 8;  // LDS slots for games (k_wide<NG <= 8>; the product runs NG = 6)

// W2 tiles: kTileRowBytes (K = kTileRowBytes / sizeof(WT) columns) of every
// row, in kPieces 16-B pieces; a wave's piece load is 64 rows x 16 B = 1 KB.
#ifndef PG_WIDE_TILE_BYTES
#define PG_WIDE_TILE_BYTES 128
#endif
constexpr int kTileRowBytes = PG_WIDE_TILE_BYTES;
constexpr int kPieces = kTileRowBytes / 16;
#ifndef PG_WIDE_DEPTH
#define PG_WIDE_DEPTH 2
#endif
constexpr int kDepth = PG_WIDE_DEPTH;  // tiles in flight per wave (register sets of the ring)
// Tile reloads: issued together after the tile's arithmetic (kBurst), so the
// compiler's in-order vmcnt accounting sees tile s's loads followed only by
// the other ring slots' (its waits then let the whole ring stay in flight);
// or one per 16-B piece, interleaved with the arithmetic (-DPG_WIDE_SPREAD).
#ifdef PG_WIDE_SPREAD
constexpr bool kBurst = false;
#else
constexpr bool kBurst = true;
#endif
// Cache policy of the W2 stream's loads: non-temporal (the cache-policy
// operand's nt bit), so the stream does not evict what the frame re-reads
// (W1 rows, h tables, the sigmoid table) -- 930 -> 851 ms per launch at pop
// 4096 (profiles/r02/sweep_wide_c8.log); -DPG_WIDE_PLAIN: default policy.
#ifdef PG_WIDE_PLAIN
constexpr int kStreamPolicy = 0;
#else
constexpr int kStreamPolicy = 2;
#endif
// A scheduling fence after each 16-B piece of a tile: the scheduler would
// otherwise hoist the LDS reads of all 32 columns' activations to the top of
// the tile and spill the partial sums.
#ifndef PG_WIDE_NO_FENCE
#define PG_WIDE_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define PG_WIDE_FENCE() do {} while (0)
#endif

// LDS carve (bytes): feats [NC][8] f64 | outputs [NC][4] f64 | control |
// opponent rows | rally keys | game states [NG] WideGame | h1 [C2][NC] f64
// (W3 staging after layer 2) | h2 [C3][NC] f64 | when they fit: every
// network's W3 [NG + 1][O][C3] WT.
constexpr int kOffOut = 1024, kOffCtl = 1536, kOffOrow = 1920, kOffRally = 2048, kOffGames = 2304,
              kOffCount = 3328, kOffH1 = 3584;

// One game's state between frames, kept in LDS by wave 0 (lane c = game c)
// instead of in VGPRs: every wave of the block carries the frame loop's
// registers, and ~30 of them live across layers 1-3 only for wave 0's
// phases A and E had been spilled around the W2 stream.
struct WideGame {
  Pong st;
  int act_r, act_l, timeout, total, frames, kind, w, active;
  int s1b, s2b, vis, lc2, rc2, left, pad0, pad1;  // this frame's, from phase A to phase E
};
static_assert(sizeof(WideGame) == 128, "WideGame: 8 x 16 B");
// whole-record LDS copies as eight 16-B words (an aggregate copy of the
// struct went through a private-memory temporary)
__device__ __forceinline__ WideGame wg_load(const WideGame *s) {
  uint4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = reinterpret_cast<const uint4 *>(s)[i];
  WideGame g;
  __builtin_memcpy(&g, v, sizeof(g));
  return g;
}
__device__ __forceinline__ void wg_store(WideGame *s, const WideGame &g) {
  uint4 v[8];
  __builtin_memcpy(v, &g, sizeof(g));
#pragma unroll
  for (int i = 0; i < 8; ++i) reinterpret_cast<uint4 *>(s)[i] = v[i];
}

// The thread index as an opaque value at the top of a loop body: what is
// derived from it (per-thread LDS and scratch offsets) is then recomputed in
// the loop instead of hoisted out of it, where ~60 such values had been kept
// live across layer 2's register ring -- and spilled (round 3: 129 spilled
// VGPRs; this and the LDS game records: the frame loop spill-free).
__device__ __forceinline__ int opaque_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}
__device__ __forceinline__ int opaque_zero() {
  int z = 0;
  asm volatile("" : "+v"(z));
  return z;
}
static_assert(kOffGames + kWideMaxGames * (int)sizeof(WideGame) <= kOffCount, "LDS carve");
// wave 0's per-lane counters (env steps, forwards, games, rally frames skipped), in LDS for the same reason
static_assert(kOffCount + kWideMaxGames * 4 * 8 <= kOffH1, "LDS carve");
__host__ __device__ constexpr int align16(int v) { return (v + 15) & ~15; }

__host__ __device__ inline int wide_lds_bytes(int NC, int H1, int H2, int b) {
  return kOffH1 + align16((H1 + b) * NC * 8) + align16((H2 + b) * NC * 8);
}

// The tile-major copy of one network's W2 in a block's scratch (written at
// genome start by wide_prep, read once per frame by layer 2):
//   tile s < T, piece q < kPieces, row r < RP: 16 B (E = 16 / sizeof(WT) weights,
//   columns s*K + q*E ..) at ((s * kPieces + q) * RP + r) * 16;
//   then the tail (columns m2 .. C2-1, at most 3) of row r at (T * kPieces * RP + r) * 16
//   (a second such piece block for f64 weights).
// m2 = C2 - C2 % 4 (blas_dot's block), T = max(1, ceil(m2 / K)), RP = H2 rounded up to 64.
struct WideLayout {
  int T, RP;
  long net_bytes;
};
__host__ __device__ inline WideLayout wide_layout(int H1, int H2, int b, int wt_bytes) {
  const int C2 = H1 + b, m2 = C2 - (C2 & 3), K = kTileRowBytes / wt_bytes;
  WideLayout l;
  l.T = m2 > K ? (m2 + K - 1) / K : 1;
  l.RP = (H2 + 63) & ~63;
  l.net_bytes = (long)(l.T * kPieces + (3 * wt_bytes + 15) / 16) * l.RP * 16;
  return l;
}

// Re-lay the W2 of each network in `need` (bit 0: the genome, bit 1 + c: game
// c's opponent) tile-major into the block's scratch (WideLayout), and copy
// the networks' W3 into LDS when it stays resident.  Thread t
// copies row t, one tile (8 pieces) per batch of loads; consecutive threads
// write consecutive 16 B, so a wave's store is 1 KB contiguous.  Once per
// genome: about 1 % of the weight bytes the genome's frames stream.
template <int NG, typename WT>
__device__ void wide_prep(unsigned char *scratch, const WideLayout lay, const WT *gw2, const WT *ow2,
                          const long long *orow, unsigned need, int C2, int H2, int t, WT *w3r, int n_w3,
                          long w3_off) {
  // W3 (n_w3 = O * C3 weights, w3_off elements after W2's start) of every
  // needed network into LDS for the genome's games (w3r: the LDS copy, or NULL)
  if (w3r) {
    for (int n = 0; n <= NG; ++n) {
      if (!((need >> n) & 1)) continue;
      const WT *src = (n == 0 ? gw2 : ow2 + orow[n - 1]) + w3_off;
      for (int i = t; i < n_w3; i += kWideThreads) w3r[n * n_w3 + i] = src[i];
    }
  }
  constexpr int E = 16 / (int)sizeof(WT), kTP = (3 * (int)sizeof(WT) + 15) / 16;
  const int m3 = C2 & 3, m2 = C2 - m3;
  const long PB = (long)lay.RP * 16;
  for (int n = 0; n <= NG; ++n) {
    if (!((need >> n) & 1) || t >= H2) continue;
    const WT *row = (n == 0 ? gw2 : ow2 + orow[n - 1]) + (long)t * C2;
    unsigned char *dst = scratch + (long)n * lay.net_bytes + t * 16;
    for (int s = 0; s < lay.T; ++s) {
      WT v[kPieces][E];
      const int k0 = s * kPieces * E;
      if (k0 + kPieces * E <= m2) {
#pragma unroll
        for (int q = 0; q < kPieces; ++q)
#pragma unroll
          for (int e = 0; e < E; ++e) v[q][e] = row[k0 + q * E + e];
      } else {
#pragma unroll
        for (int q = 0; q < kPieces; ++q)
#pragma unroll
          for (int e = 0; e < E; ++e) v[q][e] = k0 + q * E + e < m2 ? row[k0 + q * E + e] : WT(0);
      }
#pragma unroll
      for (int q = 0; q < kPieces; ++q) {
        uint4 u;
        __builtin_memcpy(&u, v[q], 16);
        *(uint4 *)(dst + (s * kPieces + q) * PB) = u;
      }
    }
    WT tv[kTP * E];
#pragma unroll
    for (int i = 0; i < kTP * E; ++i) tv[i] = i < m3 ? row[m2 + i] : WT(0);
#pragma unroll
    for (int i = 0; i < kTP; ++i) {
      uint4 u;
      __builtin_memcpy(&u, tv + i * E, 16);
      *(uint4 *)(dst + (lay.T * kPieces + i) * PB) = u;
    }
  }
  // the copies are read back through the vector caches by other waves of the block
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
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
// (the fields, not the EvalParams: a reference to the kernel's parameter
// block makes the compiler copy it to private memory, and every field read
// from there counts as divergent -- layer 2's buffer descriptors included)
__device__ __forceinline__ void log_wide(uint32_t *hard_log, uint64_t *counters, int hard_cap, int row, int is_opp,
                                      int idx, const double *x) {
  int k[6];
  for (int i = 0; i < 6; ++i) k[i] = (int)rint(x[i] * 320.0);  // the doubled centroids back from k/320
  log_hard_raw(hard_log, counters, hard_cap, row, is_opp, idx, 1, k);
}

// Diagnostic build (-DPG_WIDE_STAMPS): thread 0 adds the shader-clock cycles
// between phase boundaries into counters[4] (E + A), [5] (B), [6] (C),
// [10] (D) and [11] (a genome's prep: tile-major W2 copies, W3 to LDS).
#ifdef PG_WIDE_STAMPS
#define PG_STAMP(i)                                                        \
  do {                                                                     \
    if (t == 0) {                                                          \
      const uint64_t now_ = __builtin_amdgcn_s_memtime();                  \
      stamp_acc[i] += now_ - stamp_last;                                   \
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
  uint64_t stamp_acc[5] = {0, 0, 0, 0, 0}, stamp_last = __builtin_amdgcn_s_memtime();
#endif
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  constexpr int NC = 2 * NG;  // columns: right (genome) of game c = c, left (opponent) of game c = NG + c
  constexpr int K = kTileRowBytes / (int)sizeof(WT);
  // wid through readfirstlane: the compiler then knows it (and whatever depends
  // on it only) is wave-uniform, so layer 2's buffer descriptors and scalar
  // offsets stay in SGPRs instead of a per-load waterfall loop
  const int t = threadIdx.x, lane = t & 63, wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int b = p.bias;
  const int H1 = p.nodes[1], H2 = p.nodes[2], O = p.nodes[3];
  const int C1 = 6 + b, C2 = H1 + b, C3 = H2 + b;
  const long W1n = (long)H1 * C1, W2n = (long)H2 * C2;

  double *feat = (double *)lds_raw;              // [NC][8]
  double *outv = (double *)(lds_raw + kOffOut);  // [NC][4]
  int *ctl = (int *)(lds_raw + kOffCtl);         // [0] genome; frame-parity halves at [8..] and [40..]
  long long *orow = (long long *)(lds_raw + kOffOrow);  // [NG] opponent row offsets (elements)
  uint64_t *rkey = (uint64_t *)(lds_raw + kOffRally);    // [NG] Brent's saved rally key per game
  WideGame *games = (WideGame *)(lds_raw + kOffGames);    // [NG] the games' states (wave 0)
  uint64_t *cnt = (uint64_t *)(lds_raw + kOffCount);      // [NG][4] steps, forwards, games, skipped (wave 0)
  int *rat = (int *)(lds_raw + kOffRally + 64), *rspan = (int *)(lds_raw + kOffRally + 96);
  double *h1 = (double *)(lds_raw + kOffH1);            // [C2][NC]
  double *h2 = (double *)(lds_raw + kOffH1 + align16(C2 * NC * 8));  // [C3][NC]
  const WideLayout lay = wide_layout(H1, H2, b, (int)sizeof(WT));
  const int m3 = C2 & 3, m2 = C2 - m3;
  // this block's tile-major W2 copies: net 0 = the genome, 1 + c = game c's opponent
  unsigned char *scratch = (unsigned char *)p.wide_scratch + (long)blockIdx.x * (NG + 1) * lay.net_bytes;
  // [NG + 1][O][C3] W3 copies after the h2 region, or NULL (staged per frame)
  WT *w3r = p.wide_w3_resident ? (WT *)(lds_raw + wide_lds_bytes(NC, H1, H2, b)) : nullptr;

  const WT *genomes = (const WT *)p.genomes;
  const WT *opponents = (const WT *)p.opponents;
  const int n_games = p.n_games;
  // a genome's games in chunks of at most NG: with more than NG games a genome
  // is ceil(n_games / NG) work items of balanced size, each streaming the
  // genome's W2 for its own games (the opponents' streams are per game anyway)
  const int n_chunks = (n_games + NG - 1) / NG;
  const int chunk = (n_games + n_chunks - 1) / n_chunks;
  const bool probe = p.wide_probe_k != nullptr;  // pg_wide_decide (n_games = 1)
  uint64_t c_streams = 0;
  if (t < NG * 4) cnt[t] = 0;  // (the genome loop's first barrier orders this before any use)
  const int n_items = active_genomes(p) * n_chunks;

  for (;;) {  // genomes (or chunks of a genome's games), one per workgroup at a time
    const int t = opaque_tid(), lane = t & 63;
    if (t == 0) ctl[0] = (int)atomicAdd(p.work, 1u);
    __syncthreads();
    const int item = __builtin_amdgcn_readfirstlane(ctl[0]);  // uniform: the genome loop's exit
    if (item >= n_items) break;
    const int gi = item / n_chunks;
    const int g0 = (item - gi * n_chunks) * chunk;  // the item's first game slot
    const int ng = min(chunk, n_games - g0);
    const int grow = genome_row(p, gi);
    const WT *gbase = genomes + (long)grow * p.gstride;

    // game state: wave 0, lane c < ng (game g0 + c), in LDS between the phases (WideGame)
    if (wid == 0 && lane < ng) {
      WideGame g;
      g.w = gi * n_games + g0 + lane;
      // probe (pg_wide_decide): one scripted-opponent "game" whose single frame
      // is the genome on the given features
      g.kind = probe ? kOppHard : p.kind[g.w];
      orow[lane] = g.kind == kOppNN ? (long long)p.opp[g.w] * p.ostride : 0;
      g.st.reset(game_seed(p.seed, g0 + lane), g.kind == kOppRomCpu);
      g.act_r = g.act_l = g.timeout = g.total = g.frames = 0;
      g.active = 1;
      g.s1b = g.s2b = g.vis = g.lc2 = g.rc2 = g.left = g.pad0 = g.pad1 = 0;
      // (an opaque zero in each of the record's constant 16-B words: constant
      // words were materialised at kernel entry and kept in scratch till here)
      const int z = opaque_zero();
      g.st.bx += z;
      g.st.vis += z;
      g.st.point += z;
      wg_store(&games[lane], g);
      rat[lane] = -1;  // no rally search open
    }
    if (wid == 0) {
      const bool nng = lane < ng && !probe && p.kind[gi * n_games + g0 + (lane < ng ? lane : 0)] == kOppNN;
      const uint64_t nb = __ballot(nng);
      if (lane == 0) ctl[1] = 1 | (int)((unsigned)nb << 1);  // networks to re-lay: bit 0 genome, 1 + c opponents
    }
    __syncthreads();
    wide_prep<NG, WT>(scratch, lay, gbase + W1n, opponents + W1n, orow, ctl[1], C2, H2, t, w3r, O * C3, W2n);
    PG_STAMP(4);
    for (int fno = 0;; ++fno) {  // frames, all games in lockstep
      const int t = opaque_tid(), lane = t & 63;
      int *cf = ctl + 8 + (fno & 1) * 32;  // [0] column mask, [1] any active, [2] nets, [3..] net ids
      // ---- A: env.step + find_stuff + inference features (main.py:77-87)
      if (wid == 0) {
        const bool mine = lane < ng;
        WideGame g;
        if (mine) g = wg_load(&games[lane]);
        const bool active = mine && g.active;
        if (active && probe) {  // the given doubled centroids (log_wide's k) in place of a frame
          g.vis = 1;
          const int32_t *kk = p.wide_probe_k + (long)gi * 6;
          double *fr = feat + lane * 8;
#pragma unroll
          for (int i = 0; i < 6; ++i) fr[i] = feat64(kk[i]);
          fr[6] = 1.0;
        } else if (active) {
          Pong &st = g.st;
          g.s1b = st.s1;
          g.s2b = st.s2;
          const int pvis = st.vis, pbx2 = 2 * st.bx + kBallW - 1, pby2 = 2 * st.by + kBallH - 1;
          st.step(g.act_r, g.act_l);
          g.frames += 1;
          g.vis = st.vis;
          const int bx2 = 2 * st.bx + kBallW - 1, by2 = 2 * st.by + kBallH - 1;
          g.lc2 = paddle_c2(st.lpy);
          g.rc2 = paddle_c2(st.rpy);
          g.left = 0;
          if (g.vis) {  // get_actions main.py:143-150
            const int lbx2 = pvis ? pbx2 : bx2, lby2 = pvis ? pby2 : by2;
            double *fr = feat + lane * 8;
            fr[0] = feat64(bx2); fr[1] = feat64(by2); fr[2] = feat64(lbx2);
            fr[3] = feat64(lby2); fr[4] = feat64(g.rc2); fr[5] = feat64(g.lc2); fr[6] = 1.0;
            if (g.kind == kOppNN) {
              double *fl = feat + (NG + lane) * 8;
              fl[0] = feat64_flip(bx2); fl[1] = feat64(by2); fl[2] = feat64_flip(lbx2);
              fl[3] = feat64(lby2); fl[4] = feat64(g.lc2); fl[5] = feat64(g.rc2); fl[6] = 1.0;
            } else if (g.kind == kOppScore) {
              g.left = (st.s1 <= st.s2) ? hardcoded(by2, g.lc2) : 0;
            } else {
              g.left = hardcoded(by2, g.lc2);
            }
          }
        }
        if (active) wg_store(&games[lane], g);
        const uint64_t rb = __ballot(active && g.vis);
        const uint64_t lb = __ballot(active && g.vis && g.kind == kOppNN);
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
      // LDS loads count as divergent: readfirstlane makes the frame's control words uniform
      const unsigned mask = (unsigned)__builtin_amdgcn_readfirstlane(cf[0]);
      if (!__builtin_amdgcn_readfirstlane(cf[1])) break;
      const int n_nets = __builtin_amdgcn_readfirstlane(cf[2]);
      c_streams += n_nets;  // uniform: every thread counts, thread 0 reports

      if (mask) {
        // layer 2's streaming setup and its first kDepth tiles
        constexpr int kTP = (3 * (int)sizeof(WT) + 15) / 16;  // tail pieces per row
        const int T = lay.T;
        const int S = n_nets * T;
        const int PB = lay.RP * 16;  // bytes of one piece of every row
        // Steps s >= S load through an empty descriptor (no memory traffic), so
        // every issue is unconditional and the waits stay counted; a tail
        // piece is fetched only with a network's last tile (out-of-range
        // offset otherwise).
        struct Src {
          __amdgpu_buffer_rsrc_t rsrc;
          int soff;
          uint32_t toff;
        };
        auto source = [&](int s) -> Src {
          const bool valid = s < S;
          const int net = valid ? __builtin_amdgcn_readfirstlane(cf[3 + s / T]) : 0;
          const int tl = valid ? s % T : 0;
          const uint64_t ad = (uint64_t)(scratch + (long)net * lay.net_bytes);
          const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ad);
          const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(ad >> 32));
          Src r;
          r.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0,
                                                     valid ? (int)lay.net_bytes : 0, 0x00020000);
          r.soff = tl * kPieces * PB;
          r.toff = (valid && tl == T - 1) ? (uint32_t)(T * kPieces * PB + t * 16) : 0x80000000u;
          return r;
        };
        auto load = [&](const Src &src, int q) -> uint4 {
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(src.rsrc, t * 16, src.soff + q * PB, kStreamPolicy);
          return make_uint4(v[0], v[1], v[2], v[3]);
        };
        auto load_tail = [&](const Src &src, uint4 (&rt)[kTP]) {
#pragma unroll
          for (int i = 0; i < kTP; ++i) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(src.rsrc, src.toff + i * PB, 0, kStreamPolicy);
            rt[i] = make_uint4(v[0], v[1], v[2], v[3]);
          }
        };
        const bool stream_rows = wid * 64 < H2;  // wave-uniform: a wave past the last row streams nothing
        uint4 R[kDepth][kPieces], RT[kDepth][kTP];
        auto prologue = [&]() {
          if (stream_rows) {
#pragma unroll
            for (int d = 0; d < kDepth; ++d) {
              const Src src = source(d);
#pragma unroll
              for (int q = 0; q < kPieces; ++q) R[d][q] = load(src, q);
              load_tail(src, RT[d]);
            }
          }
        };
        const int j = t;
        WT w1[NG + 1][7];
        auto load_w1 = [&]() {
          if (j < H1) {
#pragma unroll
            for (int n = 0; n <= NG; ++n) {
              const bool need = n == 0 ? (mask & ((1u << NG) - 1)) != 0 : ((mask >> (NG + n - 1)) & 1) != 0;
              const WT *row = (n == 0 ? gbase : opponents + orow[n == 0 ? 0 : n - 1]) + (long)j * C1;
#pragma unroll
              for (int i = 0; i < 7; ++i) w1[n][i] = (need && i < C1) ? row[i] : WT(0);
            }
          }
        };
#ifdef PG_WIDE_W1_FIRST  // experiment: W1 requested ahead of the tiles
        load_w1();
#endif
#ifndef PG_WIDE_LATE_PROLOGUE
        prologue();
#endif

        // ---- B: layer 1, h1 = S(W1 . [x; 1]) per needed column (numpy_nn.py:126-129),
        // thread j = unit j (H1 <= 512), after the frame's first kDepth W2
        // tiles were requested (layer 2 starts with them in flight).  Every
        // needed network's W1 row j is requested at once, the pre-activations
        // go to h1, then the inlined sigmoid runs over all columns, four at a
        // time (unneeded columns compute garbage nobody reads; no call: the
        // tiles in flight stay in VGPRs).
#ifndef PG_WIDE_W1_FIRST
        load_w1();
#endif
        if (j < H1) {
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            if (!((mask >> c) & 1)) continue;
            double w[7];
#pragma unroll
            for (int i = 0; i < 7; ++i) w[i] = (double)w1[c < NG ? 0 : 1 + c - NG][i];
            h1[j * NC + c] = blas_dot6(w, feat + c * 8, b);
          }
#pragma unroll 4
          for (int c = 0; c < NC; ++c) h1[j * NC + c] = sigmoid_f64(h1[j * NC + c]);
        }
        if (b && t < NC) h1[H1 * NC + t] = 1.0;
        __syncthreads();
        PG_STAMP(1);

        // ---- C: layer 2, W2 streamed tile by tile from the block's tile-major
        // copies (wide_prep); thread t accumulates row t in np.dot's order
        // (pg_device.hpp blas_dot; C2 <= 513 is one block): four partial sums
        // k mod 4 over k < m2 (kind 0: fused multiply-add; kind 1: two sums
        // k mod 2; kind 2: rounded products), then the m3 trailing weights (the
        // layout's tail pieces, loaded with the network's last tile).  A wave's
        // piece load is 1 KB contiguous (64 rows x 16 B) and goes straight to
        // registers; tiles pass through a ring of kDepth register sets, the
        // next tile's loads spread over the current tile's arithmetic, so each
        // wave streams on its own -- no barrier until the layer is done.
        const int kind2 = blas_kind(t, H2);
        // wave-uniform: every row of this wave sums with fused multiply-adds
        // (branches on the per-row kind would put the tile loads under
        // divergent control flow)
        const bool wave_k0 = wid * 64 + 64 <= 4 * (H2 >> 2);
        double zg[NG][4];  // the genome's partial sums (per game)
        double zp[4];      // the current opponent network's partial sums
#pragma unroll
        for (int c = 0; c < NG; ++c) {
#pragma unroll
          for (int l = 0; l < 4; ++l) zg[c][l] = 0.0;
        }
#pragma unroll
        for (int l = 0; l < 4; ++l) zp[l] = 0.0;
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
        // the tail weight i (< m3) out of the tail pieces
        auto tail_w = [&](const uint4 (&rt)[kTP], int i) -> double {
          WT tq[kTP * 16 / (int)sizeof(WT)];
          __builtin_memcpy(tq, rt, sizeof(tq));
          return (double)tq[i];
        };
        // multiply tile s (in r / rt) into the row sums and load tile sn into r / rt
        auto compute = [&](int s, uint4 (&r)[kPieces], uint4 (&rt)[kTP], int sn) {
          const Src src = source(sn);
          // rows t >= H2 of a partial last wave sum garbage that is never stored
          const bool work = s < S;
          if (!work) {
#pragma unroll
            for (int q = 0; q < kPieces; ++q) r[q] = load(src, q);
            load_tail(src, rt);
            return;
          }
          const int net = __builtin_amdgcn_readfirstlane(cf[3 + s / T]), tl = s % T, k0 = tl * K;
          const int kn = min(K, m2 - k0);  // this tile's weights inside the block
          const bool full = kn == K;
          constexpr int E = 16 / (int)sizeof(WT);  // weights per 16-B piece
          if (net == 0) {
            if (full && wave_k0) {  // the hot case: every element a fused multiply-add
#pragma unroll
              for (int q = 0; q < kPieces; ++q) {
                const uint4 v = r[q];
                if (!kBurst) r[q] = load(src, q);
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
                PG_WIDE_FENCE();
              }
            } else {
#pragma unroll
              for (int q = 0; q < kPieces; ++q) {
                const uint4 v = r[q];
                if (!kBurst) r[q] = load(src, q);
                WT wq[E];
                __builtin_memcpy(wq, &v, 16);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                  const int k = q * E + e;
                  if (k < kn) {
                    const double *hp = h1 + (k0 + k) * NC;
#pragma unroll
                    for (int c = 0; c < NG; ++c) accum(zg[c], k & 3, (double)wq[e], hp[c]);
                  }
                }
              }
            }
            if (tl == T - 1 && t < H2) {  // the genome's pass is complete: its row sums (pre-activations) to h2
#pragma unroll
              for (int c = 0; c < NG; ++c) {
                const double y =
                    __dadd_rn(0.0, __dadd_rn(__dadd_rn(zg[c][0], zg[c][2]), __dadd_rn(zg[c][1], zg[c][3])));
                h2[t * NC + c] = blas_tail([&](int i) { return tail_w(rt, i - m2); },
                                           [&](int i) { return h1[i * NC + c]; }, m2, m3, y);
              }
            }
          } else {
            const double *hp = h1 + NG + net - 1;
            if (tl == 0) {
#pragma unroll
              for (int l = 0; l < 4; ++l) zp[l] = 0.0;
            }
            if (full && wave_k0) {
#pragma unroll
              for (int q = 0; q < kPieces; ++q) {
                const uint4 v = r[q];
                if (!kBurst) r[q] = load(src, q);
                WT wq[E];
                __builtin_memcpy(wq, &v, 16);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                  const int k = q * E + e;
                  zp[k & 3] = fma((double)wq[e], hp[(k0 + k) * NC], zp[k & 3]);
                }
                PG_WIDE_FENCE();
              }
            } else {
#pragma unroll
              for (int q = 0; q < kPieces; ++q) {
                const uint4 v = r[q];
                if (!kBurst) r[q] = load(src, q);
                WT wq[E];
                __builtin_memcpy(wq, &v, 16);
#pragma unroll
                for (int e = 0; e < E; ++e) {
                  const int k = q * E + e;
                  if (k < kn) accum(zp, k & 3, (double)wq[e], hp[(k0 + k) * NC]);
                }
              }
            }
            if (tl == T - 1 && t < H2) {  // once per network pass: the block sum and the tail, to h2
              const double y = __dadd_rn(0.0, __dadd_rn(__dadd_rn(zp[0], zp[2]), __dadd_rn(zp[1], zp[3])));
              h2[t * NC + NG + net - 1] = blas_tail([&](int i) { return tail_w(rt, i - m2); }, [&](int i) { return hp[i * NC]; },
                                       m2, m3, y);
            }
          }
          if (kBurst) {
#pragma unroll
            for (int q = 0; q < kPieces; ++q) r[q] = load(src, q);
          }
          load_tail(src, rt);
        };

        // ring: before step s, set s % kDepth holds tile s and sets
        // (s+1 .. s+kDepth-1) % kDepth hold tiles in flight
#ifdef PG_WIDE_LATE_PROLOGUE
        prologue();
#endif
        if (stream_rows) {
          for (int s = 0; s < S; s += kDepth) {
#pragma unroll
            for (int d = 0; d < kDepth; ++d) compute(s + d, R[d], RT[d], s + d + kDepth);
          }
        }
        if (t < H2) {
#pragma unroll 4
          for (int c = 0; c < NC; ++c) {
            const double v = sigmoid_f64(h2[t * NC + c]);
            h2[t * NC + c] = ((mask >> c) & 1) ? v : 0.0;
          }
        }
        if (b && t < NC) h2[H2 * NC + t] = 1.0;
        __syncthreads();
        PG_STAMP(2);

        // ---- D: layer 3 + output sigmoid (numpy_nn.py:126-131).  Four threads
        // per (needed column, output): thread l of the quad runs np.dot's
        // partial sum l (kinds 0, 2: i = l mod 4; kind 1: i = l mod 2, l < 2),
        // the quad's first thread combines the sums in dgemv_t's order, adds
        // the tail and takes the sigmoid -- blas_dot's operations exactly.
        // W3 rows come from LDS: resident since the genome started (wide_prep)
        // when they fit, else staged here into the h1 region (dead after
        // layer 2) with coalesced loads, as many networks at a time as fit.
        {
          const int nq = __builtin_popcount(mask) * O;  // chains
          const int m3o = C3 & 3, m2o = C3 - m3o;      // C3 <= 513: one block
          const int qi = t >> 2, l = t & 3;
          const int o = qi % O, c = qi < nq ? nth_set_bit(mask, qi / O) : 0;
          const int kd = blas_kind(o, O);
          const double *hp = h2 + c;
          auto chain = [&](const WT *v) {  // v: W3 row o of column c's network
            double sl = 0.0;
            if (kd == 0) {
#pragma unroll 8
              for (int i = l; i < m2o; i += 4) sl = fma((double)v[i], hp[i * NC], sl);
            } else if (kd == 2) {
#pragma unroll 8
              for (int i = l; i < m2o; i += 4) sl = __dadd_rn(sl, __dmul_rn((double)v[i], hp[i * NC]));
            } else if (l < 2) {
#pragma unroll 8
              for (int i = l; i < m2o; i += 2) sl = __dadd_rn(sl, __dmul_rn((double)v[i], hp[i * NC]));
            }
            const double s1 = __shfl_xor(sl, 1, 4), s2 = __shfl_xor(sl, 2, 4), s3 = __shfl_xor(sl, 3, 4);
            if (l == 0) {
              const double blk = kd == 1 ? __dadd_rn(sl, s1) : __dadd_rn(__dadd_rn(sl, s2), __dadd_rn(s1, s3));
              const double y = m2o ? __dadd_rn(0.0, blk) : 0.0;
              const double zz =
                  blas_tail([&](int i) { return (double)v[i]; }, [&](int i) { return hp[i * NC]; }, m2o, m3o, y);
              outv[c * 4 + o] = sigmoid_f64_call(zz);
            }
          };
          if (w3r) {
            if (qi < nq) chain(w3r + (c < NG ? 0 : 1 + c - NG) * O * C3 + o * C3);
            __syncthreads();
          } else {
            WT *w3s = (WT *)h1;
            const int per_net = O * C3;
            const int cap = (C2 * NC * 8) / (per_net * (int)sizeof(WT));
            const unsigned rbits = mask & ((1u << NG) - 1);
            // position of this thread's column's network in the frame's network list
            const int pos = c < NG ? 0 : (rbits ? 1 : 0) + __builtin_popcount((mask >> NG) & ((1u << (c - NG)) - 1));
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
              if (qi < nq && pos >= g0 && pos < g0 + gn) chain(w3s + (pos - g0) * per_net + o * C3);
              __syncthreads();
            }
          }
        }
        PG_STAMP(3);
      }

      // ---- E: actions, clamp, bookkeeping (main.py:88-107, 128-135)
      if (wid == 0 && lane < ng) {
        WideGame &g = games[lane];  // in place: the fields phase E touches, read and written in LDS
        if (g.active && probe) {
          p.wide_probe_index[gi] = argmax_np(outv, O);
          if (p.wide_probe_act)
            for (int o = 0; o < O; ++o) p.wide_probe_act[(long)gi * O + o] = outv[o];
          g.active = 0;
        } else if (g.active) {
          Pong &st = g.st;
          const int w = g.w;
          int right = 0, left = g.left;
          if (g.vis) {
            const int ir = argmax_np(outv + lane * 4, O);
            right = index_to_code(ir);
            if (p.hard_log && near_tie(outv + lane * 4, O)) log_wide(p.hard_log, p.counters, p.hard_cap, grow, 0, ir, feat + lane * 8);
            if (g.kind == kOppNN) {
              const int il = argmax_np(outv + (NG + lane) * 4, O);
              left = index_to_code(il);
              if (p.hard_log && near_tie(outv + (NG + lane) * 4, O)) log_wide(p.hard_log, p.counters, p.hard_cap, p.opp[w], 1, il, feat + (NG + lane) * 8);
            }
            cnt[lane * 4 + 1] += 1 + (g.kind == kOppNN ? 1 : 0);
          }
          g.act_l = clamp_action(g.lc2, left);
          g.act_r = clamp_action(g.rc2, right);
          if (p.trace && w < p.trace_games && g.frames <= p.trace_cap)
            p.trace[(long)w * p.trace_cap + g.frames - 1] = (uint8_t)(g.act_r | (g.act_l << 2) | (g.vis << 4));
          if (g.frames > 1) {
            if (st.s1 == g.s1b && st.s2 == g.s2b) {
              g.timeout += 1;
            } else {
              g.total += g.timeout;
              g.timeout = 0;
              rat[lane] = -1;  // a point: the next rally searches afresh
            }
          }
#ifndef PG_NO_RALLY_SKIP
          // a periodic rally ends at the timeout with nothing else changed (pg_device.hpp
          // rally_key); no state of a point recurs before its kRallyHits-th return
          if (st.hits >= kRallyHits && g.timeout <= p.timeout_thresh && (g.timeout & (kRallyStride - 1)) == 0 &&
              !p.trace) {
            const uint64_t key = rally_key(st, g.act_r, g.act_l);
            if (rat[lane] < 0) {
              rkey[lane] = key;
              rat[lane] = g.timeout;
              rspan[lane] = kRallySpan0;
            } else if (rkey[lane] == key) {
              const int rest = p.timeout_thresh + 1 - g.timeout;
              g.frames += rest;
              cnt[lane * 4 + 3] += rest;
              g.timeout = p.timeout_thresh + 1;
            } else if (g.timeout - rat[lane] >= rspan[lane]) {
              rkey[lane] = key;
              rat[lane] = g.timeout;
              rspan[lane] *= 2;
            }
          }
#endif
          if (st.s1 >= p.win_score || st.s2 >= p.win_score || st.done() || g.timeout > p.timeout_thresh) {
            finish_game(p, w, st, g.frames, g.total);
            g.active = 0;
            cnt[lane * 4 + 0] += g.frames;
            cnt[lane * 4 + 2] += 1;
          }
        }
      }
    }
  }
  if (p.counters && wid == 0 && lane < NG && cnt[lane * 4 + 2]) {
    const uint64_t c_steps = cnt[lane * 4], c_fwd = cnt[lane * 4 + 1], c_games = cnt[lane * 4 + 2],
                   c_skip = cnt[lane * 4 + 3];
    atomicAdd((unsigned long long *)&p.counters[0], (unsigned long long)(c_steps - c_skip));
    if (c_skip) atomicAdd((unsigned long long *)&p.counters[8], (unsigned long long)c_skip);
    atomicAdd((unsigned long long *)&p.counters[1], (unsigned long long)c_fwd);
    atomicAdd((unsigned long long *)&p.counters[3], (unsigned long long)c_games);
  }
#ifdef PG_WIDE_STAMPS
  if (p.counters && t == 0)
    for (int i = 0; i < 5; ++i)
      atomicAdd((unsigned long long *)&p.counters[i < 3 ? 4 + i : 7 + i], (unsigned long long)stamp_acc[i]);
#endif
  if (p.counters && t == 0 && c_streams)  // network passes: each streams W1, W2, W3 of one network once
    atomicAdd((unsigned long long *)&p.counters[7], (unsigned long long)c_streams);
}

bool wide_shape_ok(const pg_net &n, int n_games) {
  return n.n_nodes == 4 && n.nodes[0] == 6 && n.nodes[1] >= 1 && n.nodes[1] <= kWideThreads &&
         n.nodes[2] >= 1 && n.nodes[2] <= kWideThreads && n.nodes[3] >= 1 && n.nodes[3] <= 4 &&
         n_games >= 1 && n_games <= 64;
}

// games per work item (k_wide's NG): with f32 genes 6, so GAMES_TO_PLAY = 6
// plays a genome's games in one lockstep pass; more games are split into
// balanced chunks (k_wide<8> spilled 112 VGPRs: round-4 review).  With f64
// genes 4: k_wide<6, double> spilled 25 VGPRs (its wider tail pieces), so a
// 6-game genome is two items of 3 -- the genome's W2 streamed twice per frame
// on the f64-storage path (config 5 and the bench store f32 genes).
static int wide_ng(int dtype) { return dtype == PG_F64 ? 4 : 6; }
static int wide_items(int n_genomes, int n_games, int ng) { return n_genomes * ((n_games + ng - 1) / ng); }

static int wide_grid(int n_items) {
  const int cap = num_cus();
  return n_items < cap ? n_items : cap;
}

size_t wide_workspace_bytes(const pg_eval_args *a) {
  if (!a || a->n_genomes <= 0 || a->net.n_nodes != 4) return 0;
  const int NG = wide_ng(a->net.dtype);
  const WideLayout l = wide_layout(a->net.nodes[1], a->net.nodes[2], a->net.bias ? 1 : 0,
                                   a->net.dtype == PG_F64 ? 8 : 4);
  return (size_t)wide_grid(wide_items(a->n_genomes, a->n_games, NG)) * (size_t)(NG + 1) * (size_t)l.net_bytes;
}

template <int NG, typename WT>
static int32_t launch_wide_t(EvalParams p, void *scratch, hipStream_t s) {
  int lds = wide_lds_bytes(2 * NG, p.nodes[1], p.nodes[2], p.bias);
  if (lds > 160 * 1024) return fail(PG_ERR_UNSUPPORTED, "k_wide needs %d bytes of LDS", lds);
  // W3 resident for the genome's games when it fits beside h1 / h2 (config 5 in f32: 43 KB)
  const int w3_bytes = align16((NG + 1) * p.nodes[3] * (p.nodes[2] + p.bias) * (int)sizeof(WT));
  p.wide_w3_resident = lds + w3_bytes <= 160 * 1024 ? 1 : 0;
  if (p.wide_w3_resident) lds += w3_bytes;
  // above 64 KB of dynamic LDS; an older runtime that rejects the attribute launches anyway
  (void)hipFuncSetAttribute((const void *)k_wide<NG, WT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  (void)hipGetLastError();
  const int grid = wide_grid(wide_items(p.n_genomes, p.n_games, NG));  // wide_workspace_bytes sized the scratch for it
  if (grid <= 0) return PG_OK;
  p.wide_scratch = scratch;
  hipLaunchKernelGGL((k_wide<NG, WT>), dim3(grid), dim3(kWideThreads), (size_t)lds, s, p);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

int32_t launch_wide(const EvalParams &p, int dtype, void *scratch, hipStream_t s) {
  return dtype == PG_F64 ? launch_wide_t<4, double>(p, scratch, s) : launch_wide_t<6, float>(p, scratch, s);
}

}  // namespace pg
