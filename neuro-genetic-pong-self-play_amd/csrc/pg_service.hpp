// pg_service.hpp -- k_service, the split-layout evaluation kernel (see
// pong_ga.hip's header and DESIGN.md section 4.1), and its launcher.
//
// A header so that its layouts can be compiled in two translation units:
// pong_ga.hip instantiates the [6,<=64,O] bench layout L=8, U=16 under the
// iterative-ILP scheduler; pg_service_more.hip the other (L, U) layouts under
// the default one (the iterative scheduler's register allocation crashes the
// ROCm 7.2 compiler on some of them).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/pong_ga.h"
#include "pg_cascade.hpp"
#include "pg_device.hpp"
#include "pg_eval.hpp"
#include "pg_f64math.h"

namespace pg {

// requests the service wave decides together (fast_f64_decide_batch).  1 in
// the product: batches of 4 measured neutral (profiles/r04/sweep_svc_batch_a6.log)
// and their arrays count against every wave's register allocation (round-5 review)
#ifndef PG_SVC_PRIO
#define PG_SVC_PRIO 3
#endif
#ifndef PG_SVC_BATCH
#define PG_SVC_BATCH 1
#endif

// The bench layout (L = 8, U = 16, not the fixed-horizon mode) decides its
// certificate failures inside the game wave (kInline): the whole wave takes
// the still-undecided half-groups one at a time (serve_inline) instead of a
// dedicated service wave answering through an LDS mailbox.  A requester
// waited for its answer either way; the service wave's slot becomes an
// eighth game wave -- two game waves on every SIMD, where the service wave's
// SIMD had one.  PG_INLINE_SVC=0 builds the service-wave form (A/B).
#ifndef PG_INLINE_SVC
#define PG_INLINE_SVC 1
#endif
// the deciding wave's issue priority over its SIMD partner while it decides
// (3 vs 0, same box: the driver's bench 11.40 / 11.46 vs 11.36 / 11.13 ·10^9,
// one sweep launch equal; profiles/r05/bench_ab_b7.log)
#ifndef PG_INLINE_PRIO
#define PG_INLINE_PRIO 3
#endif
#ifndef PG_INLINE_FRAME_BOUND
#define PG_INLINE_FRAME_BOUND 1
#endif
// The fixed-horizon instance too since round 6 (PG_HORIZON_INLINE=0: its
// service wave, as round 5's).
#ifndef PG_HORIZON_INLINE
#define PG_HORIZON_INLINE 1
#endif
template <int L, int U, bool kHorizon>
__host__ __device__ constexpr bool inline_service() {
  return PG_INLINE_SVC && L == 8 && U == 16 && (PG_HORIZON_INLINE || !kHorizon);
}

// One request, by the whole wave (every lane active): the f32 outputs'
// plateau rule, then the two f32 rules again under the frame's own bound
// (frame_bound_wave, from the network's lane records), else the certified f64
// decision, else numpy's own order in f64 (lds: this wave's
// f64_lds_doubles(H, O) scratch).  The answer: the index, bit 8 numpy-order,
// bit 9 certified in f64, bit 10 certified by the frame's bound.
struct InlineReq {
  int k[6];    // the network's own features (x-flipped for the left paddle): the genes' f64 forward
  int kr[6];   // the game's features as the records take them (the flip is in the weights)
  float z[4];
  float e;
  const float *rec;  // the half-group's first lane record
};
template <int U, int HL, int O, typename WT>
__device__ __forceinline__ int serve_inline(const EvalParams &p, const WT *g, InlineReq r, double *lds,
                                                      int lane64, uint64_t *st_acc = nullptr) {
  const int H = p.nodes[1];
  const int b = p.bias;
  float zf[O];
#pragma unroll
  for (int o = 0; o < O; ++o) zf[o] = r.z[o];
#ifdef PG_INLINE_LOG  // diagnostic build: one record per request in p.hard_log {z0..z3, e, frame bound, stage | idx << 8 | wave << 16, network}
  float ef_log = -1.f;
  const auto log_req = [&](int stage, int idx) {
    if (p.hard_log && p.counters && lane64 == 0) {
      const unsigned long long q = atomicAdd((unsigned long long *)&p.counters[9], 1ull);
      if (q < (unsigned long long)p.hard_cap) {
        uint32_t *rec = p.hard_log + q * 8;
        for (int o = 0; o < 4; ++o) rec[o] = __float_as_uint(o < O ? zf[o] : 0.f);
        rec[4] = __float_as_uint(r.e);
        rec[5] = __float_as_uint(ef_log);
        rec[6] = (uint32_t)stage | ((uint32_t)(idx & 255) << 8) |
                 ((uint32_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) << 16);
        rec[7] = (uint32_t)((uint64_t)g >> 3);  // the network (its genome row's address / 8)
      }
    }
  };
#define PG_LOG_REQ(stage, idx) log_req(stage, idx)
#else
#define PG_LOG_REQ(stage, idx)
#endif
#ifdef PG_SERVE_STAGES  // diagnostic build: shader cycles per stage, summed in the wave's st_acc[0..11]
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  uint64_t st_t = __builtin_amdgcn_s_memtime();
  const auto stage_mark = [&](int i) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const uint64_t now = __builtin_amdgcn_s_memtime();
    st_acc[i] += now - st_t;
    st_acc[6 + i] += 1;
    st_t = now;
  };
#define PG_STAGE(i) stage_mark(i)
#else
#define PG_STAGE(i)
#endif
  // the plateau rule under the network's static bound first only where the
  // frame bound does not follow (PG_INLINE_FRAME_BOUND=0): under the frame's
  // bound the same rule decides everything it would (round 6: it settled
  // 0.1 % of the bench's requests and 15 % of --dist init's, at ~2k cycles
  // each; profiles/r06/serve_stages_{normal,init}_c10.log)
  int d = PG_INLINE_FRAME_BOUND ? -1 : plateau_decide<O>(zf, r.e, lane64);
  PG_STAGE(0);
  if (d >= 0) PG_LOG_REQ(1, d);
  // the frame's own bound (frame_bound_wave) before the f64 stage: the lane
  // records' round trip settles ~1/3 of the requests without the genome row's
  // (PG_INLINE_FRAME_BOUND=0, straight to the f64 stage: the headline -4 %,
  // --dist init neutral; profiles/r06/ab_tight_fb_c4.log)
  if (PG_INLINE_FRAME_BOUND && d < 0 && r.e < __builtin_inff()) {  // e = inf: weights over the cap, f64 only
    const float ef = fminf(r.e, frame_bound_wave<HL, U, O>(r.rec, r.kr, lane64));
#ifdef PG_INLINE_LOG
    ef_log = ef;
#endif
    PG_STAGE(1);
    d = certify_c<O>(zf, make_cert(ef));
    if (d < 0) d = plateau_f32<O>(zf, ef);
    if (d < 0) d = plateau_decide<O>(zf, ef, lane64);
    PG_STAGE(2);
    if (d >= 0) {
      PG_LOG_REQ(2, d);
      return d | 1024;
    }
  }
  if (d < 0) {
    d = fast_f64_decide<O, WT>(g, H, b, r.k, lane64);
    PG_STAGE(3);
    if (d >= 0) PG_LOG_REQ(3, d);
  }
  if (d >= 0) return d | 512;
  d = forward_f64_group<64, (U * HL + 63) / 64, O, WT>(g, H, b, r.k, lds, lane64);
  PG_LOG_REQ(4, d);
  PG_STAGE(4);
#undef PG_LOG_REQ
#undef PG_STAGE
#if defined(PG_INLINE_LOG) || defined(PG_SERVE_STAGES)
  if (false) {
#else
  if (p.hard_log && lane64 == 0) {
#endif
    const long oo = g - (const WT *)p.opponents;
    const bool opp = p.opponents != p.genomes && oo >= 0 && oo < (long)p.n_opponents * p.ostride;
    log_hard(p, (int)(opp ? oo / p.ostride : (g - (const WT *)p.genomes) / p.gstride), opp ? 1 : 0, d, 0, r.k);
  }
  return d | 256;
}

// Every network a launch plays, once, in the layout a game lane holds it
// (load_net_pk: pre-scaled f32 weights, the left paddle's x-flip folded in,
// the certificate's bound): record r < n_genomes is entry r's genome as the
// right paddle, record n_genomes + j opponent row j as the left paddle.  HL
// consecutive threads prepare one network (the bound's group sums).
template <int L, int U, int O, typename WT>
__global__ __launch_bounds__(256) void k_prep_records(EvalParams p) {
  constexpr int HL = L / 2;
  constexpr int F = rec_floats<U, O>();
  // the launch before the games: the work header and the counters start at zero
  // (one kernel instead of a memset and a fill ahead of it in the stream)
  if (p.prep != PG_PREP_GENOMES && blockIdx.x == 0) {
    if (threadIdx.x < 64) p.work[threadIdx.x] = 0u;
    if (p.counters && threadIdx.x < 16) p.counters[threadIdx.x] = 0ull;
  }
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  // PG_PREP_GENOMES: records [0, n_genomes); PG_PREP_REST: [n_genomes, n_genomes + n_opponents)
  const long net = t / HL + (p.prep == PG_PREP_REST ? p.n_genomes : 0);
  const int hl = (int)(t % HL);
  const long end = p.prep == PG_PREP_GENOMES ? (long)p.n_genomes : (long)p.n_genomes + p.n_opponents;
  if (net >= end) return;  // whole groups (HL divides 64)
  const WT *g;
  int flip;
  if (net < p.n_genomes) {
    if (net >= active_genomes(p)) return;  // not played by this launch
    g = (const WT *)p.genomes + (long)genome_row(p, (int)net) * p.gstride;
    flip = 0;
  } else {
    g = (const WT *)p.opponents + (net - p.n_genomes) * p.ostride;
    flip = 1;
  }
  NetP<U, O> n;
  load_net_pk<HL, U, O, WT>(n, g, p.nodes[1], p.bias, hl, flip);
  store_rec<U, O>(n, p.recs + (net * HL + hl) * F);
}

#ifdef PG_PROBE_EXTRA
// Timing-only experiment (tools/runs/r5_b2.sh): N independent instructions of
// one class per visible frame, writing a dummy register from live inputs, so
// the games play exactly as in the product and the launch time's change is the
// in-situ issue cost of that class.  Modes: 1 v_rcp_f32 x16, 2 v_exp_f32 x16,
// 3 v_pk_fma_f32 x24, 4 v_fma_f32 x48, 5 v_add_u32 x24,
// 7 v_mov_b32 x24, 8 v_pk_add_f32 x24, 9 v_add_f32 x48.
template <int M>
__device__ __forceinline__ void pg_probe_extra(float2v w, float2v w2, float a, float b, float &v, float2v &pp,
                                               int &sv) {
#pragma unroll
  for (int r = 0; r < (M == 4 || M == 9 ? 48 : (M <= 2 ? 16 : 24)); ++r) {
    if constexpr (M == 1) asm volatile("v_rcp_f32 %0, %1" : "=v"(v) : "v"((r & 1) ? a : b));
    if constexpr (M == 2) asm volatile("v_exp_f32 %0, %1" : "=v"(v) : "v"((r & 1) ? a : b));
    if constexpr (M == 3) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(pp) : "v"(w), "v"(w2), "v"((r & 1) ? w : w2));
    if constexpr (M == 4) asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(v) : "v"(a), "v"(b), "v"((r & 1) ? a : b));
    if constexpr (M == 5) asm volatile("v_add_u32 %0, %1, %2" : "=v"(v) : "v"(a), "v"(b));
    if constexpr (M == 7) asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"((r & 1) ? a : b));
    if constexpr (M == 8) asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(pp) : "v"(w), "v"((r & 1) ? w : w2));
    if constexpr (M == 9) asm volatile("v_add_f32 %0, %1, %2" : "=v"(v) : "v"(a), "v"((r & 1) ? a : b));
  }
}
#endif

// kUntraced: a launch without a trace buffer (the GA's), the trace tests
// compiled out of the frame instead of tested on p.trace every frame.
// kHorizon: SURVEY 8(d)'s fixed-horizon measurement mode (pg_eval_args.horizon,
// untraced): every game slot runs exactly p.horizon frames, episodes auto-reset,
// nothing is advanced in closed form.
template <int L, int U, int O, typename WT, bool kUntraced = false, bool kHorizon = false>
__global__ __launch_bounds__(svc_threads<U>()) void k_service(EvalParams p) {
  constexpr int kSvcThreads = svc_threads<U>();
  constexpr bool kInline = inline_service<L, U, kHorizon>();
  static_assert(!kInline || O <= 4, "InlineReq.z");
  constexpr int kSvcGameWaves = kSvcThreads / 64 - (kInline ? 0 : 1);
  constexpr int HL = L / 2;
  constexpr int kSlots = kSvcGameWaves * (64 / L) * 2;
  __shared__ SlowSlot slots[kSlots];
  // fixed-horizon bookkeeping, one per game group (kHorizon instances only)
  __shared__ HorizonSlot hz[kHorizon ? kSlots / 2 : 1];
  __shared__ int waves_done;
  __shared__ int posted;  // requests posted so far (the service wave polls this one word)
  // every serve of every game slot (Pong::serve_entry is a function of the
  // slot's physics seed and the point): a serve is one ds_read instead of a
  // splitmix64 and a 64-bit remainder; launches with more slots compute them
  __shared__ uint32_t serve_tab[kServeTabSlots * kServeTabPoints];
  extern __shared__ double lds_svc[];  // f64_lds_doubles(H, O): the service wave's, or (kInline) each wave's
  const int H = p.nodes[1];
  const int b = p.bias;
  const int wave = threadIdx.x >> 6;
  const int lane64 = threadIdx.x & 63;
  for (int i = threadIdx.x; i < kSlots; i += kSvcThreads) {
    lds_st(&slots[i].flag, 0);
    slots[i].rec = 0;
  }
  const bool tabbed = p.n_games <= kServeTabSlots;
  if (tabbed)
    for (int i = threadIdx.x; i < p.n_games * kServeTabPoints; i += kSvcThreads)
      serve_tab[i] = Pong::serve_entry(game_seed(p.seed, i / kServeTabPoints), i % kServeTabPoints);
  if (threadIdx.x == 0) {
    lds_st(&waves_done, 0);
    lds_st(&posted, 0);
  }
  __syncthreads();

  if (!kInline && wave == kSvcGameWaves) {
    // ---------------- service wave: f64 re-decisions for the whole block ----
    // the service wave's issue priority over its SIMD partner (a game wave):
    // an answer sooner is a requester's wait shorter (PG_SVC_PRIO 3 vs 0,
    // same box: the driver's bench +4 %, one launch of the sweep neutral,
    // profiles/r05/bench_ab_b6.log, sweep_ab_b6.log)
    if constexpr (PG_SVC_PRIO > 0) __builtin_amdgcn_s_setprio(PG_SVC_PRIO);
    // requests taken together (H <= 64 layouts: one hidden unit per lane)
    constexpr int kSvcBatch = U * HL <= 64 ? PG_SVC_BATCH : 1;
    const WT *genomes_svc = (const WT *)p.genomes;
    // An idle poll reads one word (the posted count): the slot scan runs only
    // when it moved.  A request posted after the read moves it again, so the
    // next poll scans once more; the poster's flag store is ordered before
    // its count increment (LDS operations of a wave complete in order).
    int seen = 0;
    for (;;) {
      const int now = __builtin_amdgcn_readfirstlane(lds_ld(&posted));
      if (now == seen) {
        if (lds_ld(&waves_done) == kSvcGameWaves) break;
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      seen = now;
      for (int base = 0; base < kSlots; base += 64) {
        const int sidx = base + lane64;
        const bool posted = sidx < kSlots && lds_ld(&slots[sidx].flag) == 1;
        unsigned long long mask = __ballot(posted);
        while (mask) {
          // up to kSvcBatch posted requests at once: the plateau rule on their
          // f32 outputs, then the certified f64 decision of the rest with all
          // their weights requested before any arithmetic (fast_f64_decide_batch)
          int sl[kSvcBatch], idx[kSvcBatch], k[kSvcBatch][6];
          const WT *g[kSvcBatch];
          bool need[kSvcBatch];
#pragma unroll
          for (int q = 0; q < kSvcBatch; ++q) {
            sl[q] = -1;
            if (mask) {
              sl[q] = base + __builtin_ctzll(mask);
              mask &= mask - 1;
            }
          }
          __threadfence_block();
#pragma unroll
          for (int q = 0; q < kSvcBatch; ++q) {
            need[q] = false;
            idx[q] = -1;
            g[q] = genomes_svc;
            if (sl[q] >= 0) {
              g[q] = (const WT *)slots[sl[q]].g;
#pragma unroll
              for (int i = 0; i < 6; ++i) k[q][i] = slots[sl[q]].k[i];
              float zf[O];
#pragma unroll
              for (int o = 0; o < O; ++o) zf[o] = slots[sl[q]].z[o];
              idx[q] = plateau_decide<O>(zf, slots[sl[q]].e, lane64);
              need[q] = idx[q] < 0;
            }
          }
          if constexpr (kSvcBatch > 1) {
            int f[kSvcBatch];
            fast_f64_decide_batch<O, WT, kSvcBatch>(g, k, need, H, b, lane64, f);
#pragma unroll
            for (int q = 0; q < kSvcBatch; ++q)
              if (need[q]) idx[q] = f[q];
          } else {
            if (need[0]) idx[0] = fast_f64_decide<O, WT>(g[0], H, b, k[0], lane64);
          }
#pragma unroll
          for (int q = 0; q < kSvcBatch; ++q) {
            if (sl[q] < 0) continue;
            int d = idx[q];
            // bit 8 / bit 9 of the answer: decided by the numpy-order forward / by the certified one
            if (d < 0) {
              d = forward_f64_group<64, (U * HL + 63) / 64, O, WT>(g[q], H, b, k[q], lds_svc, lane64);
              if (p.hard_log && lane64 == 0) {
                const long oo = g[q] - (const WT *)p.opponents;
                const bool opp = p.opponents != p.genomes && oo >= 0 && oo < (long)p.n_opponents * p.ostride;
                log_hard(p, (int)(opp ? oo / p.ostride : (g[q] - (const WT *)p.genomes) / p.gstride), opp ? 1 : 0,
                         d, 0, k[q]);
              }
              d |= 256;
            } else {
              d |= 512;
            }
            if (lane64 == 0) {
              slots[sl[q]].idx = d;
              __threadfence_block();
              lds_st(&slots[sl[q]].flag, 2);
            }
          }
        }
      }
    }
    return;
  }

  // ---------------- game waves: k_split's loop --------------------------------
  const int lig = threadIdx.x & (L - 1);
  const int side = lig >= HL ? 1 : 0;  // 0: right paddle's network, 1: left paddle's
  const int hl = lig & (HL - 1);
  const int leader = lane64 & ~(L - 1);
  // index (not a pointer) into the __shared__ array keeps every mailbox access
  // a ds_* instruction; a SlowSlot * decays to a flat pointer
  // The group's mailbox slots, recomputed from the lane id where a rare block
  // uses them (v_mbcnt in volatile asm, not hoisted): as loop-invariant lane
  // values they were spilled and reloaded from scratch in those blocks.
  const int wave_slot0 = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * (64 / L) * 2;
  const auto slot_grp = [&]() { return wave_slot0 + (fresh_lane64() / L) * 2; };  // the group's side-0 slot
  const auto slot_me = [&]() {  // this half's slot
    const int l = fresh_lane64();
    return wave_slot0 + (l / L) * 2 + ((l & (L - 1)) >= HL ? 1 : 0);
  };
  const WT *genomes = (const WT *)p.genomes;
  const WT *opponents = (const WT *)p.opponents;

  NetP<U, O> net;
  PongK st;  // the game in the features' doubled units (pg_device.hpp)
  // Frame bookkeeping against a wave-scalar frame counter (every lane of the
  // loop steps one frame per iteration): a game's frames = sframe - fstart, its
  // no-score counter (main.py:128-135) = sframe - (tend - TIMEOUT_THRESH), so a
  // plain frame updates neither; total (main.py:73) and the score-based end
  // (main.py:102-107) change only at a point, inside the rare block
  // act_r / act_l: the actions written into action[4:6] / [6:8] (main.py:91-92)
  // as the paddles' moves in centroid units (clamp_move: -6 up, +6 down, 0), which the step adds
  // c_vis: the game's visible frames (a forward each), counted per frame --
  // or, kVisByFrames, the frame counter at its start: an instance that
  // advances every hidden serve delay at once steps exactly one hidden frame
  // per point (the miss), so visible = iterations - points, taken at the end
  int kind = 0, act_r = 0, act_l = 0, total = 0, fstart = 0, tend = 0, c_vis = 0, tab_off = 0;
  int sframe = 0;
#ifndef PG_NO_HIDDEN_JUMP
  constexpr bool kVisByFrames = kUntraced && !kHorizon;
#else
  constexpr bool kVisByFrames = false;
#endif
  const WT *gm = genomes;
  uint32_t slow = 0, c_fwd = 0, c_steps = 0, c_games = 0, fails = 0, plateau = 0, inwave = 0, skipped = 0, hidden = 0;

  const int games_total = active_total(p);
  int w;
  {
    int ww = 0;
    if (lig == 0) ww = (int)atomicAdd(p.work, 1u);
    w = group_broadcast<L>(ww, leader);
  }
  bool fresh = true;
  // kInline: every lane stays in the loop until its wave has no game left
  // (serve_inline needs the whole wave); a group without work is parked as a
  // ball at rest mid-field, visible (vis = 2: no decision, no face, no point)
  // and never timed out, and the wave leaves when none of its groups is live
  bool live = w < games_total;
  const auto park = [&]() {
    st.bx2 = 2 * 79 + kBallW - 1;
    st.by2 = 2 * 78 + kBallH - 1;
    st.vx2 = st.vy2 = 0;
    st.vis = 2;
    st.one_player = 0;
    kind = kOppNN;
    tend = 0x7fffffff;
    fstart = 0x3fffffff;  // (the fixed-horizon end test sframe - fstart >= T never fires either)
    fresh = false;
  };
  if (kInline && !live) park();
  // wave-uniform (kept as scalars: readfirstlane, so no lane mask is rebuilt
  // from a vector copy every frame); set at the first frame's starts
  int w_scripted = 1, w_onep = 1;
  // wave-uniform: some game of the wave starts, or has a hidden ball whose serve
  // delay the top block advances; set where that can change (the top block, the
  // rare block), so a plain frame tests one scalar
  int top = 1;
#ifdef PG_PROBE_EXTRA
  float probe_v = 0.f;
  float2v probe_p = float2v{0.f, 0.f};
  int probe_s = 0;
#endif
#ifdef PG_START_PROBE  // diagnostic build: shader cycles of the game-start blocks vs the wave's total
  uint64_t probe_fresh = 0;
  const uint64_t probe_t0 = __builtin_amdgcn_s_memtime();
#endif
#ifdef PG_SERVE_STAGES  // diagnostic build: serve_inline's cycles per stage (and a second call's, PG_SERVE_TWICE)
  uint64_t st_acc[24];
#pragma unroll
  for (int i = 0; i < 24; ++i) st_acc[i] = 0;
#endif
#ifdef PG_DECIDE_PROBE  // diagnostic build: shader cycles of kInline's f64 decisions (until the reload has landed) vs the wave's total
  uint64_t probe_dec = 0;
  const uint64_t probe_t0 = __builtin_amdgcn_s_memtime();
#endif
#ifdef PG_TIMELINE
  uint64_t t_start = 0;
  uint32_t g_fails = 0, g_slow = 0;
#endif
#ifdef PG_PATH_PROBE  // diagnostic build: wave-frames that take each rare path (any game of the wave)
  uint32_t pp_frames = 0, pp_rally = 0, pp_face = 0, pp_fail = 0, pp_hidden = 0;
#define PG_PP(cnt, cond) \
  if (__builtin_amdgcn_ballot_w64(cond) != 0) cnt += 1
#else
#define PG_PP(cnt, cond)
#endif
  // a group leaves the loop at its game-end block when the queue is empty (no
  // per-frame test); kInline: the wave, when its last live group has ended
  if (kInline ? __builtin_amdgcn_ballot_w64(live) != 0 : live) for (;;) {
#ifdef PG_START_PROBE
    const bool any_fresh = __builtin_amdgcn_ballot_w64(fresh) != 0;
    const uint64_t probe_f0 = __builtin_amdgcn_s_memtime();
#endif
    PG_PP(pp_frames, true);
    sframe += 1;
#ifdef PG_TIMELINE
    constexpr bool kJumps = !kHorizon;
#else
    const bool kJumps = !kHorizon && (kUntraced || p.trace == nullptr);  // the serve delay advanced at once
#endif
    // a game start or a hidden ball: one wave-uniform scalar test on the common path
    if (top) {
    if (fresh) {  // start game w (genome-major: the 6 games of a genome are adjacent)
      const int i = w / p.n_games;
      const int g = w - i * p.n_games;
      kind = p.kind[w];
      const WT *gr = genomes + (long)genome_row(p, i) * p.gstride;
      // the left half: opponent row opp (its record has the x-flip folded in);
      // idle (a copy of the genome) against a scripted opponent.  A network
      // game needs opponents (pong_ga.h); without any, the genome plays itself.
      const bool nn = side && kind == kOppNN && p.n_opponents > 0;
      const int oj = nn ? min(max(p.opp[w], 0), p.n_opponents - 1) : 0;
      gm = nn ? opponents + (long)oj * p.ostride : gr;
      const int rec = nn ? p.n_genomes + oj : i;
      load_rec<U, O>(net, p.recs + ((long)rec * HL + hl) * rec_floats<U, O>());
      const int sx = slot_me();
      if (kInline && hl == 0) slots[sx].rec = rec;
      // the output bias enters the first lane's two partial chains, half each
      // (exact), so the frame adds no bias after the group sum (partial_pk)
#pragma unroll
      for (int o = 0; o < O; ++o) net.c[o] = hl == 0 ? 0.5f * net.c[o] : 0.f;
      st.reset(0, kind == kOppRomCpu);
      // the slot's serve seed: the LDS table holds a tabbed slot's first
      // kServeTabPoints serves; a horizon slot carries its point count across
      // auto-resets past them, where the step falls back to serve_entry(seed, pt)
      if (kHorizon || !tabbed) st.seed = game_seed(p.seed, g);  // (a wave-uniform test)
      tab_off = g * kServeTabPoints;
      act_r = act_l = total = 0;
      c_vis = kVisByFrames ? sframe - 1 : 0;
      fstart = sframe - 1;             // this iteration is the game's frame 1
      tend = sframe + p.timeout_thresh;  // frame 1 does not count (main.py:94-96): it takes the counter to 0
      fresh = false;
      if (hl == 0) slots[sx].n_memo = 0;
      if (lig == 0) slots[sx].rally_at = -1;  // (sx is the side-0 slot there)
      if (kHorizon && lig == 0) {
        const int gx = threadIdx.x / L;
        hz[gx].sum = 0.0;
        hz[gx].eps = hz[gx].s1 = hz[gx].s2 = hz[gx].zd = 0;
      }
#ifdef PG_TIMELINE  // experiment build: per-game wall-clock start/end into p.trace
      t_start = wall_clock64();
      g_fails = g_slow = 0;
#endif
    }
#ifdef PG_START_PROBE
    if (any_fresh) probe_fresh += __builtin_amdgcn_s_memtime() - probe_f0;
#endif
#ifndef PG_NO_HIDDEN_JUMP
    // The serve delay in closed form: while the ball is hidden no point can be
    // scored, nothing is decided by a network (get_actions: [0,0],
    // main.py:151-153) and a paddle only drifts back inside the clamp band
    // (Pong::drift), so the frames before the serve frame are advanced at
    // once -- the same state, actions, timeout and frame counts as stepping
    // them (never while tracing, which records every frame).
    {
      const bool hid = !st.vis && st.timer >= 2;
      PG_PP(pp_hidden, hid);
      if (kJumps && hid) {
        const int h = st.timer - 1;
        st.rc2 = PongK::drift2(st.rc2, h);
        if (!st.one_player) st.lc2 = PongK::drift2(st.lc2, h);
        st.timer = 1;
        act_r = clamp_move(st.rc2, 0);
        act_l = clamp_move(st.lc2, 0);  // (a 1-player env's CPU paddle: unclipped, the same side of the band)
        fstart -= h;  // frames += h, and the no-score counter with them
        tend -= h;
        hidden += h;
      }
    }
#endif
    // the wave's games after any start: is one of them scripted, or a
    // 1-player env (both fixed for a game; no per-frame test otherwise)
    w_scripted = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(kind != kOppNN) != 0);
    w_onep = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(st.one_player != 0) != 0);
    top = 0;  // every start and serve delay above is done
    }
    const int pvis = st.vis, pbx2 = st.bx2, pby2 = st.by2;
#ifdef PG_PATH_PROBE
    const int pt_b = st.point, hits_b = st.hits;
#endif
    const int ev = st.step(act_r, act_l, [&](int pt) {
      return tabbed && pt < kServeTabPoints ? serve_tab[tab_off + pt] : Pong::serve_entry(st.seed, pt);
    }, w_onep != 0);
    PG_PP(pp_face, ev != kStepFly || st.hits != hits_b || st.point != pt_b);
    const int vis = st.vis;
    const int bx2 = st.bx2, by2 = st.by2;
    // the paddles' centroids: inside the clamp band, the features themselves
    const int rc2 = st.rc2;
    int lc2 = st.lc2;
    if (__builtin_expect(w_onep, 0)) lc2 = PongK::c2_clip(st.lc2);  // the built-in CPU's paddle leaves it
    int left, right;
    // get_actions main.py:143-150; features utils.py:139-153.  The networks run
    // in every lane: a stepped frame with the ball hidden is rare (the miss
    // frame of a point, when the serve delays are advanced at once), so the
    // wave runs the block anyway, and such a lane's decision is [0,0]
    // (main.py:151-153) -- one select instead of a branch and two moves
    {
      const int lbx2 = pvis ? pbx2 : bx2, lby2 = pvis ? pby2 : by2;
      // [bx, by, lbx, lby, me = right, enemy = left] for both halves: the left
      // network's x-flip and me/enemy swap (main.py:146-147) are in its weights
      const int k[6] = {bx2, by2, lbx2, lby2, rc2, lc2};
      float acc[O], z[O];
      partial_pk<U, O, true>(net, k, acc);
#pragma unroll
      for (int o = 0; o < O; ++o) z[o] = group_sum<HL>(acc[o]);
      int code = certify_c8<O>(z, net.ct);  // the decision as its paddle move (index_to_move), or -1
#ifdef PG_PROBE_EXTRA  // timing-only experiment build: extra instructions of one class every visible frame
      pg_probe_extra<PG_PROBE_EXTRA>(net.w1[0][0], net.w1[1][1], z[0], z[1], probe_v, probe_p, probe_s);
#endif
      const bool left_nn = kind == kOppNN;
      if (side && !left_nn) code = 0;  // the left half is idle against a scripted opponent
      if (vis != 1) code = 0;  // the ball hidden ([0,0]) or a parked group
#ifdef PG_ABLATE_SLOW  // timing-only build: never re-decide in f64
      if (code == -1) code = z[1] > z[0] ? 6 : -6;
#endif
      PG_PP(pp_fail, code == -1);
      // rare, half-uniform: the in-wave plateau rule, then the memo, else the
      // f64 stage -- the whole wave (kInline) or the service wave (one
      // wave-uniform test on the common path)
      if (PG_ANY(code == -1)) {
      if (code == -1) {
        fails += 1;
#ifdef PG_TIMELINE
        g_fails += 1;
#endif
        // the gap rule at the plateau's true width (one exp2), else the f32 plateau rule
#ifndef PG_NO_TIGHT
        int mv = tight_gap_move<O>(z, net.e, net.ct);
        if (mv == -1)
#else
        int mv = -1;
#endif
        {
          const int idx = plateau_f32<O>(z, net.e);
          mv = idx >= 0 ? index_to_move(idx) : -1;
        }
        inwave += mv != -1 ? 1 : 0;
        code = mv;
      }
#ifdef PG_ABLATE_SERVE  // timing-only build: the requests serve_inline would take, decided by a compare
      if (code == -1) code = z[1] > z[0] ? 6 : -6;
#endif
      if (kInline && PG_ANY(code == -1)) {
        // the memo, then the whole wave decides each still-undecided half-group in turn
        uint64_t key = 0;
        int nm = 0;
        const int sx = slot_me();
        if (code == -1) {
          key = memo_key(k);
          nm = slots[sx].n_memo;
          int hit = -1;
#pragma unroll 1
          for (int c = 0; c < kMemo && c < nm; ++c)
            if (slots[sx].memo_key[c] == key) hit = slots[sx].memo_idx[c];
          code = hit;
        }
        // the request: the network's own features (x-flipped for the left paddle), its f32 outputs and bound
        const int kn[6] = {side ? 320 - bx2 : bx2, by2, side ? 320 - lbx2 : lbx2, lby2, side ? lc2 : rc2,
                           side ? rc2 : lc2};
        const float my_e = net.e;
        uint64_t need = __builtin_amdgcn_ballot_w64(code == -1 && hl == 0);
        if (need) {
#ifdef PG_DECIDE_PROBE
        const uint64_t probe_d0 = __builtin_amdgcn_s_memtime();
#endif
        if constexpr (PG_INLINE_PRIO > 0) __builtin_amdgcn_s_setprio(PG_INLINE_PRIO);
#pragma unroll 1
        do {
          const int src = (int)__builtin_ctzll(need);
          need &= need - 1;
          InlineReq r;
#pragma unroll
          for (int i = 0; i < 6; ++i) r.k[i] = __builtin_amdgcn_readlane(kn[i], src);
#pragma unroll
          for (int i = 0; i < 6; ++i) r.kr[i] = __builtin_amdgcn_readlane(k[i], src);
          r.rec = p.recs + (long)__builtin_amdgcn_readlane(slots[sx].rec, src) * HL * rec_floats<U, O>();
#pragma unroll
          for (int o = O; o < 4; ++o) r.z[o] = 0.f;
#pragma unroll
          for (int o = 0; o < O; ++o) r.z[o] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(z[o]), src));
          r.e = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_e), src));
          const uint64_t ga = (uint64_t)gm;
          const WT *g = (const WT *)(((uint64_t)__builtin_amdgcn_readlane((int)(ga >> 32), src) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ga, src));
#if defined(PG_SERVE_TWICE)  // diagnostic: the same request served twice, the second call's stages at +12
          serve_inline<U, HL, O, WT>(p, g, r, lds_svc + wave * f64_lds_doubles(H, O), lane64, st_acc);
          const int ans = serve_inline<U, HL, O, WT>(p, g, r, lds_svc + wave * f64_lds_doubles(H, O), lane64, st_acc + 12);
#elif defined(PG_SERVE_STAGES)
          const int ans = serve_inline<U, HL, O, WT>(p, g, r, lds_svc + wave * f64_lds_doubles(H, O), lane64, st_acc);
#else
          const int ans = serve_inline<U, HL, O, WT>(p, g, r, lds_svc + wave * f64_lds_doubles(H, O), lane64);
#endif
          if ((lane64 & ~(HL - 1)) == src) {  // the requesting half-group
            slow += (ans >> 8) & 1;
            plateau += (ans >> 9) & 1;
            inwave += ans >> 10;
            code = index_to_move(ans & 255);
            if (hl == 0) {
              const int c = nm % kMemo;  // round-robin replacement
              slots[sx].memo_key[c] = key;
              slots[sx].memo_idx[c] = code;
              slots[sx].n_memo = nm + 1;
            }
          }
        } while (need);
        if constexpr (PG_INLINE_PRIO > 0) __builtin_amdgcn_s_setprio(0);
        {
          // the output layer back from the lane records: its registers were
          // the f64 code's (the input layer's stay live across it)
#if defined(PG_RELOAD_ALL)  // the whole network reloaded: its registers all the f64 code's while it decides
          load_rec<U, O>(net, p.recs + ((long)slots[sx].rec * HL + hl) * rec_floats<U, O>());
#elif !defined(PG_NO_RELOAD)  // (PG_NO_RELOAD: every weight kept live across the f64 code)
          load_rec_out<U, O>(net, p.recs + ((long)slots[sx].rec * HL + hl) * rec_floats<U, O>());
#endif
#ifndef PG_NO_RELOAD
#pragma unroll
          for (int o = 0; o < O; ++o) net.c[o] = hl == 0 ? 0.5f * net.c[o] : 0.f;
#endif
#ifdef PG_SERVE_STAGES
          {
            const uint64_t r0 = __builtin_amdgcn_s_memtime();
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            st_acc[5] += __builtin_amdgcn_s_memtime() - r0;
            st_acc[11] += 1;
          }
#endif
#ifdef PG_DECIDE_PROBE
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          probe_dec += __builtin_amdgcn_s_memtime() - probe_d0;
#endif
        }
        }
      }
      if (!kInline && PG_ANY(code == -1) && code == -1) {
        const int sx = slot_me();
        const uint64_t key = memo_key(k);
        const int nm = slots[sx].n_memo;
        int hit = -1;
#pragma unroll 1
        for (int c = 0; c < kMemo && c < nm; ++c)
          if (slots[sx].memo_key[c] == key) hit = slots[sx].memo_idx[c];
        if (hit != -1) {
          code = hit;
        } else {
          if (hl == 0) {
            // the network's own features (x-flipped for the left paddle): the f64 path uses the genes
            const int kn[6] = {side ? 320 - bx2 : bx2, by2, side ? 320 - lbx2 : lbx2, lby2, side ? lc2 : rc2,
                               side ? rc2 : lc2};
            slots[sx].g = gm;
#pragma unroll
            for (int i = 0; i < 6; ++i) slots[sx].k[i] = kn[i];
#pragma unroll
            for (int o = 0; o < O; ++o) slots[sx].z[o] = z[o];
            slots[sx].e = net.e;
            __threadfence_block();
            lds_st(&slots[sx].flag, 1);
            __hip_atomic_fetch_add(&posted, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          while (lds_ld(&slots[sx].flag) != 2) __builtin_amdgcn_s_sleep(1);
          __threadfence_block();
          const int ans = slots[sx].idx;
          slow += (ans >> 8) & 1;
#ifdef PG_TIMELINE
          g_slow += 1;  // service round trips
#endif
          plateau += ans >> 9;
          code = index_to_move(ans & 255);
          if (hl == 0) {
            const int c = nm % kMemo;  // round-robin replacement
            slots[sx].memo_key[c] = key;
            slots[sx].memo_idx[c] = code;
            slots[sx].n_memo = nm + 1;
            lds_st(&slots[sx].flag, 0);
          }
        }
      }
      }
      const int mine = code;
      const int other = other_half<L>(mine);
      right = side ? other : mine;
      left = side ? mine : other;
      // HardcodedAi / ScoreHardcodedAi (dumb_ais.py): behind a wave-uniform
      // test, which a self-play schedule never passes
      if (__builtin_expect(w_scripted, 0) && !left_nn) {
        left = vis ? hardcoded_move(by2, lc2) : 0;
        if (kind == kOppScore && st.s1 > st.s2) left = 0;
      }
      if constexpr (!kVisByFrames) c_vis += vis;  // forwards: c_vis x (1 or 2 networks), counted at the game's end
    }
    act_l = clamp_move(lc2, left);
    act_r = clamp_move(rc2, right);
#ifndef PG_TIMELINE
    if (!kUntraced && p.trace) {  // a wave-uniform test first: untraced launches skip the per-lane ones
      const int frames = sframe - fstart;
      if (w < p.trace_games && frames <= p.trace_cap && lig == 0 && (!kInline || live))
        p.trace[(long)w * p.trace_cap + frames - 1] = (uint8_t)(move_code(act_r) | (move_code(act_l) << 2) | (vis << 4));
    }
#endif
    // calculate_timeout_and_frames (main.py:128-135); at most one point a frame
    const bool same = ev != kStepPoint;  // a miss grows exactly one score
#ifndef PG_NO_RALLY_SKIP
    // a periodic rally ends at the timeout with nothing else changed: jump there
    // (never while tracing, which records every frame's actions)
#ifdef PG_TIMELINE
    constexpr bool kTracing = false;  // the timeline build's trace buffer holds stamps, not actions
#else
    const bool kTracing = !kUntraced && p.trace != nullptr;
#endif
    // Brent's cycle search sampled at the frames where a paddle returned the
    // ball (the states at the bounces of a periodic rally repeat too).  The key
    // holds min(hits, 8) and hits grows by one per bounce within a point, so no
    // state of a point repeats before its 8th return: that bounce opens the
    // search (a point or a game start clears the save), a later bounce state
    // equal to the saved one proves the rally periodic, and the save moves
    // forward when the distance reaches the span (kRallySpan0 frames,
    // doubling).  Sampling at bounces instead of every kRallyStride frames:
    // 15 % -> 2 % of wave-frames build a key (profiles/r03/sweep_frame_trims_g5.log);
    // opening at the 8th return instead of at timeout 256, with a 64-frame
    // first span, fires at the cycle's first repetition in the common
    // two-bounce rally (tools/long_games.py: 460 instead of 610 frames).
    const bool rally_check = !kTracing && !kHorizon && ev == kStepRally;  // (step_c<true>: hits >= kRallyHits)
#else
    constexpr bool rally_check = false;
#endif
    PG_PP(pp_rally, rally_check);
    // the no-score counter past TIMEOUT_THRESH (main.py:102-107); the scores end a game only at a point
    bool over = sframe > tend;
    if constexpr (kHorizon) over = over || sframe - fstart >= p.horizon;
    // a point, a rally check or a game end: one wave-uniform test on the common path
    // (a bounce past the kRallyHits-th return enters it even when the rally
    // check is off, tracing: one compare on the common path instead of three)
    if (PG_ANY((kHorizon ? !same : ev >= kStepPoint) || over)) {
    if (!same) {  // a point: total_frames += timeout, timeout = 0 (main.py:128-135); the scores' end test
      total += sframe - 1 - (tend - p.timeout_thresh);
      tend = sframe + p.timeout_thresh;
      // the counter is reset before the termination test (main.py:94-107): a
      // point on the frame the counter would pass TIMEOUT_THRESH ends the game
      // only by the scores (round-5 review: `over` kept the pre-point timeout)
      over = st.s1 >= p.win_score || st.s2 >= p.win_score || st.done();
      if constexpr (kHorizon) over = over || sframe - fstart >= p.horizon;
      if (lig == 0) slots[slot_grp()].rally_at = -1;  // the next rally searches afresh
    }
#ifndef PG_NO_RALLY_SKIP
    const int timeout = sframe - (tend - p.timeout_thresh);
    if (rally_check && timeout <= p.timeout_thresh) {
      const int rs = slot_grp();  // the group's side-0 slot
      const uint64_t key = st.key(move_code(act_r), move_code(act_l));
      const int at = slots[rs].rally_at;
      if (at > timeout || at < 0) {
        if (lig == 0) {
          slots[rs].rally_key = key;
          slots[rs].rally_at = timeout;
          slots[rs].rally_span = kRallySpan0;
        }
      } else if (slots[rs].rally_key == key) {
        const int rest = p.timeout_thresh + 1 - timeout;
        fstart -= rest;  // frames += rest; the counter at TIMEOUT_THRESH + 1
        skipped += rest;
        tend = sframe - 1;
      } else if (timeout - at >= slots[rs].rally_span) {
        if (lig == 0) {
          slots[rs].rally_key = key;
          slots[rs].rally_at = timeout;
          slots[rs].rally_span = 2 * slots[rs].rally_span;
        }
      }
    }
    over = over || sframe > tend;  // a rally jump ends the game
#endif
    if constexpr (kHorizon) {
      if (over) {  // an episode's end or the horizon's
        const int gx = threadIdx.x / L;
        const bool ep_end = st.s1 >= p.win_score || st.s2 >= p.win_score || st.done() || sframe > tend;
        if (lig == 0) {
          if (ep_end) {  // perform_episode's reward (main.py:108-112), summed in episode order
            int zd;
            hz[gx].sum = __dadd_rn(hz[gx].sum, episode_reward(st, total, p.mult[w], zd));
            hz[gx].zd |= zd;
            hz[gx].eps += 1;
          }
          hz[gx].s1 += st.s1;
          hz[gx].s2 += st.s2;
        }
        if (ep_end && sframe - fstart < p.horizon) {  // auto-reset: a fresh episode in the slot, the serves continuing
          const int pt = st.point;
          st.reset(st.seed, st.one_player);
          st.point = pt;
          act_r = act_l = total = 0;
          tend = sframe + 1 + p.timeout_thresh;  // the next iteration is the episode's frame 1
          over = false;
        }
      }
    }
    if (over) {
      if constexpr (kHorizon) {
        if (lig == 0) {
          const int gx = threadIdx.x / L;
          p.rewards[w] = hz[gx].sum;
          p.scores[2 * w] = hz[gx].s1;
          p.scores[2 * w + 1] = hz[gx].s2;
          p.frames[w] = sframe - fstart;
          p.total_frames[w] = (double)hz[gx].eps;
          p.status_game[w] = hz[gx].zd;
        }
      } else {
        if (lig == 0) finish_game(p, w, st, sframe - fstart, total);
      }
#ifdef PG_TIMELINE
      if (p.trace && w < p.trace_games && lig == 0) {
        uint32_t *tl = (uint32_t *)(p.trace + (long)w * p.trace_cap);
        tl[0] = (uint32_t)t_start;
        tl[1] = (uint32_t)wall_clock64();
        tl[2] = g_fails;
        tl[3] = g_slow;
        if (p.trace_cap >= 24) {  // where it ran: block and wave
          tl[4] = blockIdx.x;
          tl[5] = (uint32_t)wave;
        }
      }
#endif
      c_steps += sframe - fstart;
      const int vis_frames = kVisByFrames ? sframe - c_vis - (st.s1 + st.s2) : c_vis;
      c_fwd += (kind == kOppNN ? 2u : 1u) * (uint32_t)vis_frames;
      c_games += 1;
      int ww = 0;
      if (lig == 0) ww = (int)atomicAdd(p.work, 1u);
      w = group_broadcast<L>(ww, leader);
      if constexpr (kInline) {
        if (w >= games_total) {
          live = false;
          park();
        } else {
          fresh = true;
        }
      } else {
        if (w >= games_total) break;
        fresh = true;
      }
    }
    if constexpr (kInline) {
      if (__builtin_amdgcn_ballot_w64(live) == 0) break;
    }
    // what the next frame's top block has to do: a start, or (a point) a serve delay to advance
    top = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(fresh || (kJumps && !st.vis && st.timer >= 2)) != 0);
    }
  }
  if (p.counters && c_games) {
    if (lig == 0) {
      // env steps stepped one at a time: the episodes' frames minus those a
      // periodic rally skipped [8] and the serve delays advanced at once [12]
      atomicAdd((unsigned long long *)&p.counters[0], (unsigned long long)(c_steps - skipped - hidden));
      if (hidden) atomicAdd((unsigned long long *)&p.counters[12], (unsigned long long)hidden);
      atomicAdd((unsigned long long *)&p.counters[1], (unsigned long long)c_fwd);
      atomicAdd((unsigned long long *)&p.counters[3], (unsigned long long)c_games);
      if (skipped) atomicAdd((unsigned long long *)&p.counters[8], (unsigned long long)skipped);
    }
    if (hl == 0 && slow) atomicAdd((unsigned long long *)&p.counters[2], (unsigned long long)slow);
    if (hl == 0 && fails) atomicAdd((unsigned long long *)&p.counters[4], (unsigned long long)fails);
    if (hl == 0 && plateau) atomicAdd((unsigned long long *)&p.counters[5], (unsigned long long)plateau);
    if (hl == 0 && inwave) atomicAdd((unsigned long long *)&p.counters[6], (unsigned long long)inwave);
  }
#ifdef PG_DECIDE_PROBE
  if (p.counters && lane64 == 0) {
    atomicAdd((unsigned long long *)&p.counters[13], (unsigned long long)probe_dec);
    atomicAdd((unsigned long long *)&p.counters[14], (unsigned long long)(__builtin_amdgcn_s_memtime() - probe_t0));
    atomicAdd((unsigned long long *)&p.counters[15], 1ull);
  }
#endif
#ifdef PG_START_PROBE
  if (p.counters && lane64 == 0) {
    atomicAdd((unsigned long long *)&p.counters[13], (unsigned long long)probe_fresh);
    atomicAdd((unsigned long long *)&p.counters[14], (unsigned long long)(__builtin_amdgcn_s_memtime() - probe_t0));
    atomicAdd((unsigned long long *)&p.counters[15], 1ull);
  }
#endif
#ifdef PG_PATH_PROBE
  if (p.counters && lane64 == 0) {
    atomicAdd((unsigned long long *)&p.counters[11], (unsigned long long)pp_frames);
    atomicAdd((unsigned long long *)&p.counters[10], (unsigned long long)pp_rally);
    atomicAdd((unsigned long long *)&p.counters[13], (unsigned long long)pp_face);
    atomicAdd((unsigned long long *)&p.counters[14], (unsigned long long)pp_fail);
    atomicAdd((unsigned long long *)&p.counters[15], (unsigned long long)pp_hidden);
  }
#endif
#ifdef PG_PROBE_EXTRA  // keep the probe's results alive (never true)
  if (p.counters && probe_v == 1234.5f && probe_p.x == 1234.5f && probe_s == 1234567) p.counters[15] = 1;
#endif
#ifdef PG_SERVE_STAGES
  if (p.hard_log && lane64 == 0)
#pragma unroll
    for (int i = 0; i < 24; ++i)
      if (st_acc[i]) atomicAdd((unsigned long long *)&((uint64_t *)p.hard_log)[i], (unsigned long long)st_acc[i]);
#endif
  // this wave will post no more requests
  if (lane64 == 0) atomicAdd(&waves_done, 1);
}

// bytes of lane records a split launch needs (pg_eval_workspace_bytes)
inline size_t service_records_bytes(int n_genomes, int n_opponents, int L, int U, int O) {
  const int F = ((U + 1) / 2 * 2 * (7 + O) + O + 1 + 3) / 4 * 4;  // rec_floats<U, O>()
  return ((size_t)n_genomes + (size_t)(n_opponents > 0 ? n_opponents : 0)) * (size_t)(L / 2) * F * sizeof(float);
}

// kSplitTrace: instantiate the untraced frame too and launch it when p.trace
// is null (the bench layout, pong_ga.hip; the other layouts test p.trace)
template <int L, int U, int O, typename WT, bool kSplitTrace = false>
inline int32_t launch_service(const EvalParams &p, hipStream_t s) {
  constexpr int kSvcThreads = svc_threads<U>();
  // game groups per block, and the f64 scratch: the service wave's, or each wave's
  // (the horizon instance keeps the service wave: inline_service<L, U, true>)
  const bool inl = p.horizon > 0 ? inline_service<L, U, true>() : inline_service<L, U, false>();
  const int GPB = (kSvcThreads / 64 - (inl ? 0 : 1)) * (64 / L);
  const size_t lds = (size_t)f64_lds_doubles(p.nodes[1], O) * sizeof(double) * (inl ? kSvcThreads / 64 : 1);
  const int want = (p.total + GPB - 1) / GPB;
  const int cap = num_cus() * 2;
  const int grid = want < cap ? want : cap;
  if (grid <= 0) return PG_OK;
  if (!p.recs) return fail(PG_ERR_INVALID, "split kernel: no lane-record workspace");
  if (!kSplitTrace && p.horizon > 0)
    return fail(PG_ERR_UNSUPPORTED, "horizon mode: [6, 33..64, 3] networks on 8-lane groups only");
  const long nets = p.prep == PG_PREP_GENOMES ? (long)p.n_genomes
                   : (p.prep == PG_PREP_REST ? (long)p.n_opponents : (long)p.n_genomes + p.n_opponents);
  const long prep_threads = nets * (L / 2);
  // at least one block: it also zeroes the work header and the counters
  const unsigned prep_blocks = (unsigned)((prep_threads + 255) / 256);
  hipLaunchKernelGGL((k_prep_records<L, U, O, WT>), dim3(prep_blocks > 0 ? prep_blocks : 1u), dim3(256), 0, s, p);
  if (p.prep == PG_PREP_GENOMES) {
    PG_HIP(hipGetLastError());
    return PG_OK;
  }
  if (kSplitTrace && p.horizon > 0)  // the fixed-horizon mode: the bench layout's untraced instance
    hipLaunchKernelGGL((k_service<L, U, O, WT, true, true>), dim3(grid), dim3(kSvcThreads), lds, s, p);
  else if (kSplitTrace && !p.trace)
    hipLaunchKernelGGL((k_service<L, U, O, WT, true>), dim3(grid), dim3(kSvcThreads), lds, s, p);
  else
    hipLaunchKernelGGL((k_service<L, U, O, WT, false>), dim3(grid), dim3(kSvcThreads), lds, s, p);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

// layouts L != 8 or U != 16 (pg_service_more.hip); PG_ERR_UNSUPPORTED when none fits
int32_t launch_service_more(const EvalParams &p, int L, int O, bool f64, hipStream_t s);

// the units per lane the split dispatch instantiates for (L, H): launch_service_any
// (pong_ga.hip: L = 8 with H in (32, 64] -> 16) and launch_more (pg_service_more.hip:
// the smallest of 1, 2, 4, 8 with (L / 2) U >= H); 0 when none fits
inline int service_units(int L, int H) {
  if (L == 8 && H > 32 && H <= 64) return 16;
  for (int u = 1; u <= 8; u *= 2)
    if ((L / 2) * u >= H) return u;
  return 0;
}

}  // namespace pg
