// pg_staged.hip -- k_staged<L,U,O,WT>: the evaluation kernel with every frame
// split into an environment stage and a network stage (PG_KERNEL_STAGED).
//
// The same games as k_service (pong_ga.hip), the same arithmetic, a different
// division of labour.  k_service replicates each game's scalar work -- physics
// step, features, bookkeeping, rally detection -- over the L lanes that hold
// the game's two networks, so a wave of 8 games issues the whole per-frame
// physics for only 8 games; those instructions were ~2/3 of its VALU issue.
// Here a block of 8 waves has
//   * one ENVIRONMENT wave: lane s owns game slot s (56 slots at L = 8) and
//     runs, per frame, env.step (main.py:77), the centroid features
//     (utils.py:14-19, 139-153), get_actions' visibility rule (main.py:138-154),
//     the scripted left paddles (dumb_ais.py), keep_within_game_bounds
//     (utils.py:71-77), calculate_timeout_and_frames (main.py:128-135), the
//     periodic-rally jump, termination and calculate_reward (utils.py:104-109)
//     -- one instruction stream for 56 games;
//   * seven NETWORK waves: 8 slots each, L lanes per slot as in k_service
//     (L/2 lanes per paddle's network, U hidden units per lane in VGPRs), which
//     only run the certified f32 forward (numpy_nn.py:120-137, pg_cascade.hpp)
//     on the features the environment wave published.
// One frame: [env: apply last frame's decisions, bookkeeping, next step,
// features -> LDS] s_barrier [net: forwards -> decisions in LDS, done
// counter] -- while the network waves run, the environment wave serves the
// forwards whose f32 certificate failed (plateau rule, certified f64, numpy-
// order f64: the k_service service wave's cascade) and then applies the
// decisions.
//
// Game start without stalls: a network wave must never wait on global memory
// (its vmcnt would hold every slot of the block at the next barrier).  Each
// evaluated row is converted once per launch by k_prep_rows into the lane
// records the network lanes hold (pre-scaled f32 weights + the certificate
// bound, load_net_pk); the environment wave claims games one frame ahead,
// loads their two records with its own (otherwise idle) registers and copies
// them into an LDS staging buffer one frame later, and the slot's network
// lanes pick them up from LDS.  The ball is hidden for the first 30 frames of
// every game, so the pipeline costs no game time.
#include <hip/hip_runtime.h>

#include "../../include/pong_ga.h"
#include "pg_cascade.hpp"
#include "pg_device.hpp"
#include "pg_eval.hpp"

namespace pg {

// native 4-float vector (HIP's float4 is a class with a union, which kept the
// environment wave's load registers on the stack)
typedef float f4v __attribute__((ext_vector_type(4)));

// floats of one lane record (NetP<U,O> flattened), rounded up to whole float4s
template <int U, int O>
__host__ __device__ constexpr int prep_floats() {
  return (2 * NetP<U, O>::P * (7 + O) + O + 1 + 3) & ~3;
}

template <int U, int O>
__device__ __forceinline__ void net_to_floats(const NetP<U, O> &n, float *d) {
  constexpr int P = NetP<U, O>::P;
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      d[(p * 7 + i) * 2] = n.w1[p][i].x;
      d[(p * 7 + i) * 2 + 1] = n.w1[p][i].y;
    }
  float *d2 = d + P * 14;
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int o = 0; o < O; ++o) {
      d2[(p * O + o) * 2] = n.w2[p][o].x;
      d2[(p * O + o) * 2 + 1] = n.w2[p][o].y;
    }
  float *d3 = d2 + P * O * 2;
#pragma unroll
  for (int o = 0; o < O; ++o) d3[o] = n.c[o];
  d3[O] = n.e;
}

// k_prep_rows: lane records of n rows (row t = rows[index ? index[t] : t]),
// HL consecutive records per row -- what load_net_pk leaves in the registers
// of the HL lanes of one network half.  One thread per (row, lane).
template <int HL, int U, int O, typename WT>
__global__ __launch_bounds__(256) void k_prep_rows(const WT *__restrict__ rows, int64_t stride,
                                                   const int32_t *__restrict__ index, int n, int H, int b,
                                                   float *__restrict__ out) {
  constexpr int KR = prep_floats<U, O>();
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long t = gid / HL;
  const int hl = (int)(gid % HL);
  if (t >= n) return;  // whole lane groups (blockDim is a multiple of HL)
  const WT *g = rows + (long)(index ? index[t] : t) * stride;
  NetP<U, O> net;
  load_net_pk<HL, U, O, WT>(net, g, H, b, hl);
  float r[KR];
#pragma unroll
  for (int i = 0; i < KR; ++i) r[i] = 0.f;
  net_to_floats<U, O>(net, r);
  f4v *d = (f4v *)(out + (t * HL + hl) * KR);
#pragma unroll
  for (int i = 0; i < KR / 4; ++i) d[i] = f4v{r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]};
}

// ---- the slot record the environment wave publishes every frame ----------
// lo: bx2 [0,9) by2 [9,18) lbx2 [18,27) vis 27, reload 28, staging buffer
//     [29,31), left-is-network 31
// hi: lby2 [0,9) lc2 [9,18) rc2 [18,27)
// (doubled centroids, each < 320: utils.inference's features x 320)
constexpr uint32_t kRecVis = 1u << 27, kRecReload = 1u << 28, kRecLnn = 1u << 31;
constexpr int kRecStgShift = 29;

// an f32 certificate failure the network wave hands to the environment wave
struct StagedReq {
  int k[6];
  float z[4];
  float e;
  int flag;  // 0 free, 1 posted (accessed with lds_ld / lds_st)
};
struct StagedMemo {  // the network's last kMemo f64 decisions (as k_service's memo)
  uint64_t key[kMemo];
  int idx[kMemo];
  int n;
};

constexpr int kStagedNetWaves = 7;
constexpr int kStagedThreads = 64 * (kStagedNetWaves + 1);
constexpr int kStagedLoads = 4;  // staging buffers: two game starts per frame x frame parity
constexpr int kPend = 0x7f;      // decision code of a posted request

// slot states of the environment wave
enum : int {
  kSlotEmpty = 0,     // needs a game: claims one this frame
  kSlotClaim = 1,     // claim in flight (the work counter's answer is read next frame)
  kSlotAssigned = 2,  // schedule entries (kind, opp, mult) in flight
  kSlotQueued = 3,    // waits for a record load
  kSlotIssued = 4,    // records in flight: staged and started next frame
  kSlotPlaying = 5,
  kSlotDrained = 6    // no more games
};

__device__ __forceinline__ void finish_game_m(const EvalParams &p, int w, const Pong &st, int frames, int total,
                                              double mult) {
  double reward = 0.0;
  int zero_div = 0;
  if (st.s1 != st.s2) {
    const double tf = (double)total;
    if (tf == 0.0) {
      zero_div = 1;
      reward = __builtin_nan("");
    } else {  // ((my - enemy) + my * mult) / (total_frames / 100.0), utils.py:104-109
      const double diff = (double)(st.s2 - st.s1);
      const double bonus = __dmul_rn((double)st.s2, mult);
      reward = __dadd_rn(diff, bonus) / (tf / 100.0);
    }
  }
  p.rewards[w] = reward;
  p.scores[2 * w] = st.s1;
  p.scores[2 * w + 1] = st.s2;
  p.frames[w] = frames;
  p.total_frames[w] = (double)total;
  p.status_game[w] = zero_div;
}

// PG_STAGED_PROFILE (diagnostic builds, tools/staged_probe.py): per-block
// cycle counts of the frame phases into the trace buffer (16 u64 per block)
// instead of action traces.
#ifdef PG_STAGED_PROFILE
#define PG_PT(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define PG_PADD(i, x) prof[i] += (x)
#else
#define PG_PT(v)
#define PG_PADD(i, x)
#endif

template <int L, int U, int O, typename WT>
__global__ __launch_bounds__(kStagedThreads) void k_staged(EvalParams p, const float *__restrict__ prep,
                                                           int n_prep_genomes) {
  constexpr int HL = L / 2;
  constexpr int GPW = 64 / L;                     // slots per network wave
  constexpr int NS = kStagedNetWaves * GPW;       // slots per block (<= 64)
  constexpr int KR = prep_floats<U, O>();         // floats per lane record
  constexpr int NETF = HL * KR;                   // floats per network
  constexpr int STG4 = 2 * NETF / 4;              // float4s per staged game (both networks)
  constexpr int LD4 = (STG4 + 63) / 64;           // float4 loads per env lane per game
  static_assert(NS <= 64, "one environment lane per slot");

  __shared__ uint64_t rec[NS];
  __shared__ int dec[2 * NS];
  __shared__ StagedReq req[2 * NS];
  __shared__ StagedMemo memo[2 * NS];
  __shared__ f4v stg[kStagedLoads][STG4];
  __shared__ int sync_word;  // network waves done (<< 16) + requests posted, this frame
  __shared__ int exit_flag;
  extern __shared__ double lds_svc[];  // f64_lds_doubles(H, O): the numpy-order forward

  const int H = p.nodes[1];
  const int b = p.bias;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 2 * NS; i += kStagedThreads) {
    lds_st(&req[i].flag, 0);
    memo[i].n = 0;
    dec[i] = 0;
  }
  if (threadIdx.x < NS) rec[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    lds_st(&sync_word, 0);
    lds_st(&exit_flag, 0);
  }
#ifdef PG_STAGED_PROFILE
  __shared__ unsigned long long t_done_max;
  if (threadIdx.x == 0) t_done_max = 0;
  uint64_t t_release = 0;
  uint64_t prof[16];
  for (int i = 0; i < 16; ++i) prof[i] = 0;
  PG_PT(t_begin);
#endif
  __syncthreads();

  if (wave < kStagedNetWaves) {
    // =========================== network wave ===============================
    const int grp = lane / L;
    const int lig = lane & (L - 1);
    const int side = lig >= HL ? 1 : 0;  // 0: right paddle's network (the genome), 1: left paddle's
    const int hl = lig & (HL - 1);
    const int slot = wave * GPW + grp;
    const int sl = 2 * slot + side;
    NetP<U, O> net;
#pragma unroll
    for (int p2 = 0; p2 < NetP<U, O>::P; ++p2) {
#pragma unroll
      for (int i = 0; i < 7; ++i) net.w1[p2][i] = float2v{0.f, 0.f};
#pragma unroll
      for (int o = 0; o < O; ++o) net.w2[p2][o] = float2v{0.f, 0.f};
    }
#pragma unroll
    for (int o = 0; o < O; ++o) net.c[o] = 0.f;
    net.e = 0.f;
    uint32_t fails = 0, inwave = 0;
    for (;;) {
      PG_PT(tb0);
      __syncthreads();
      PG_PT(tb1);
      PG_PADD(6, tb1 - tb0);
      if (lds_ld(&exit_flag)) break;
      const uint64_t r = rec[slot];
      const uint32_t lo = (uint32_t)r, hi = (uint32_t)(r >> 32);
      if (lo & kRecReload) {  // a new game: this lane's record from the staging buffer
        const int sb = (lo >> kRecStgShift) & 3;
        const int base4 = (side * NETF + hl * KR) / 4;
        float f[KR];
#pragma unroll
        for (int i = 0; i < KR / 4; ++i) {
          const f4v v = stg[sb][base4 + i];
          f[4 * i] = v.x;
          f[4 * i + 1] = v.y;
          f[4 * i + 2] = v.z;
          f[4 * i + 3] = v.w;
        }
        constexpr int P = NetP<U, O>::P;
#pragma unroll
        for (int p2 = 0; p2 < P; ++p2)
#pragma unroll
          for (int i = 0; i < 7; ++i) net.w1[p2][i] = float2v{f[(p2 * 7 + i) * 2], f[(p2 * 7 + i) * 2 + 1]};
#pragma unroll
        for (int p2 = 0; p2 < P; ++p2)
#pragma unroll
          for (int o = 0; o < O; ++o)
            net.w2[p2][o] = float2v{f[P * 14 + (p2 * O + o) * 2], f[P * 14 + (p2 * O + o) * 2 + 1]};
#pragma unroll
        for (int o = 0; o < O; ++o) net.c[o] = f[P * (14 + 2 * O) + o];
        net.e = f[P * (14 + 2 * O) + O];
      }
      if (lo & kRecVis) {  // get_actions: a forward only while the ball is visible (main.py:143-153)
        const int bx2 = lo & 511, by2 = (lo >> 9) & 511, lbx2 = (lo >> 18) & 511;
        const int lby2 = hi & 511, lc2 = (hi >> 9) & 511, rc2 = (hi >> 18) & 511;
        // right: [bx, by, lbx, lby, me = right, enemy = left]; left x-flipped (main.py:146-147)
        const int k[6] = {side ? 320 - bx2 : bx2, by2, side ? 320 - lbx2 : lbx2, lby2, side ? lc2 : rc2,
                          side ? rc2 : lc2};
        float acc[O], z[O];
        partial_pk<U, O>(net, k, acc);
#pragma unroll
        for (int o = 0; o < O; ++o) z[o] = group_sum<HL>(acc[o]) + net.c[o];
        int idx = certify<O>(z, net.e);
        if (side && !(lo & kRecLnn)) idx = 0;  // the left half is idle against a scripted opponent
        if (idx < 0) {
          fails += 1;
          idx = plateau_f32<O>(z, net.e);
          inwave += idx >= 0 ? 1 : 0;
        }
        if (hl == 0) {
          if (idx < 0) {  // hand it to the environment wave; the decision is written there
#pragma unroll
            for (int i = 0; i < 6; ++i) req[sl].k[i] = k[i];
#pragma unroll
            for (int o = 0; o < O; ++o) req[sl].z[o] = z[o];
            req[sl].e = net.e;
            dec[sl] = kPend;
            __threadfence_block();
            lds_st(&req[sl].flag, 1);
            __hip_atomic_fetch_add(&sync_word, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else {
            dec[sl] = index_to_code(idx);
          }
        }
      }
      __threadfence_block();
      PG_PT(tb2);
      PG_PADD(5, tb2 - tb1);
#ifdef PG_STAGED_PROFILE
      if (lane == 0) atomicMax(&t_done_max, (unsigned long long)tb2);
#endif
      if (lane == 0) __hip_atomic_fetch_add(&sync_word, 1 << 16, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
#ifdef PG_STAGED_PROFILE
    if (lane == 0 && p.trace) {
      uint64_t *d = (uint64_t *)(p.trace + (long)blockIdx.x * p.trace_cap);
      if (wave == 0) {
        d[5] = prof[5];
        d[6] = prof[6];
      }
      d[16 + wave] = prof[5];  // every network wave's compute cycles
    }
#endif
    if (p.counters) {
      if (hl == 0 && fails) atomicAdd((unsigned long long *)&p.counters[4], (unsigned long long)fails);
      if (hl == 0 && inwave) atomicAdd((unsigned long long *)&p.counters[6], (unsigned long long)inwave);
    }
    return;
  }

  // ============================= environment wave =============================
  // A game's start is pipelined over frames, all in the part of the frame that
  // overlaps the network stage: claim (work counter) -> its schedule entries
  // load -> its two records load -> staged into LDS, game starts.  Each global
  // load lands in registers that are first read a frame later, behind one
  // explicit vmcnt(0) at the top of the frame.
  const WT *genomes = (const WT *)p.genomes;
  const WT *opponents = (const WT *)p.opponents;
  const int games_total = active_total(p);
#ifdef PG_STAGED_PROFILE
  const bool tracing = false;  // the trace buffer holds the profile
#else
  const bool tracing = p.trace != nullptr;
#endif
  int state = lane < NS ? kSlotEmpty : kSlotDrained;
  int w = 0, kind = 0, orow = 0, grow = 0, claim_rank = 0;
  double mult = 0.0;
  int n_kind = 0, n_orow = 0, n_grow = 0;  // schedule entries in flight (kSlotAssigned)
  double n_mult = 0.0;
  Pong st;
  st.reset(0, 0);
  int act_r = 0, act_l = 0, timeout = 0, total = 0, frames = 0, vis = 0, by2 = 0, lc2 = 0, rc2 = 0;
  int s1b = 0, s2b = 0;
  uint64_t rkey = 0;
  int rat = 0, rspan = 0;
  uint32_t c_steps = 0, c_fwd = 0, c_games = 0, skipped = 0;
  uint32_t slow = 0, certified = 0;  // wave-uniform: service decisions (numpy-order / certified f64)
  uint32_t claim_base = 0;           // lane 0: the work-counter claim in flight
  int claim_n = 0;                   // games claimed last frame (wave-uniform)
  // records in flight for two slots (-1: none), in named registers (an
  // array indexed [q][j] was left in scratch)
  int ld_slot0 = -1, ld_slot1 = -1;
  f4v ld0[LD4], ld1[LD4];
  static_assert(kStagedLoads == 4, "two loads per frame, double-buffered by frame parity");
  const long rec_row = (long)HL * KR;  // floats per network in the prepared rows
  const long opp_base = (long)n_prep_genomes * rec_row;
  int parity = 0;
  bool first = true;

  for (;;) {
    // Every global load and store of last frame is complete here, while the
    // network waves compute; the registers they fill are first read below.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    PG_PT(te0);

    // ---- (T) last step's decision-independent bookkeeping (main.py:94-107,
    // 128-135): the no-score counter and termination need the scores after
    // the step, not this frame's decisions, so they run before the wait; a
    // game that ended frees its slot for this frame's claim
    bool fin_now = false;
    const int w_traced = w;
    if (state == kSlotPlaying) {
      if (frames > 1) {  // calculate_timeout_and_frames main.py:128-135
        if (st.s1 == s1b && st.s2 == s2b) {
          timeout += 1;
        } else {
          total += timeout;
          timeout = 0;
        }
      }
      if (st.s1 >= kWinScore || st.s2 >= kWinScore || st.done() || timeout > kTimeoutThresh) {
        finish_game_m(p, w, st, frames, total, mult);
        c_steps += frames;
        c_games += 1;
        state = kSlotEmpty;
        fin_now = true;
      }
    }

    // ---- (a) records loaded last frame -> this frame's staging buffers; those games start now
    uint32_t reload = 0;
    bool start = false;
#define PG_STAGE(Q, LQ, SLOT)                                                    \
    if (SLOT >= 0) {                                                             \
      _Pragma("unroll") for (int j = 0; j < LD4; ++j) {                          \
        const int i4 = lane + 64 * j;                                            \
        if (i4 < STG4) stg[2 * parity + Q][i4] = LQ[j];                          \
      }                                                                          \
      if (lane == SLOT) {                                                        \
        reload = kRecReload | ((uint32_t)(2 * parity + Q) << kRecStgShift);      \
        start = true;                                                            \
      }                                                                          \
      SLOT = -1;                                                                 \
    }
    PG_STAGE(0, ld0, ld_slot0) PG_STAGE(1, ld1, ld_slot1)
#undef PG_STAGE
    // ---- (b) schedule entries loaded last frame
    if (state == kSlotAssigned) {
      kind = n_kind;
      orow = n_orow;
      grow = n_grow;
      mult = n_mult;
      state = kSlotQueued;
    }
    // ---- (c) last frame's work claim: game indices, their schedule entries
    if (claim_n > 0) {
      const uint32_t base = __builtin_amdgcn_readfirstlane(claim_base);
      if (state == kSlotClaim) {
        const int ww = (int)(base + (uint32_t)claim_rank);
        if (ww < games_total) {
          w = ww;
          n_kind = p.kind[w];
          n_orow = p.opp[w];
          n_mult = p.mult[w];
          n_grow = genome_row(p, w / p.n_games);
          state = kSlotAssigned;
        } else {
          state = kSlotDrained;
        }
      }
      claim_n = 0;
    }
    // ---- (d) the records of up to two queued games (staged next frame)
    {
      unsigned long long qm = __ballot(state == kSlotQueued);
#define PG_LOAD(LQ, SLOT)                                                                           \
      if (qm) {                                                                                     \
        const int s = __builtin_ctzll(qm);                                                          \
        qm &= qm - 1;                                                                               \
        const int gi = __builtin_amdgcn_readlane(w, s) / p.n_games; /* genome record = game block */ \
        const int ks = __builtin_amdgcn_readlane(kind, s);                                          \
        const int os = __builtin_amdgcn_readlane(orow, s);                                          \
        const f4v *src0 = (const f4v *)(prep + (long)gi * rec_row);                                 \
        const f4v *src1 = ks == kOppNN ? (const f4v *)(prep + opp_base + (long)os * rec_row) : src0; \
        _Pragma("unroll") for (int j = 0; j < LD4; ++j) {                                           \
          const int i4 = lane + 64 * j;                                                             \
          const f4v *src = i4 < NETF / 4 ? src0 + i4 : src1 + (i4 - NETF / 4);                      \
          if (i4 < STG4) LQ[j] = *src;                                                              \
        }                                                                                           \
        SLOT = s;                                                                                   \
        if (lane == s) state = kSlotIssued;                                                         \
      }
      PG_LOAD(ld0, ld_slot0) PG_LOAD(ld1, ld_slot1)
#undef PG_LOAD
    }
    // ---- (e) claim games for the slots that emptied last frame (read next frame)
    {
      const unsigned long long em = __ballot(state == kSlotEmpty);
      if (em) {
        const int n = __popcll(em);
        if (lane == 0) claim_base = atomicAdd(p.work, (unsigned)n);
        claim_rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
        if (state == kSlotEmpty) state = kSlotClaim;
        claim_n = n;
      }
    }

    if (!first) {
      // ---- wait for the network stage, serving certificate failures meanwhile
      PG_PT(tw0);
      // one LDS word per poll: requests posted (low half) and network waves done
      // (high half); a request's flag is set before its count, so a scan after
      // seeing the count finds it
      int n_served = 0;
      for (;;) {
        const int sw = lds_ld(&sync_word);
        if ((sw & 0xFFFF) == n_served) {
          if ((sw >> 16) == kStagedNetWaves) break;
          continue;  // spin: the network stage is short and this wave has nothing else to do
        }
        for (int base = 0; base < 2 * NS; base += 64) {
          const int i = base + lane;
          const bool posted = i < 2 * NS && lds_ld(&req[i].flag) == 1;
          unsigned long long mask = __ballot(posted);
          while (mask) {
            const int rs = base + __builtin_ctzll(mask);
            mask &= mask - 1;
            __threadfence_block();
            n_served += 1;
            PG_PT(ts0);
            int k[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) k[q] = req[rs].k[q];
            const uint64_t key = memo_key(k);
            const int nm = memo[rs].n;
            int hit = -1;
            if (lane < kMemo && lane < nm && memo[rs].key[lane] == key) hit = memo[rs].idx[lane];
            const unsigned long long hm = __ballot(hit >= 0);
            int idx;
            if (hm) {
              idx = __builtin_amdgcn_readlane(hit, __builtin_ctzll(hm));
            } else {
              const int s = rs >> 1;
              const int rside = rs & 1;
              const int gr_s = __builtin_amdgcn_readlane(grow, s);
              const int or_s = __builtin_amdgcn_readlane(orow, s);
              const WT *g = rside ? opponents + (long)or_s * p.ostride : genomes + (long)gr_s * p.gstride;
              float zf[O];
#pragma unroll
              for (int o = 0; o < O; ++o) zf[o] = req[rs].z[o];
              idx = plateau_decide<O>(zf, req[rs].e, lane);
              if (idx < 0) idx = fast_f64_decide<O, WT>(g, H, b, k, lane);
              if (idx >= 0) {
                certified += 1;
              } else {
                idx = forward_f64_group<64, (U * HL + 63) / 64, O, WT>(g, H, b, k, lds_svc, lane);
                slow += 1;
                if (p.hard_log && lane == 0) log_hard(p, rside ? or_s : gr_s, rside, idx, 0, k);
              }
              if (lane == 0) {
                const int c = nm % kMemo;  // round-robin replacement
                memo[rs].key[c] = key;
                memo[rs].idx[c] = idx;
                memo[rs].n = nm + 1;
              }
            }
            if (lane == 0) {
              dec[rs] = index_to_code(idx);
              __threadfence_block();
              lds_st(&req[rs].flag, 0);
            }
            PG_PT(ts1);
            PG_PADD(2, ts1 - ts0);
            PG_PADD(10, 1);
          }
        }
      }
      __threadfence_block();
      PG_PT(te1);
      PG_PADD(1, te1 - tw0);
      PG_PADD(11, tw0 - te0);
#ifdef PG_STAGED_PROFILE
      {
        const uint64_t tdm = t_done_max;
        PG_PADD(12, te1 - tdm);         // done seen after the last network wave finished
        PG_PADD(13, tdm - t_release);   // network stage span from the barrier release
      }
#endif

      // ---- apply the decisions: get_actions, bounds, the rally jump (the
      // decision-independent bookkeeping of this frame ran before the wait)
      if (state == kSlotPlaying || fin_now) {
        int left = 0, right = 0;
        if (vis) {
          const bool lnn = kind == kOppNN;
          right = dec[2 * lane];
          int scripted = hardcoded(by2, lc2);
          if (kind == kOppScore && st.s1 > st.s2) scripted = 0;
          left = lnn ? dec[2 * lane + 1] : scripted;
          c_fwd += lnn ? 2 : 1;
        }
        act_l = clamp_action(lc2, left);
        act_r = clamp_action(rc2, right);
        if (tracing && w_traced < p.trace_games && frames <= p.trace_cap)
          p.trace[(long)w_traced * p.trace_cap + frames - 1] = (uint8_t)(act_r | (act_l << 2) | (vis << 4));
#ifndef PG_NO_RALLY_SKIP
        // a periodic rally ends at the timeout with nothing else changed: jump there
        if (state == kSlotPlaying && timeout >= kRallyStart && timeout <= kTimeoutThresh &&
            (timeout & (kRallyStride - 1)) == 0 && !tracing) {
          const uint64_t key = rally_key(st, act_r, act_l);
          if (timeout == kRallyStart) {
            rkey = key;
            rat = timeout;
            rspan = kRallyStart;
          } else if (rkey == key) {
            const int rest = kTimeoutThresh + 1 - timeout;
            frames += rest;
            skipped += rest;
            timeout = kTimeoutThresh + 1;
            finish_game_m(p, w, st, frames, total, mult);  // main.py:105: ends at the timeout
            c_steps += frames;
            c_games += 1;
            state = kSlotEmpty;
          } else if (timeout - rat == rspan) {
            rkey = key;
            rat = timeout;
            rspan = 2 * rspan;
          }
        }
#endif
      }
    }
    first = false;

    // ---- env.step with last frame's actions, features for the network stage
    if (start) {  // a game whose records were staged this frame
      state = kSlotPlaying;
      st.reset(game_seed(p.seed, w % p.n_games), kind == kOppRomCpu);
      act_r = act_l = timeout = total = frames = 0;
      memo[2 * lane].n = 0;
      memo[2 * lane + 1].n = 0;
    }
    uint64_t r = 0;
    if (state == kSlotPlaying) {
      s1b = st.s1;
      s2b = st.s2;
      const int pvis = st.vis, pbx2 = 2 * st.bx + kBallW - 1, pby2 = 2 * st.by + kBallH - 1;
      st.step(act_r, act_l);
      frames += 1;
      vis = st.vis;
      const int bx2 = 2 * st.bx + kBallW - 1;
      by2 = 2 * st.by + kBallH - 1;
      lc2 = paddle_c2(st.lpy);
      rc2 = paddle_c2(st.rpy);
      const int lbx2 = pvis ? pbx2 : bx2, lby2 = pvis ? pby2 : by2;
      const uint32_t lo = (uint32_t)bx2 | ((uint32_t)by2 << 9) | ((uint32_t)lbx2 << 18) | (vis ? kRecVis : 0u) |
                          reload | (kind == kOppNN ? kRecLnn : 0u);
      const uint32_t hi = (uint32_t)lby2 | ((uint32_t)lc2 << 9) | ((uint32_t)rc2 << 18);
      r = (uint64_t)lo | ((uint64_t)hi << 32);
    }
    if (lane < NS) rec[lane] = r;
    const bool alive = __ballot(state != kSlotDrained) != 0;
    lds_st(&sync_word, 0);
    if (!alive) lds_st(&exit_flag, 1);
    parity ^= 1;
#ifdef PG_STAGED_PROFILE
    PG_PT(te2);
    PG_PADD(0, 1);
    PG_PADD(8, __popcll(__ballot(state == kSlotPlaying)));
    PG_PADD(9, __popcll(__ballot(state == kSlotPlaying && vis)));
#endif
#ifdef PG_STAGED_PROFILE
    if (lane == 0) t_done_max = 0;
#endif
    __syncthreads();
#ifdef PG_STAGED_PROFILE
    PG_PT(te3);
    PG_PADD(3, te2 - te0);
    PG_PADD(4, te3 - te2);
    t_release = te3;
#endif
    if (!alive) break;
  }
#ifdef PG_STAGED_PROFILE
  if (lane == 0 && p.trace) {
    PG_PT(t_end);
    uint64_t *d = (uint64_t *)(p.trace + (long)blockIdx.x * p.trace_cap);
    d[0] = prof[0]; d[1] = prof[1]; d[2] = prof[2]; d[3] = prof[3]; d[4] = prof[4];
    d[7] = t_end - t_begin; d[8] = prof[8]; d[9] = prof[9]; d[10] = prof[10]; d[11] = prof[11];
    d[12] = prof[12]; d[13] = prof[13];
  }
#endif
  if (p.counters) {
    if (lane < NS && c_games) {
      atomicAdd((unsigned long long *)&p.counters[0], (unsigned long long)(c_steps - skipped));
      atomicAdd((unsigned long long *)&p.counters[1], (unsigned long long)c_fwd);
      atomicAdd((unsigned long long *)&p.counters[3], (unsigned long long)c_games);
      if (skipped) atomicAdd((unsigned long long *)&p.counters[8], (unsigned long long)skipped);
    }
    if (lane == 0 && slow) atomicAdd((unsigned long long *)&p.counters[2], (unsigned long long)slow);
    if (lane == 0 && certified) atomicAdd((unsigned long long *)&p.counters[5], (unsigned long long)certified);
  }
}

// ------------------------------------------------------------------ host ----
// lanes per game / units per lane for hidden width H
struct StagedChoice {
  int L, U;
};
static StagedChoice choose_staged(int H) {
  static const StagedChoice table[] = {{8, 1}, {8, 2}, {8, 4}, {8, 8}, {8, 16}, {16, 16}, {32, 16}};
  for (const auto &c : table)
    if ((c.L / 2) * c.U >= H) return c;
  return {0, 0};
}

bool staged_shape_ok(const pg_net &n) {
  return n.n_nodes == 3 && n.nodes[0] == 6 && n.nodes[1] >= 1 && n.nodes[1] <= 256 && n.nodes[2] >= 2 &&
         n.nodes[2] <= 4;
}

template <int U, int O>
static size_t staged_prep_floats_per_row(int L) {
  return (size_t)(L / 2) * prep_floats<U, O>();
}

// rows k_prep_rows prepares: the evaluated genome blocks, then the opponents
// (the genomes themselves when the call has no opponents)
static void staged_prep_rows(const pg_eval_args *a, long &n_gen, long &n_opp) {
  n_gen = a->n_genomes > 0 ? a->n_genomes : 0;
  n_opp = (a->opponents && a->n_opponents > 0) ? a->n_opponents : n_gen;
}

size_t staged_workspace_bytes(const pg_eval_args *a) {
  if (!staged_shape_ok(a->net)) return 0;
  const StagedChoice c = choose_staged(a->net.nodes[1]);
  if (c.L == 0) return 0;
  const int O = a->net.nodes[2];
  const int P = (c.U + 1) / 2;
  const size_t kr = (size_t)((2 * P * (7 + O) + O + 1 + 3) & ~3);
  long ng, no;
  staged_prep_rows(a, ng, no);
  return (size_t)(ng + no) * (size_t)(c.L / 2) * kr * sizeof(float);
}

template <int L, int U, int O, typename WT>
static int32_t launch_staged_t(const EvalParams &p, const pg_eval_args *a, void *prep_ws, hipStream_t s) {
  constexpr int HL = L / 2;
  constexpr int KR = prep_floats<U, O>();
  constexpr int NS = kStagedNetWaves * (64 / L);
  float *prep = (float *)prep_ws;
  long ng, no;
  staged_prep_rows(a, ng, no);
  const int H = p.nodes[1];
  if (ng > 0) {
    const long thr = ng * HL;
    hipLaunchKernelGGL((k_prep_rows<HL, U, O, WT>), dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s,
                       (const WT *)p.genomes, p.gstride, p.rows, (int)ng, H, p.bias, prep);
    PG_HIP(hipGetLastError());
  }
  if (no > 0) {
    const bool own = a->opponents && a->n_opponents > 0;
    const long thr = no * HL;
    hipLaunchKernelGGL((k_prep_rows<HL, U, O, WT>), dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s,
                       (const WT *)(own ? p.opponents : p.genomes), own ? p.ostride : p.gstride,
                       (const int32_t *)nullptr, (int)no, H, p.bias, prep + ng * HL * KR);
    PG_HIP(hipGetLastError());
  }
  const size_t lds = (size_t)f64_lds_doubles(H, O) * sizeof(double);
  const long want = ((long)p.total + NS - 1) / NS;
  const long cap = num_cus();
  const int grid = (int)(want < cap ? want : cap);
  if (grid <= 0) return PG_OK;
  hipLaunchKernelGGL((k_staged<L, U, O, WT>), dim3(grid), dim3(kStagedThreads), lds, s, p, (const float *)prep,
                     (int)ng);
  PG_HIP(hipGetLastError());
  return PG_OK;
}

template <typename WT>
static int32_t launch_staged_wt(const EvalParams &p, const pg_eval_args *a, void *prep, hipStream_t s) {
  const StagedChoice c = choose_staged(p.nodes[1]);
  const int O = p.nodes[2];
#define PG_STG(LL, UU)                                                        \
  if (c.L == LL && c.U == UU) {                                               \
    if (O == 2) return launch_staged_t<LL, UU, 2, WT>(p, a, prep, s);         \
    if (O == 3) return launch_staged_t<LL, UU, 3, WT>(p, a, prep, s);         \
    if (O == 4) return launch_staged_t<LL, UU, 4, WT>(p, a, prep, s);         \
  }
#ifdef PG_STAGED_ONLY_BENCH  // development builds: the bench instance only
  PG_STG(8, 16)
#else
  PG_STG(8, 1) PG_STG(8, 2) PG_STG(8, 4) PG_STG(8, 8) PG_STG(8, 16) PG_STG(16, 16) PG_STG(32, 16)
#endif
#undef PG_STG
  return fail(PG_ERR_UNSUPPORTED, "no staged kernel for H=%d O=%d", p.nodes[1], O);
}

int32_t launch_staged(const EvalParams &p, const pg_eval_args *a, void *prep, hipStream_t s) {
  return a->net.dtype == PG_F64 ? launch_staged_wt<double>(p, a, prep, s) : launch_staged_wt<float>(p, a, prep, s);
}

}  // namespace pg
