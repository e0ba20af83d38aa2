// pg_decide.hip -- k_decide: k_service's decision cascade on given inputs
// (pg_decide, include/pong_ga.h), in its own translation unit so that it is
// compiled on the default machine scheduler (pong_ga.hip's iterative-ILP
// scheduler, which k_service is tuned for, crashes ROCm 7.2's register
// allocator on k_decide).
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/pong_ga.h"
#include "pg_cascade.hpp"
#include "pg_device.hpp"
#include "pg_eval.hpp"
#include "pg_f64math.h"
#include "pg_service.hpp"

namespace pg {

// --------------------------------------------------------------- decide ----
// k_service's decision cascade on given inputs (pg_decide): the split layout's
// f32 pass (load_net_pk / partial_pk / group_sum<HL>, the same z and bound e a
// game half-group computes), certify, the in-wave plateau rule, then the
// service wave's plateau_decide, the frame's own bound where k_service uses it
// (serve_inline's layout: frame_bound_wave over the passes' lane records, kept
// in LDS here), fast_f64_decide and numpy-order forward -- the same device
// functions, so a fixture of hard inputs pins the decisions k_service makes on
// them.  One wave: 64 / HL passes' f32 parts in parallel, then each failing
// pass through the wave-wide service cascade.


template <int HL, int U, int O, typename WT>
__global__ __launch_bounds__(64) void k_decide(DecideParams p) {
  constexpr int GPW = 64 / HL;
  constexpr bool kFrameBound = inline_service<2 * HL, U, false>() && PG_INLINE_FRAME_BOUND;
  constexpr int F = rec_floats<U, O>();
  __shared__ float recs_dec[kFrameBound ? 64 * F : 1];  // lane t's record at t * F
  extern __shared__ double lds_dec[];  // f64_lds_doubles(H, O)
  __shared__ float zs[GPW][4];
  __shared__ float es[GPW];
  __shared__ int res[GPW], stg[GPW];
  const int lane = threadIdx.x, grp = lane / HL, hl = lane % HL;
  const WT *genomes = (const WT *)p.genomes;
  for (int base = blockIdx.x * GPW; base < p.n; base += gridDim.x * GPW) {
    const int t = base + grp;
    if (t < p.n) {
      const WT *g = genomes + (long)(p.gidx ? p.gidx[t] : t) * p.gstride;
      NetP<U, O> net;
      load_net_pk<HL, U, O, WT>(net, g, p.H, p.b, hl);
      if constexpr (kFrameBound) store_rec<U, O>(net, recs_dec + lane * F);
      int k[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) k[i] = p.k[(long)t * 6 + i];
      // k_service's order: the output bias enters the first lane's two partial
      // chains, half each (exact), no add after the group sum -- the same f32 z
      // bit for bit (round-5 review: this pass had kept the bias after the sum)
#pragma unroll
      for (int o = 0; o < O; ++o) net.c[o] = hl == 0 ? 0.5f * net.c[o] : 0.f;
      float acc[O], z[O];
      partial_pk<U, O, true>(net, k, acc);
#pragma unroll
      for (int o = 0; o < O; ++o) z[o] = group_sum<HL>(acc[o]);
      int idx = certify<O>(z, net.e), st = 0;
      if (idx < 0) {
        idx = plateau_f32<O>(z, net.e);
        st = 1;
      }
      if (hl == 0) {
#pragma unroll
        for (int o = 0; o < O; ++o) zs[grp][o] = z[o];
        es[grp] = net.e;
        res[grp] = idx;
        stg[grp] = st;
      }
    }
    wave_lds_sync();
    for (int q = 0; q < GPW; ++q) {
      const int t2 = base + q;
      if (t2 >= p.n || res[q] >= 0) continue;  // wave-uniform
      const WT *g = genomes + (long)(p.gidx ? p.gidx[t2] : t2) * p.gstride;
      int k[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) k[i] = p.k[(long)t2 * 6 + i];
      float zf[O];
#pragma unroll
      for (int o = 0; o < O; ++o) zf[o] = zs[q][o];
      // serve_inline's order: with the frame bound, no plateau rule under the static one first
      int idx = kFrameBound ? -1 : plateau_decide<O>(zf, es[q], lane);
      int st = 2;
      if constexpr (kFrameBound) {
        if (idx < 0 && es[q] < __builtin_inff()) {  // serve_inline's order
          const float ef = fminf(es[q], frame_bound_wave<HL, U, O>(recs_dec + q * HL * F, k, lane));
          idx = certify_c<O>(zf, make_cert(ef));
          if (idx < 0) idx = plateau_f32<O>(zf, ef);
          if (idx < 0) idx = plateau_decide<O>(zf, ef, lane);
          st = idx >= 0 ? 4 : 2;
        }
      }
      if (idx < 0) idx = fast_f64_decide<O, WT>(g, p.H, p.b, k, lane);
      if (idx < 0) {
        idx = forward_f64_group<64, 1, O, WT>(g, p.H, p.b, (const int *)k, lds_dec, lane);
        st = 3;
      }
      wave_lds_sync();
      if (lane == 0) {
        res[q] = idx;
        stg[q] = st;
      }
      wave_lds_sync();
    }
    if (hl == 0 && t < p.n) {
      p.index[t] = res[grp];
      if (p.stage) p.stage[t] = stg[grp];
    }
    wave_lds_sync();
  }
}

int32_t launch_decide(const DecideParams &p, int L, int O, bool f64, size_t lds, hipStream_t s) {
  const int cap = num_cus() * 8;
  const int H = p.H;
#define PG_DEC(LL, UU)                                                                              \
  if (L == LL && (LL / 2) * UU >= H) {                                                              \
    constexpr int GPW = 64 / (LL / 2);                                                              \
    const int want = (p.n + GPW - 1) / GPW;                                                         \
    const int grid = want < cap ? want : cap;                                                       \
    if (O == 2) {                                                                                   \
      if (f64) hipLaunchKernelGGL((k_decide<LL / 2, UU, 2, double>), dim3(grid), dim3(64), lds, s, p); \
      else hipLaunchKernelGGL((k_decide<LL / 2, UU, 2, float>), dim3(grid), dim3(64), lds, s, p);      \
    } else if (O == 3) {                                                                            \
      if (f64) hipLaunchKernelGGL((k_decide<LL / 2, UU, 3, double>), dim3(grid), dim3(64), lds, s, p); \
      else hipLaunchKernelGGL((k_decide<LL / 2, UU, 3, float>), dim3(grid), dim3(64), lds, s, p);      \
    } else {                                                                                        \
      if (f64) hipLaunchKernelGGL((k_decide<LL / 2, UU, 4, double>), dim3(grid), dim3(64), lds, s, p); \
      else hipLaunchKernelGGL((k_decide<LL / 2, UU, 4, float>), dim3(grid), dim3(64), lds, s, p);      \
    }                                                                                               \
    PG_HIP(hipGetLastError());                                                                      \
    return PG_OK;                                                                                   \
  }
  // the layouts launch_service_any picks for choose_split_lanes(H)
#ifndef PG_DEV_MIN
  PG_DEC(8, 1) PG_DEC(8, 2) PG_DEC(8, 4) PG_DEC(8, 8) PG_DEC(8, 16) PG_DEC(32, 8) PG_DEC(64, 8)
#endif
#undef PG_DEC
  return fail(PG_ERR_UNSUPPORTED, "pg_decide: no layout for H=%d", H);
}

}  // namespace pg
