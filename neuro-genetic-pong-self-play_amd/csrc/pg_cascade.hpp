// pg_cascade.hpp -- the certified f32 forward of the game networks and its
// decision cascade, shared by k_service (pg_service.hpp), the batched forward
// k_forward_resident (pg_forward) and pg_decide:
//   load_net / load_net_pk   a lane's share of a [6, H, O] network in VGPRs
//                            (numpy_nn.py:52-69 gene layout) + the f32 bound
//   partial_f32 / partial_pk the hidden layer and lane-partial output sums
//   certify                  argmax of numpy's f64 S(z) proven from f32 z +- e
//   plateau_f32              the same near saturation, in-wave
//   plateau_decide / frame_bound_wave / fast_f64_decide / forward_f64_group
//                            the f64 stage and its f32 frame bound (numpy_nn.py:120-137)
// DESIGN.md 4.1 "Certified argmax, as a cascade".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pg_device.hpp"
#include "pg_eval.hpp"
#include "pg_f64math.h"

namespace pg {

// ======================================= one network per lane group (pg_forward) ==
#ifndef PG_SLOW_INLINE
#define PG_SLOW_INLINE __forceinline__
#endif
// hidden units whose weight loads are in flight together in load_net
#ifndef PG_LOAD_BATCH
#define PG_LOAD_BATCH 2
#endif
// minimum waves per SIMD requested from the register allocator (0 = no request)
#ifndef PG_RES_WAVES
#define PG_RES_WAVES 0
#endif
#if PG_RES_WAVES > 0
#define PG_RES_BOUNDS __launch_bounds__(256, PG_RES_WAVES)
#else
#define PG_RES_BOUNDS __launch_bounds__(256)
#endif
constexpr float kU = 5.9604644775390625e-8f;  // 2^-24, f32 unit roundoff

template <int U, int O>
struct Net {
  float w1[U][7];  // hidden unit j = lane + L*u: 6 input weights + bias weight
  float w2[U][O];  // output weights of that hidden unit
  float c[O];      // output biases
  float e;         // certified bound on |z_o(f32) - z_o(exact)|, max over outputs
};

// A network whose f32 weights could overflow an f32 sum (or are NaN / inf)
// gets the bound e = inf: certify() then never decides and the f64 path
// (numpy's semantics, NaN rule included) does.  With each lane's sum of
// |weights| <= kWeightCap (a sum, so NaN and inf propagate) no f32
// pre-activation or output can overflow or become NaN, so the per-frame
// certificate needs no NaN test.
constexpr float kWeightCap = 1e30f;
__device__ __forceinline__ bool weights_ok(float big) { return big <= kWeightCap; }  // false for NaN

// Loads the [6, H, O] genome's weights for this lane (numpy_nn.py:52-69
// layout: layer l is a row-major (out, in + bias) block, bias column last) and
// computes the error bound of the f32 output pre-activations:
//   hidden a_j error  <= 11u R_j           (R_j = sum_i |W1_ji| incl. bias; |x_i| <= 1)
//   sigmoid error     <= 2.75u R_j + 4.5u  (v_exp_f32/v_rcp_f32 ~1 ulp, slope <= 1/4)
//   output z_o error  <= sum_j |W2_oj| (3u R_j + 5u) + 13u (sum_j |W2_oj| + |c_o|)
// and keeps twice the largest over o (DESIGN.md "Certified argmax").
template <int L, int U, int O, typename WT>
__device__ __forceinline__ void load_net(Net<U, O> &n, const WT *__restrict__ g, int H, int b, int lig) {
  const int cols = 6 + b;
  const long off2 = (long)H * cols;
  float acc[O];
  float big = 0.f;  // sum of this lane's |weights|: NaN / inf / huge -> see kWeightCap
#pragma unroll
  for (int o = 0; o < O; ++o) acc[o] = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = lig + L * u;
    const bool ok = j < H;
    const int jj = ok ? j : 0;  // padding units load a valid row and are zeroed
    // Issue the unit's loads unconditionally, then mask arithmetically: a
    // select on a load is turned into a branch around it by the backend,
    // which serialises every load behind its own s_waitcnt.
    WT raw[7 + O];
#pragma unroll
    for (int i = 0; i < 7; ++i) raw[i] = g[(long)jj * cols + ((i < 6 || b) ? i : 0)];
#pragma unroll
    for (int o = 0; o < O; ++o) raw[7 + o] = g[off2 + (long)o * (H + b) + jj];
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const float m = (ok && (i < 6 || b)) ? 1.f : 0.f;
      n.w1[u][i] = (float)raw[i] * m;
      r += fabsf(n.w1[u][i]);
    }
#pragma unroll
    for (int o = 0; o < O; ++o) {
      n.w2[u][o] = (float)raw[7 + o] * (ok ? 1.f : 0.f);
      acc[o] += fabsf(n.w2[u][o]) * (3.f * r + 18.f);
    }
    big += r;
#pragma unroll
    for (int o = 0; o < O; ++o) big += fabsf(n.w2[u][o]);
    // bound the loads in flight (f64: 2 VGPRs each): this cold spot would
    // otherwise set the register budget of the whole kernel
    if ((u + 1) % PG_LOAD_BATCH == 0) __builtin_amdgcn_sched_barrier(0);
  }
  WT rawc[O];
#pragma unroll
  for (int o = 0; o < O; ++o) rawc[o] = g[off2 + (long)o * (H + b) + (b ? H : 0)];
  float e = 0.f;
#pragma unroll
  for (int o = 0; o < O; ++o) {
    n.c[o] = (float)rawc[o] * (b ? 1.f : 0.f);
    big += fabsf(n.c[o]);
  }
#pragma unroll
  for (int o = 0; o < O; ++o) e = fmaxf(e, 2.f * kU * (group_sum<L>(acc[o]) + 13.f * fabsf(n.c[o])));
  // any lane of the group over the cap (or NaN): the whole network is f64-decided
  n.e = group_sum<L>(weights_ok(big) ? 0.f : 1.f) > 0.f ? __builtin_inff() : e;
}

__device__ __forceinline__ float sigmoid_f32(float a) {
  // 1 / (1 + e^-a) with v_exp_f32 (2^x) and v_rcp_f32, ~1 ulp each
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a * -1.4426950408889634f));
}

// Hidden layer and the lane-partial output sums of one network for this lane.
template <int U, int O>
__device__ __forceinline__ void partial_f32(const Net<U, O> &n, const float x[6], float acc[O]) {
#pragma unroll
  for (int o = 0; o < O; ++o) acc[o] = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float a = n.w1[u][6];
#pragma unroll
    for (int i = 0; i < 6; ++i) a = fmaf(n.w1[u][i], x[i], a);
    const float s = sigmoid_f32(a);
#pragma unroll
    for (int o = 0; o < O; ++o) acc[o] = fmaf(n.w2[u][o], s, acc[o]);
  }
}

// ---- packed layout of the split kernel -------------------------------------
// Units in pairs (u = 2p, 2p+1) as float2, so the hidden layer runs on
// v_pk_fma_f32: one instruction advances two independent dot products, which
// halves the issue count and the length of the dependent chain per frame.
// W1 is stored pre-scaled by -log2(e) / 320 (feature columns; the features
// then enter as the exact integers k) and -log2(e) (bias column), so the
// pre-activation feeds v_exp_f32 directly: a' = -a log2 e.  Each stored
// weight carries one more rounding (<= 2u relative in all), and the fma chain
// over exact inputs stays within the 11u R_j hidden-error term of load_net.
typedef float float2v __attribute__((ext_vector_type(2)));

// certify()'s per-network constants, made once per game from the bound e
// (make_cert) instead of every frame: the moved thresholds, the low-z limit,
// the gap rule's 2e plus the plateau width's constant part, and the exponent
// offset of its e^(top1 + e) part: 2^-50 (e^(top1+e) + 1) = 2^(top1 log2 e +
// ee) + 2^-50 with ee = e log2 e - 50 (the f32 roundings of these forms are
// ~1e-6 relative, inside the width's x4 margin and the bound's x2 slack).
struct Cert {
  float tlo, thi, lowz, e2, ee;
};
constexpr float kCertTlo = 36.7367f, kCertThi = 36.7369f, kCertLowZ = -708.0f;

__device__ __forceinline__ Cert make_cert(float e) {
  return Cert{kCertTlo - e, kCertThi + e, kCertLowZ + e, 2.f * e + 8.8817842e-16f,
              e * 1.4426950408889634f - 50.f};
}

template <int U, int O>
struct NetP {
  static constexpr int P = (U + 1) / 2;  // unit pairs
  float2v w1[P][7];  // pre-scaled input weights (6 features + bias) of units 2p, 2p+1
  float2v w2[P][O];  // output weights of the pair
  float c[O];        // output biases
  float e;           // certified bound, as Net::e
  Cert ct;           // certify_c's constants from e (load_rec)
};

// Number of f32 roundings one term of an output sum of the packed forward
// passes: the chain of P = (U + 1) / 2 pk_fma of its component (partial_pk:
// unit 2p + h lands in component h), the .x + .y fold, the log2(HL) levels of
// the group tree, the + c after it (or, partial_pk's kBiasIn, nothing: the
// bias shares start the chains), and the f32 rounding of W2: P + log2(HL) + 3.
// (Until round 5 the bound took U for P, twice the chain: a wider bound, more
// certificate failures, the same decisions.)
template <int HL, int U>
__host__ __device__ constexpr int out_roundings() {
  return (U + 1) / 2 + (HL >= 32 ? 5 : HL >= 16 ? 4 : HL >= 8 ? 3 : HL >= 4 ? 2 : HL >= 2 ? 1 : 0) + 3;
}

// flip (the left paddle's network in k_service): the x-flip and me/enemy
// swap of get_actions (main.py:146-147) folded into the weights, so both
// halves of a group read the same feature vector k = [bx, by, lbx, lby, right,
// left]: the left network sees x = [1 - k0, k1, 1 - k2, k3, k5, k4] (x320),
// i.e. W'0 = -W0, W'2 = -W2, W'4 = W5, W'5 = W4 and bias' = bias + W0 + W2,
// folded in f64 and rounded to f32 once -- an f32 network of the same exact
// pre-activations, so the bound below (computed from the folded weights)
// covers it; the f64 fold error (<= 2^-51 R_j) fits the 3u R_j term's slack.
template <int L, int U, int O, typename WT>
__device__ __forceinline__ void load_net_pk(NetP<U, O> &n, const WT *__restrict__ g, int H, int b, int lig,
                                            int flip = 0) {
  constexpr int P = NetP<U, O>::P;
  constexpr float kScaleX = -1.4426950408889634f / 320.f;
  constexpr float kScaleB = -1.4426950408889634f;
  const int cols = 6 + b;
  const long off2 = (long)H * cols;
  float acc[O];
  float big = 0.f;
#pragma unroll
  for (int o = 0; o < O; ++o) acc[o] = 0.f;
#pragma unroll
  for (int p = 0; p < P; ++p) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = 2 * p + h;
      const int j = lig + L * u;
      const bool ok = u < U && j < H;
      const int jj = ok ? j : 0;  // padding units load a valid row and are zeroed
      WT raw[7 + O];  // unconditional loads, masked arithmetically (see load_net)
#pragma unroll
      for (int i = 0; i < 7; ++i) raw[i] = g[(long)jj * cols + ((i < 6 || b) ? i : 0)];
#pragma unroll
      for (int o = 0; o < O; ++o) raw[7 + o] = g[off2 + (long)o * (H + b) + jj];
      float wf[7];
#pragma unroll
      for (int i = 0; i < 7; ++i) wf[i] = (float)raw[i] * ((ok && (i < 6 || b)) ? 1.f : 0.f);
      if (flip) {  // only the bias is folded in f64 (one rounding); the rest are exact f32 moves
        const double bias = (((ok && b) ? (double)raw[6] : 0.0) + (ok ? (double)raw[0] : 0.0)) +
                            (ok ? (double)raw[2] : 0.0);
        const float w4 = wf[4];
        wf[0] = -wf[0];
        wf[2] = -wf[2];
        wf[4] = wf[5];
        wf[5] = w4;
        wf[6] = (float)bias;
      }
      float r = 0.f;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        r += fabsf(wf[i]);
        n.w1[p][i][h] = wf[i] * (i < 6 ? kScaleX : kScaleB);
      }
      big += r;
#pragma unroll
      for (int o = 0; o < O; ++o) {
        const float w = (float)raw[7 + o] * (ok ? 1.f : 0.f);
        n.w2[p][o][h] = w;
        acc[o] += fabsf(w) * (3.f * r + 5.f + (float)out_roundings<L, U>());
        big += fabsf(w);
      }
    }
    if ((p + 1) % PG_LOAD_BATCH == 0) __builtin_amdgcn_sched_barrier(0);
  }
  WT rawc[O];
#pragma unroll
  for (int o = 0; o < O; ++o) rawc[o] = g[off2 + (long)o * (H + b) + (b ? H : 0)];
  float e = 0.f;
#pragma unroll
  for (int o = 0; o < O; ++o) {
    n.c[o] = (float)rawc[o] * (b ? 1.f : 0.f);
    big += fabsf(n.c[o]);
  }
#pragma unroll
  for (int o = 0; o < O; ++o)
    e = fmaxf(e, 2.f * kU * (group_sum<L>(acc[o]) + (float)out_roundings<L, U>() * fabsf(n.c[o])));
  // any lane of the group over the cap (or NaN): the whole network is f64-decided
  n.e = group_sum<L>(weights_ok(big) ? 0.f : 1.f) > 0.f ? __builtin_inff() : e;
}

// ---- lane records: what load_net_pk leaves in one lane's registers, laid
// out flat (w1 pairs, w2 pairs, c, e; padded to whole 16-B pieces) so a game
// start is rec_floats / 4 independent 16-B loads and one wait instead of the
// genome gather, the f32 conversion, the x-flip fold and the bound's group
// sums (k_prep_records prepares every network of a launch once).
template <int U, int O>
__host__ __device__ constexpr int rec_floats() {
  return ((U + 1) / 2 * 2 * (7 + O) + O + 1 + 3) / 4 * 4;
}

template <int U, int O>
__device__ __forceinline__ void store_rec(const NetP<U, O> &n, float *__restrict__ r) {
  constexpr int P = NetP<U, O>::P;
  constexpr int F = rec_floats<U, O>();
  float v[F];
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      v[(p * 7 + i) * 2] = n.w1[p][i].x;
      v[(p * 7 + i) * 2 + 1] = n.w1[p][i].y;
    }
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int o = 0; o < O; ++o) {
      v[P * 14 + (p * O + o) * 2] = n.w2[p][o].x;
      v[P * 14 + (p * O + o) * 2 + 1] = n.w2[p][o].y;
    }
#pragma unroll
  for (int o = 0; o < O; ++o) v[P * 14 + P * O * 2 + o] = n.c[o];
  v[P * 14 + P * O * 2 + O] = n.e;
#pragma unroll
  for (int f = P * 14 + P * O * 2 + O + 1; f < F; ++f) v[f] = 0.f;
  float4 *d = reinterpret_cast<float4 *>(r);
#pragma unroll
  for (int q = 0; q < F / 4; ++q) d[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

// The output layer's part of a lane record (w2 pairs, c, e; after the P x 7
// w1 pairs): what k_service's in-wave decision path hands to the f64 code's
// registers and reloads afterwards (the record's 16-B pieces from the one
// holding the first w2 float).
template <int U, int O>
__device__ __forceinline__ void load_rec_out(NetP<U, O> &n, const float *__restrict__ r) {
  constexpr int P = NetP<U, O>::P;
  constexpr int F = rec_floats<U, O>();
  constexpr int B = P * 14 / 4 * 4;  // the 16-B piece holding the first w2 float
  constexpr int D = P * 14 - B;       // (0 when P is even)
  const float4 *s = reinterpret_cast<const float4 *>(r + B);
  float v[F - B];
#pragma unroll
  for (int q = 0; q < (F - B) / 4; ++q) {
    const float4 x = s[q];
    v[4 * q] = x.x;
    v[4 * q + 1] = x.y;
    v[4 * q + 2] = x.z;
    v[4 * q + 3] = x.w;
  }
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int o = 0; o < O; ++o) n.w2[p][o] = float2v{v[D + (p * O + o) * 2], v[D + (p * O + o) * 2 + 1]};
#pragma unroll
  for (int o = 0; o < O; ++o) n.c[o] = v[D + P * O * 2 + o];
  n.e = v[D + P * O * 2 + O];
  n.ct = make_cert(n.e);
}

template <int U, int O>
__device__ __forceinline__ void load_rec(NetP<U, O> &n, const float *__restrict__ r) {
  constexpr int P = NetP<U, O>::P;
  constexpr int F = rec_floats<U, O>();
  const float4 *s = reinterpret_cast<const float4 *>(r);
  float v[F];
#pragma unroll
  for (int q = 0; q < F / 4; ++q) {
    const float4 x = s[q];
    v[4 * q] = x.x;
    v[4 * q + 1] = x.y;
    v[4 * q + 2] = x.z;
    v[4 * q + 3] = x.w;
  }
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int i = 0; i < 7; ++i) n.w1[p][i] = float2v{v[(p * 7 + i) * 2], v[(p * 7 + i) * 2 + 1]};
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int o = 0; o < O; ++o) n.w2[p][o] = float2v{v[P * 14 + (p * O + o) * 2], v[P * 14 + (p * O + o) * 2 + 1]};
#pragma unroll
  for (int o = 0; o < O; ++o) n.c[o] = v[P * 14 + P * O * 2 + o];
  n.e = v[P * 14 + P * O * 2 + O];
  n.ct = make_cert(n.e);
}

// Hidden layer and the lane-partial output sums of one packed network; k are
// the six doubled-centroid features (x_i = k_i / 320 is folded into W1).
// kBiasIn: n.c holds the lane's share of the output bias (k_service: half of
// it on the group's first lane, both halves of its packed chains start from
// it; zero elsewhere), so the group sum is z itself -- no add per output.
// Each share passes the same roundings as a W2 term (<= out_roundings).
template <int U, int O, bool kBiasIn = false>
__device__ __forceinline__ void partial_pk(const NetP<U, O> &n, const int k[6], float acc[O]) {
  constexpr int P = NetP<U, O>::P;
  float2v kx[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float f = (float)k[i];
    kx[i] = float2v{f, f};
  }
  float2v a2[O];
#pragma unroll
  for (int o = 0; o < O; ++o) a2[o] = kBiasIn ? float2v{n.c[o], n.c[o]} : float2v{0.f, 0.f};
  // two unit pairs per step: their dependent pk_fma chains interleave, so the
  // wait state a packed op owes its dependent successor is filled with work
#pragma unroll
  for (int p = 0; p < P; p += 2) {
    constexpr int kStep = 2;
    const bool two = p + 1 < P;
    float2v a = n.w1[p][6], b = two ? n.w1[p + 1][6] : float2v{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      a = __builtin_elementwise_fma(n.w1[p][i], kx[i], a);
      if (two) b = __builtin_elementwise_fma(n.w1[p + 1][i], kx[i], b);
    }
    const float2v qa = float2v{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)} + 1.0f;
    const float2v qb = float2v{__builtin_amdgcn_exp2f(b.x), __builtin_amdgcn_exp2f(b.y)} + 1.0f;
    const float2v sa = float2v{__builtin_amdgcn_rcpf(qa.x), __builtin_amdgcn_rcpf(qa.y)};
    const float2v sb = float2v{__builtin_amdgcn_rcpf(qb.x), __builtin_amdgcn_rcpf(qb.y)};
#pragma unroll
    for (int o = 0; o < O; ++o) {
      a2[o] = __builtin_elementwise_fma(n.w2[p][o], sa, a2[o]);
      if (two) a2[o] = __builtin_elementwise_fma(n.w2[p + 1][o], sb, a2[o]);
    }
    (void)kStep;
  }
#pragma unroll
  for (int o = 0; o < O; ++o) acc[o] = a2[o].x + a2[o].y;
}

// The bound of one frame (serve_inline, before the f64 stage): load_net_pk's
// derivation with this frame's magnitudes where it takes the worst case.  Per
// hidden unit j, in a' = -a log2 e units (the records'):
//   R'_j  = sum_i |w'_ji k_i| + |w'_j6|  (+ 2^-20 320 sum_i |w'_ji|, the
//           x-flip fold's f64 rounding)       instead of |x_i| <= 1
//   da'_j = 11u R'_j                            the pre-activation error
//   slope = min(1/4, 2^(2 da'_j - |a'_j|))      s(1-s) <= e^-|a| = 2^-|a'|, over
//           every point within 2 da'_j of the recomputed a'_j (the true one
//           and partial_pk's: both within da'_j of the exact value)
//                                               instead of 1/4
//   ds_j  = slope da'_j ln 2 + 5u s_j + 2^-100  the sigmoid's error: the
//           propagated part and v_exp/+1/v_rcp's relative ~1 ulp each (s = 0
//           or 1 saturated: the floor)          instead of 3u R_j + 5u
//   z_o error <= sum_j |W2_oj| (ds_j + OR u s_j) + OR u |c_o|
//           (OR = out_roundings, its terms' magnitudes |W2_oj s_j|)
// and twice the largest over o, as load_net_pk.  Saturated units -- most of
// an evolved network's -- drop out of the propagated part and negative ones
// out of the sums', so the frame's bound is ~4x tighter than the network's on
// the bench's N(0, 3) genes (tests/test_frame_bound.py restates it in numpy
// and checks it against f64): the near-ties it separates skip the f64 stage.
// By the whole wave for one half-group's network: lane t takes the units of
// slot t (rec: the half-group's first lane record; record hl holds units
// hl + HL u, u = 2p + h, and the full output biases), so the requesting
// lanes' registers are not needed -- they are the f64 code's by then.
template <int HL, int U, int O>
__device__ __forceinline__ float frame_bound_wave(const float *__restrict__ rec, const int k[6], int lane64) {
  constexpr int P = NetP<U, O>::P;
  constexpr int F = rec_floats<U, O>();
  constexpr float kOR = (float)out_roundings<HL, U>();
  float acc[O];
#pragma unroll
  for (int o = 0; o < O; ++o) acc[o] = 0.f;
#pragma unroll 1
  for (int t = lane64; t < HL * 2 * P; t += 64) {  // padding units hold zero weights
    const int hl = t % HL, u = t / HL, p = u >> 1, h = u & 1;
    const float *r = rec + hl * F;
    float w[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) w[i] = r[(p * 7 + i) * 2 + h];
    float w2[O];
#pragma unroll
    for (int o = 0; o < O; ++o) w2[o] = r[P * 14 + (p * O + o) * 2 + h];
    float a = w[6], rr = fabsf(w[6]), ws = fabsf(w[6]);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      a = fmaf(w[i], (float)k[i], a);
      rr = fmaf(fabsf(w[i]), (float)k[i], rr);
      ws += fabsf(w[i]);
    }
    const float da = (rr + ws * (320.f * 9.5367431640625e-7f)) * (11.f * kU);
    const float sl = fminf(0.25f, __builtin_amdgcn_exp2f(2.f * da - fabsf(a)));
    const float s = __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(a) + 1.0f);
    const float ds = sl * da * 0.6931471805599453f + s * ((5.f + kOR) * kU) + 7.8886090522101181e-31f;
#pragma unroll
    for (int o = 0; o < O; ++o) acc[o] = fmaf(fabsf(w2[o]), ds, acc[o]);
  }
  float e = 0.f;
#pragma unroll
  for (int o = 0; o < O; ++o)
    e = fmaxf(e, 2.f * (group_sum<64>(acc[o]) + kOR * kU * fabsf(rec[P * 14 + P * O * 2 + o])));
  return e;
}

// Certified argmax of S(z) = 1/(1 + pow(e, -z)) in f64 (numpy_nn.py:22-23,131)
// given |z_true - z[o]| <= e.  S is exactly 1.0 iff z >= 53 ln 2 =
// 36.73680056967710 (then every saturated output ties and the first wins);
// below that S rounds onto plateaus no wider than 2^-52 (e^z + 1) in z (x4
// margin below).  Returns -1 when the bound cannot prove the f64 decision;
// the caller then recomputes the forward pass in f64.
// certify() on the per-network constants (same rule; k_service's frame)
template <int O>
__device__ __forceinline__ int certify_c(const float z[O], const Cert &c) {
  int sat_res = z[O - 1] > c.thi ? O - 1 : -1;
#pragma unroll
  for (int o = O - 2; o >= 0; --o) sat_res = z[o] > c.thi ? o : (z[o] >= c.tlo ? -1 : sat_res);
  float top1, top2;
  int w;
  if constexpr (O == 3) {
    top1 = fmaxf(fmaxf(z[0], z[1]), z[2]);
    top2 = __builtin_amdgcn_fmed3f(z[0], z[1], z[2]);
    w = z[0] == top1 ? 0 : (z[1] == top1 ? 1 : 2);
  } else {
    top1 = z[0];
    top2 = -3.0e38f;
    w = 0;
#pragma unroll
    for (int o = 1; o < O; ++o) {
      const bool gt = z[o] > top1;
      top2 = gt ? top1 : fmaxf(top2, z[o]);
      w = gt ? o : w;
      top1 = gt ? z[o] : top1;
    }
  }
  const float tw = __builtin_amdgcn_exp2f(__builtin_fmaf(top1, 1.4426950408889634f, c.ee));
  const int uns_res = (top1 - top2 > c.e2 + tw && top1 > c.lowz) ? w : -1;
  return top1 >= c.tlo ? sat_res : uns_res;
}

// certify_c's decision as the paddle move it selects (index_to_move:
// k_service keeps its actions so), or -1 (no move is -1).  Three outputs: the winner's code
// straight from the compares, and the saturated rule as "the first output at
// or above tlo decides if it is above thi" (one select chain instead of a
// chain per output).
template <int O>
__device__ __forceinline__ int certify_c8(const float z[O], const Cert &c) {
  if constexpr (O == 3) {
    const float top1 = fmaxf(fmaxf(z[0], z[1]), z[2]);
    const float top2 = __builtin_amdgcn_fmed3f(z[0], z[1], z[2]);
    const int wc = z[0] == top1 ? -6 : (z[1] == top1 ? 6 : 0);  // index_to_move of the first maximum
    const float tw = __builtin_amdgcn_exp2f(__builtin_fmaf(top1, 1.4426950408889634f, c.ee));
#ifndef PG_CERT_FULL_SAT
    // saturated: decided here only when the winner is the one output that may
    // be saturated (top2 < tlo) and surely is; two or more maybe-saturated
    // outputs (ties at 1.0 in f64) are left to the plateau rule (plateau_f32)
    // (bitwise on the compares: lane masks, no divergent branches; top1 > thi
    // implies top1 >= tlo, the saturated regime)
    const bool ok = ((top2 < c.tlo) & (top1 > c.thi)) | ((top1 < c.tlo) & (top1 - top2 > c.e2 + tw) & (top1 > c.lowz));
    return ok ? wc : -1;
#else
    const bool m0 = z[0] >= c.tlo, m1 = z[1] >= c.tlo;  // (with top1 >= tlo one of the three is)
    const int fc = m0 ? -6 : (m1 ? 6 : 0);  // index_to_move of the first maybe-saturated output
    const float zf = m0 ? z[0] : (m1 ? z[1] : z[2]);
    const int sat_res = zf > c.thi ? fc : -1;
    const int uns_res = (top1 - top2 > c.e2 + tw && top1 > c.lowz) ? wc : -1;
    return top1 >= c.tlo ? sat_res : uns_res;
#endif
  } else {
    const int idx = certify_c<O>(z, c);
    return idx < 0 ? -1 : index_to_move(idx);
  }
}

// The gap rule of certify_c with the plateau width at its true size, for the
// frames certify_c8 leaves undecided in the plateau regime (k_service's rare
// block, before plateau_f32).  When both of the two largest outputs are in the
// regime (top2 - e >= 22.2: S = 1 - m 2^-52, m = rint(2^52 pow(e, -z)), pow
// within 1 ulp), the winner's m is strictly the smaller -- its S strictly the
// larger -- once 2^52 (e^-(top2 + e) (1 - 2^-52) - e^-(top1 - e) (1 + 2^-52)) > 1,
// which holds when top1 - top2 > 2e + 2^-52 e^top1 + 2^-51 (ln(1 + x) <= x).
// certify_c prices the width at 4 2^-52 (e^(top1 + e) + 1), valid at every z;
// here it is 2^-52 e^top1 x 1.01 (the f32 exponent's and v_exp_f32's error,
// ~2e-6 relative) -- about 4x fewer undecided frames in populations evolved
// from U[0,1) genes (ga.py:85), no transcendental beyond the one exp2.
// Returns the paddle move (index_to_move) or -1.
template <int O>
__device__ __forceinline__ int tight_gap_move(const float z[O], float e, const Cert &c) {
  float top1, top2;
  int w;
  if constexpr (O == 3) {
    top1 = fmaxf(fmaxf(z[0], z[1]), z[2]);
    top2 = __builtin_amdgcn_fmed3f(z[0], z[1], z[2]);
    w = z[0] == top1 ? 0 : (z[1] == top1 ? 1 : 2);
  } else {
    top1 = z[0];
    top2 = -3.0e38f;
    w = 0;
#pragma unroll
    for (int o = 1; o < O; ++o) {
      const bool gt = z[o] > top1;
      top2 = gt ? top1 : fmaxf(top2, z[o]);
      w = gt ? o : w;
      top1 = gt ? z[o] : top1;
    }
  }
  // 2^(top1 log2 e - 52 + log2 1.01) + 2^-51; the sum's f32 roundings inside the (1 + 2^-20)
  const float tw = __builtin_amdgcn_exp2f(__builtin_fmaf(top1, 1.4426950408889634f, -51.985645f)) +
                   4.4408921e-16f;
  const bool ok = (top2 - e >= 22.2f) & (top1 < c.tlo) & (top1 - top2 > (2.f * e + tw) * 1.000001f);
  return ok ? index_to_move(w) : -1;
}

template <int O>
__device__ __forceinline__ int certify(const float z[O], float e) {
  // Branch-free: (a) the first output that may be saturated decides if it
  // surely is (it ties at 1.0 with every later saturated one and beats every
  // unsaturated one); (b) with none possibly saturated, the f32 winner must
  // lead the runner-up by 2e plus the plateau width at its value.
  // The thresholds move by e once instead of every z by e: z >= kTlo - e
  // "may be saturated", z > kThi + e "surely is" (the f32 rounding of either
  // form is ~1e-6 of the 1e-4 margins around 53 ln 2 and within the bound's x2
  // slack).  An infinite e (weights_ok failed) makes every output "maybe" and
  // none "sure": -1.
  constexpr float kTlo = 36.7367f, kThi = 36.7369f;
  constexpr float kLowZ = -708.0f;
  const float tlo = kTlo - e, thi = kThi + e;
  // (a) the first maybe-saturated output decides if it surely is (a sure
  // output is a maybe one), else -1
  int sat_res = z[O - 1] > thi ? O - 1 : -1;
#pragma unroll
  for (int o = O - 2; o >= 0; --o) sat_res = z[o] > thi ? o : (z[o] >= tlo ? -1 : sat_res);
  float top1, top2;
  int w;
  if constexpr (O == 3) {  // v_max3 / v_med3: the largest and the runner-up (equal to it on a tie)
    top1 = fmaxf(fmaxf(z[0], z[1]), z[2]);
    top2 = __builtin_amdgcn_fmed3f(z[0], z[1], z[2]);
    w = z[0] == top1 ? 0 : (z[1] == top1 ? 1 : 2);
  } else {
    top1 = z[0];
    top2 = -3.0e38f;
    w = 0;
#pragma unroll
    for (int o = 1; o < O; ++o) {
      const bool gt = z[o] > top1;
      top2 = gt ? top1 : fmaxf(top2, z[o]);
      w = gt ? o : w;
      top1 = gt ? z[o] : top1;
    }
  }
  // (top1 + e < kTlo whenever this rule is used: no saturated output)
  const float tw = 8.8817842e-16f * (__expf(top1 + e) + 1.0f);
  // the gap rule needs the winner's S(z) normal: below z = -1022 ln 2 it is
  // subnormal (coarse steps), and 0.0 for every z < -709.78 (pow overflows),
  // where all such outputs tie and the first wins -- the f64 path decides there
  const int uns_res = (top1 - top2 > 2.f * e + tw && top1 > kLowZ + e) ? w : -1;
  // no NaN test: outputs are finite whenever e is (weights_ok at load time);
  // the largest output maybe-saturated <=> some output is
  return top1 >= tlo ? sat_res : uns_res;
}

// The f64 re-decision of one forward pass by the L lanes of a group, in
// numpy's order: every dot product as np.dot runs it (blas_dot: OpenBLAS
// dgemv_t's summation), every sigmoid correctly rounded (pg_sigmoid_f64).
// Hidden units are strided over the lanes; the output rows are staged in LDS
// by all lanes (coalesced) and lane o < O sums output o out of LDS -- no
// serial global loads.
// LDS: lds[0, H) hidden activations, lds[H + o*(H+1) + j] output weights,
// then O output activations (f64_out_offset); f64_lds_doubles(H, O) doubles.
__host__ __device__ constexpr int f64_lds_doubles(int H, int O) { return H + O * (H + 1) + O + 1; }
__host__ __device__ constexpr int f64_out_offset(int H, int O) { return H + O * (H + 1); }

template <int L, int U, int O, typename WT>
__device__ PG_SLOW_INLINE int forward_f64_group(const WT *__restrict__ g, int H, int b, const double *x, double *lds,
                                              int lig) {
  const int cols = 6 + b;
#pragma unroll 1
  for (int j = lig; j < H; j += L) {
    const WT *row = g + (long)j * cols;
    double w[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) w[i] = (i < 6 || b) ? (double)row[i] : 0.0;
    lds[j] = pg_sigmoid_f64(blas_dot6(w, x, b));
  }
  double *w2 = lds + H;
  const WT *v = g + (long)H * cols;
#pragma unroll 1
  for (int t = lig; t < O * (H + b); t += L) {
    const int o = t / (H + b), j = t - o * (H + b);
    w2[o * (H + 1) + j] = (double)v[(long)o * (H + b) + j];
  }
  wave_lds_sync();
  double *out = lds + f64_out_offset(H, O);
  if (lig < O) {
    const double *wr = w2 + lig * (H + 1);
    const double z = blas_dot([&](int j) { return wr[j]; }, [&](int j) { return j < H ? lds[j] : 1.0; }, H + b,
                              blas_kind(lig, O));
    out[lig] = pg_sigmoid_f64(z);
  }
  wave_lds_sync();
  int best = 0;  // np.argmax: the first NaN if any, else the first maximum
  for (int o = 1; o < O && !__builtin_isnan(out[best]); ++o)
    if (__builtin_isnan(out[o]) || out[o] > out[best]) best = o;
  wave_lds_sync();
  return best;
}

// The same from the doubled-centroid features k (utils.inference's values).
template <int L, int U, int O, typename WT>
__device__ PG_SLOW_INLINE int forward_f64_group(const WT *__restrict__ g, int H, int b, const int *k, double *lds,
                                              int lig) {
  double x[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = __dmul_rn(0.5, (double)k[i]) / 160.0;
  return forward_f64_group<L, U, O, WT>(g, H, b, (const double *)x, lds, lig);
}

__device__ __forceinline__ float feat32(int k) { return (float)k * 0.003125f; }  // k / 320, <= 2u rel. error

template <int L>
__device__ __forceinline__ int group_broadcast(int v, int leader_lane) {
  if constexpr (L == 64) return __builtin_amdgcn_readfirstlane(v);
  return __shfl(v, leader_lane, 64);
}

// ================================================ split-lane helpers ==
template <int L>
__device__ __forceinline__ int other_half(int v) {
  // (every lane reads a valid source lane, so no old value is needed: one
  // v_mov_b32_dpp, no copy or zero ahead of it)
  if constexpr (L == 8) {
    return __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false);  // row_half_mirror: i <-> 7-i
  } else if constexpr (L == 16) {
    return __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false);  // row_mirror: i <-> 15-i
  } else if constexpr (L == 32) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (threadIdx.x & 16) ? (int)r[0] : (int)r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (threadIdx.x & 32) ? (int)r[0] : (int)r[1];
  }
}

// ============================================ split lanes + f64 service wave ==
// k_split's layout, with the rare f64 re-decision moved to a dedicated wave:
// a block (svc_threads) runs its game waves and ONE service wave.  A half-group
// whose certificate fails posts {genome, features} to an LDS mailbox and
// sleeps until the service wave (64 lanes, numpy_nn order, f64) answers.  The
// f64 code then lives in its own control-flow region, so it no longer sets
// the game waves' register budget (which decides their occupancy).
// Block size by register budget: a game lane holds 10U + 4 weight floats, so
// U <= 4 fits 128 VGPRs (4 waves/SIMD: 16-wave blocks), U = 8 fits 168
// (3 waves/SIMD: 12-wave blocks), U = 16 fits 256 (2 waves/SIMD: 8-wave blocks).
// One block per CU either way; PG_SVC_NT forces one size (experiments).
template <int U>
__host__ __device__ constexpr int svc_threads() {
#ifdef PG_SVC_NT
  return PG_SVC_NT;
#else
  return U <= 4 ? 1024 : (U <= 8 ? 768 : 512);
#endif
}

// A game whose rally settles into a periodic orbit meets the same near-tie
// states every period; without a memo each costs a round trip to the service
// wave (~3 us), and such games ran 3-4x slower per frame and set the launch's
// tail (tools/timeline.py).  The memo holds the network's last kMemo f64
// decisions keyed by the packed features -- the decision is a pure function
// of (network, features), so a hit is exact.  Cleared at every game start.
constexpr int kMemo = 8;

// The lane's index in its wave, computed afresh (volatile: never hoisted or
// merged), for lane values a rare block needs but the hot loop should not
// keep live.
__device__ __forceinline__ int fresh_lane64() {
  int r;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
  return r;
}

// Relaxed workgroup-scope atomics on LDS words that another wave polls.  Not
// `volatile`: a volatile access through the generic pointer of a __shared__
// variable is not rewritten to LDS and becomes a flat access (sc0 sc1, a trip
// through the vector-memory pipe, and a wait on every outstanding global load
// and store of the wave).
__device__ __forceinline__ int lds_ld(int *a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(int *a, int v) {
  __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

struct SlowSlot {
  const void *g;    // genome row of the network to re-decide
  int k[6];         // its doubled-centroid features
  float z[4];       // the f32 output pre-activations and their bound e
  float e;
  int idx;          // answer: argmax index
  int flag;  // 0 free, 1 posted, 2 answered (shared with the service wave: lds_ld / lds_st)
  int n_memo;  // decisions memoised for the current game's network (the owning group only)
  uint64_t memo_key[kMemo];
  int memo_idx[kMemo];  // the decision: its paddle move (index_to_move)
  uint64_t rally_key;  // Brent's saved rally key of the slot's game (side-0 slot of a group)
  int rally_at, rally_span;
  int rec;  // k_service inline form: the slot's network's lane-record index (its reload after a decision)
};

// fixed-horizon mode (pg_eval_args.horizon), one per game group: the completed
// episodes' reward sum, count and ZeroDivisionError flag, every episode's points
struct HorizonSlot {
  double sum;
  int eps, s1, s2, zd;
};

// The plateau certificate in f32, tried by the game wave itself where
// certify() failed (no round trip to the service wave).  Same rule as
// plateau_decide below, but m(z) = rint(2^52 pow(e, -z)) is only bracketed:
// v = exp2(52 - z log2 e) in f32 is within 2e-5 v of 2^52 e^-z (exponent
// rounding <= (|t| + 2 |z| log2 e) u, v_exp_f32 ~1 ulp, x4 margin), so
// ceil(v(z + e) - d - 1/2) <= m_true <= floor(v(z - e) + d + 1/2).  Useful
// where v is small (z >~ 28); near 22 the bracket is wide and the service
// decides.
template <int O>
__device__ __forceinline__ int plateau_f32(const float z[O], float e) {
  constexpr int kBelow = 0x7ffffff0;  // S below the plateau regime (z < 22)
  constexpr int kNone = 0x7fffffff;   // cannot bracket
  int mlo[O], mhi[O];
  bool bad = false;
#pragma unroll
  for (int o = 0; o < O; ++o) {
    const float zl = z[o] - e, zh = z[o] + e;
    bad = bad || !(zl == zl);  // NaN
    // upper bracket of m from the low end z - e (valid when z - e >= 22.2)
    if (zl >= 22.2f) {
      const float v = __builtin_amdgcn_exp2f(fmaf(-zl, 1.44269504f, 52.f));
      mhi[o] = (int)floorf(v * (1.f + 2e-5f) + 0.5f);
    } else {
      mhi[o] = kNone;
    }
    // lower bracket of m from the high end z + e
    if (zh >= 22.2f) {
      const float v = __builtin_amdgcn_exp2f(fmaf(-zh, 1.44269504f, 52.f));
      mlo[o] = (int)ceilf(v * (1.f - 2e-5f) - 0.5f);
    } else {
      mlo[o] = zh < 22.0f ? kBelow : -1;  // -1: straddles the regime edge, never "surely below"
    }
  }
  if (bad) return -1;
  int res = -1;
#pragma unroll
  for (int w = O - 1; w >= 0; --w) {
    bool ok = mhi[w] != kNone;
#pragma unroll
    for (int o = 0; o < O; ++o)
      if (o != w) ok = ok && (o < w ? mhi[w] < mlo[o] : mhi[w] <= mlo[o]);
    res = ok ? w : res;
  }
  return res;
}

// Plateau certificate, tried first by the service wave (no memory traffic).
// For z >= 22.2, numpy's S(z) = 1/(1 + pow(e, -z)) is exactly
// 1 - m(z) 2^-52 with m(z) = rint(2^52 pow(e, -z)) (1 + p rounds to
// 1 + m 2^-52; its reciprocal rounds to 1 - m 2^-52 while m < 2^20), so two
// outputs tie iff their m are equal and the larger S is the smaller m.  m is
// monotone in z, so with |z_true - z| <= e the f32 outputs bound each m
// between m(z + e) and m(z - e).  This decides the near-saturation rallies
// whose plateaus are too wide for certify()'s gap test.  Lanes 0..2O-1 each
// evaluate one endpoint; returns -1 when undecided (the full f64 path runs).
template <int O>
__device__ int plateau_decide(const float *z, float e, int lane) {
  constexpr int kBig = 0x7fffffff;  // "below the plateau regime": worse than any m
  int m = kBig;
  bool amb = false;
  if (lane < 2 * O) {
    float zo = z[0];  // z[lane >> 1] without a dynamic (scratch) index
#pragma unroll
    for (int o = 1; o < O; ++o) zo = (lane >> 1) == o ? z[o] : zo;
    const double zz = (double)zo + ((lane & 1) ? (double)e : -(double)e);
    if (zz != zz) {
      amb = true;  // NaN: numpy's NaN rule, in the f64 path
    } else if (zz >= PG_K(22.2)) {
      double t = pg_exp_f64(-zz);
      t = fma(t, zz * PG_K(5.318237706605891e-17), t);  // pow(e_d, -z) to ~1 ulp (the 1e-6 margin covers it)
      const double v = t * 4503599627370496.0;    // 2^52 p
      const double fr = v - floor(v);
      amb = fabs(fr - 0.5) < PG_K(1e-6);  // too close to a rounding boundary to call
      m = (int)rint(v);
    }
  }
  if (__ballot(amb)) return -1;
  int mlo[O], mhi[O];  // m(z + e) <= m_true <= m(z - e)
#pragma unroll
  for (int o = 0; o < O; ++o) {
    mhi[o] = __builtin_amdgcn_readlane(m, 2 * o);
    mlo[o] = __builtin_amdgcn_readlane(m, 2 * o + 1);
  }
#pragma unroll
  for (int w = 0; w < O; ++w) {
    bool ok = mhi[w] != kBig;
#pragma unroll
    for (int o = 0; o < O; ++o)
      if (o != w) ok = ok && (o < w ? mhi[w] < mlo[o] : mhi[w] <= mlo[o]);
    if (ok) return w;
  }
  return -1;
}

// Certified f64 decision, tried by the service wave before the numpy-order
// f64 forward.  The wave evaluates the network in f64 in parallel (one hidden
// unit per lane, tree sums) and bounds its distance to numpy's own f64 result
// z_np (numpy_nn.py:120-131: sequential dot products, bias last):
//   |z - z_np| <= e_o = 2 eps (sum_j |W2_oj| (4 A_j + 84) + 2 |c_o|),
// eps = 2^-53, A_j = sum_i |W1_ji x_i| + |b_j| -- both dot products within
// gamma_7 A_j of the exact one, slope <= 1/4, both sigmoids within 6 ulp,
// both output sums within gamma_66 + gamma_8 of exact, x2 margin.  That is
// ~1e-11, ten orders below the f32 bound, so the decision is almost always
// provable; with O outputs on lanes:
//  * for z >= 22.2, S_np(z) = 1 - m(z) 2^-52 exactly, m(z) = rint(2^52
//    pow(e, -z)) (1 + p rounds to 1 + m 2^-52, whose reciprocal rounds to
//    1 - m 2^-52 while m < 2^20); m is monotone, so [z - e, z + e] bounds m
//    between m(z + e) and m(z - e); ties are equal m, larger S is smaller m;
//  * below that, S is strictly increasing on gaps above the plateau width
//    4 2^-52 (e^z + 1), so a gap test decides.
// Returns -1 when undecided (NaN, a rounding boundary within 1e-6 of m's
// half-integer, or a tie the intervals cannot settle).
// Sum of a double over the 64 lanes (DPP within rows, permlane swaps across).
__device__ __forceinline__ double wave_sum_f64(double v) {
#define PG_DPP64(CTRL)                                                                          \
  {                                                                                           \
    const uint64_t bits = (uint64_t)__double_as_longlong(v);                                  \
    const uint32_t lo = __builtin_amdgcn_update_dpp(0u, (uint32_t)bits, CTRL, 0xF, 0xF, false); \
    const uint32_t hi = __builtin_amdgcn_update_dpp(0u, (uint32_t)(bits >> 32), CTRL, 0xF, 0xF, false); \
    v += __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));                        \
  }
  PG_DPP64(0xB1) PG_DPP64(0x4E) PG_DPP64(0x141) PG_DPP64(0x140)
#undef PG_DPP64
  {
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)bits, (uint32_t)bits, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(bits >> 32), (uint32_t)(bits >> 32), false, false);
    v = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0])) +
        __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
  }
  {
    const uint64_t bits = (uint64_t)__double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)bits, (uint32_t)bits, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(bits >> 32), (uint32_t)(bits >> 32), false, false);
    v = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0])) +
        __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
  }
  return v;
}

// One lane's hidden unit j in f64 (inputs x, weights w1[0..5], bias w1[6]):
// its sigmoid and the unit's share of fast_f64_decide's error bound, 4 A_j + 84.
__device__ __forceinline__ void f64_unit(const double *x, const double *w1, int b, double &sj, double &aj) {
  double a = b ? w1[6] : 0.0;
  double A = fabs(a);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    a = fma(w1[i], x[i], a);
    A = fma(fabs(w1[i]), x[i], A);
  }
  // the compact sigmoid (pow(e_d, -a) as exp(-a)(1 + a delta), ~1-2 ulp; the
  // bound above allows 6): no table load on the service's critical path
  double tq = pg_exp_f64(-a);
  if (tq < INFINITY) tq = fma(tq, a * PG_K(5.318237706605891e-17), tq);
  sj = 1.0 / (1.0 + tq);
  aj = 4.0 * A + 84.0;
}

__device__ __forceinline__ void f64_features(const int *k, double *x) {
#pragma unroll
  for (int i = 0; i < 6; ++i) x[i] = __dmul_rn(0.5, (double)k[i]) / 160.0;
}

// fast_f64_decide's decision from the lanes' partial output sums zp and bound
// sums ep (any lane order: e covers it) and the output biases c.  The bound's
// sum runs in f32 (a bound only needs to stay above its true value: 64 positive
// terms in f32 are within 64 2^-24 < 4e-6 of their exact sum, covered by the
// x1.001 margin below; each term is rounded up by 1 + 2^-22 first), one DPP
// f32 reduction instead of an f64 one of twice the moves.
template <int O>
__device__ int f64_decide_sums(const double *zp, const float *ep, const double *c, int lane) {
  constexpr double kEps = 1.1102230246251565e-16;  // 2^-53
  double z[O], e[O];
#pragma unroll
  for (int o = 0; o < O; ++o) {
    const double t = wave_sum_f64(zp[o]);
    const double u = (double)group_sum<64>(ep[o] * 1.00000024f);
    z[o] = t + c[o];
    e[o] = 2.0 * kEps * (u + 2.0 * fabs(c[o])) * PG_K(1.001) + PG_K(1e-300);
  }
  // m-intervals: lanes 0..2O-1 each evaluate one endpoint (z -/+ e)
  constexpr int kBig = 0x7fffffff;  // below the plateau regime
  int m = kBig;
  bool amb = false;
  if (lane < 2 * O) {
    double zo = z[0], eo = e[0];
#pragma unroll
    for (int o = 1; o < O; ++o)
      if ((lane >> 1) == o) { zo = z[o]; eo = e[o]; }
    const double zz = (lane & 1) ? zo + eo : zo - eo;
    if (zz != zz) {
      amb = true;  // NaN: numpy's NaN rule, in the full path
    } else if (zz >= PG_K(22.2)) {
      double t = pg_exp_f64(-zz);
      t = fma(t, zz * PG_K(5.318237706605891e-17), t);  // pow(e_d, -z) to ~1 ulp (the 1e-6 margin covers it)
      const double vv = t * 4503599627370496.0;   // 2^52 p
      amb = fabs(vv - floor(vv) - 0.5) < PG_K(1e-6);
      m = (int)rint(vv);
    } else if (zz >= 22.0) {
      amb = true;  // too close to the regime edge to compare across it
    }
  }
  if (__ballot(amb)) return -1;
  int mlo[O], mhi[O];  // m(z + e) <= m_np <= m(z - e)
#pragma unroll
  for (int o = 0; o < O; ++o) {
    mhi[o] = __builtin_amdgcn_readlane(m, 2 * o);
    mlo[o] = __builtin_amdgcn_readlane(m, 2 * o + 1);
  }
  // the plateau width above each output's top, lane w for output w: one
  // exp per lane instead of one per (w, o) pair of the test below (their
  // registers spilled on this path)
  double tw[O];
  {
    double top = z[0] + e[0];
#pragma unroll
    for (int o = 1; o < O; ++o)
      if (lane == o) top = z[o] + e[o];
    const double twl = 8.881784197001252e-16 * (pg_exp_f64(fmin(top, 40.0)) + 1.0);  // (2^-50: a literal)
    const uint64_t tb = (uint64_t)__double_as_longlong(twl);
#pragma unroll
    for (int o = 0; o < O; ++o)
      tw[o] = __longlong_as_double((long long)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(tb >> 32), o) << 32) |
                                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)tb, o)));
  }
#pragma unroll
  for (int w = 0; w < O; ++w) {
    bool ok = true;
#pragma unroll
    for (int o = 0; o < O; ++o) {
      if (o == w) continue;
      if (mhi[w] != kBig) {  // w surely in the plateau regime
        ok = ok && (o < w ? mhi[w] < mlo[o] : mhi[w] <= mlo[o]);
      } else {  // S_w below the regime: a strict gap above the plateau width tw[w]
        // and S_w normal (z > -1022 ln 2; S = 0.0 for all z < -709.78, see certify)
        ok = ok && (z[w] - e[w] > z[o] + e[o] + tw[w]) && (z[w] - e[w] > -708.0);
      }
    }
    if (ok) return w;
  }
  return -1;
}

template <int O, typename WT>
__device__ int fast_f64_decide(const WT *__restrict__ g, int H, int b, const int *k, int lane) {
  double x[6];
  f64_features(k, x);
  const int cols = 6 + b;
  const WT *v = g + (long)H * cols;
  double zp[O], c[O];
  float ep[O];
#pragma unroll
  for (int o = 0; o < O; ++o) { zp[o] = 0.0; ep[o] = 0.f; }
#pragma unroll 1
  for (int j = lane; j < H; j += 64) {
    const WT *row = g + (long)j * cols;
    double w1[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) w1[i] = (i < 6 || b) ? (double)row[i] : 0.0;
    double sj, aj;
    f64_unit(x, w1, b, sj, aj);
#pragma unroll
    for (int o = 0; o < O; ++o) {
      const double w2 = (double)v[(long)o * (H + b) + j];
      zp[o] = fma(w2, sj, zp[o]);
      // |w2| aj rounded up to f32 (x 1.00000024 = 1 + 2^-22: above one f32 rounding of each of the two)
      ep[o] = fmaf((float)(fabs(w2) * aj), 1.00000024f, ep[o]);
    }
  }
#pragma unroll
  for (int o = 0; o < O; ++o) c[o] = b ? (double)v[(long)o * (H + b) + H] : 0.0;
  return f64_decide_sums<O>(zp, ep, c, lane);
}

// fast_f64_decide for up to kB requests at once (H <= 64: lane j holds hidden
// unit j of every request): every request's weights are requested before any
// arithmetic, then the kB decisions run as independent chains -- the service
// wave's throughput when requests queue (out[q] = -1 where !need[q]).
template <int O, typename WT, int kB>
__device__ __forceinline__ void fast_f64_decide_batch(const WT *const *g, const int (*k)[6], const bool *need, int H,
                                                      int b, int lane, int *out) {
  const int cols = 6 + b;
  const bool on = lane < H;
  const int j = on ? lane : 0;  // lanes past H read unit 0 and contribute nothing
  double w1[kB][7], w2[kB][O], c[kB][O];
#pragma unroll
  for (int q = 0; q < kB; ++q) {
    if (need[q]) {
      const WT *row = g[q] + (long)j * cols;
      const WT *v = g[q] + (long)H * cols;
#pragma unroll
      for (int i = 0; i < 7; ++i) w1[q][i] = (i < 6 || b) ? (double)row[i] : 0.0;
#pragma unroll
      for (int o = 0; o < O; ++o) {
        w2[q][o] = (double)v[(long)o * (H + b) + j];
        c[q][o] = b ? (double)v[(long)o * (H + b) + H] : 0.0;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kB; ++q) {
    out[q] = -1;
    if (need[q]) {
      double x[6];
      f64_features(k[q], x);
      double sj, aj;
      f64_unit(x, w1[q], b, sj, aj);
      double zp[O];
      float ep[O];
#pragma unroll
      for (int o = 0; o < O; ++o) {
        zp[o] = on ? w2[q][o] * sj : 0.0;
        ep[o] = on ? (float)(fabs(w2[q][o]) * aj) * 1.00000024f : 0.f;
      }
      out[q] = f64_decide_sums<O>(zp, ep, c[q], lane);
    }
  }
}

// the six doubled-centroid features, each in [0, 512), as one 54-bit key
__device__ __forceinline__ uint64_t memo_key(const int k[6]) {
  uint64_t key = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) key = (key << 9) | (uint64_t)(k[i] & 511);
  return key;
}

}  // namespace pg
