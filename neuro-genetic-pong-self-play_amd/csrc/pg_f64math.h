// pg_f64math.h -- numpy's sigmoid in f64 for the f64 paths (k_general,
// k_wide, the f32 path's f64 re-decisions), plus a compact exp for bounds.
//
// numpy_nn's sigmoid is 1 / (1 + np.e ** -z) (numpy_nn.py:22-23): pow(e_d, -z)
// with e_d the double nearest e, then an IEEE add and divide.  pow(e_d, -z) =
// exp(-z ln e_d) = exp(-z + z delta), delta = 1 - ln(e_d) = 5.318237706605891e-17.
// pg_pow_e_neg evaluates it to ~2^-67 relative before the one final rounding
// (table 2^(j/64) in double-double, |r| <= ln2/128, degree-7 polynomial, the
// tail carried as a double-double), so it returns the correctly rounded value
// except when the exact one lies within ~2^-67 of a rounding boundary.  numpy's
// own pow is not correctly rounded and is platform-specific (SVML's AVX-512
// pow on AVX-512 hosts, libm's pow elsewhere; they disagree in ~5 % of values
// by 1 ulp): no f64 sigmoid matches every numpy bit for bit; this one matches
// the correctly rounded value (tests/test_f64math.py measures all three).
// Plain C/C++: compiled into the HIP library and, for the accuracy test, on the
// host.
#ifndef PG_F64MATH_H
#define PG_F64MATH_H

#if defined(__HIPCC__)
#define PG_HD __host__ __device__ inline
#define PG_TABLE static constexpr
#else
#define PG_HD static inline
#define PG_TABLE static const
#endif

#include <math.h>

/* PG_K(c): an f64 constant of the f64 decision code.  On the device it is
 * materialized where it is used (its bits plus an opaque zero that a volatile
 * asm makes there, which no pass hoists): k_service's game loop runs this code in its rare decision
 * path, and plain constants were hoisted out of the loop into registers that
 * the allocator then spilled to scratch -- each use a dependent scratch load
 * inside the decision (tools/isa_frame.py).  Elsewhere (host) the constant. */
#if defined(__HIP_DEVICE_COMPILE__) && !defined(PG_NO_K)  /* PG_NO_K: plain constants (A/B) */
template <unsigned long long B>
__device__ __forceinline__ double pg_k64() {
  unsigned long long zero;  // an opaque 0 made here: B + 0 is not loop-invariant
  asm volatile("s_mov_b64 %0, 0" : "=s"(zero));
  return __builtin_bit_cast(double, B + zero);
}
#define PG_K(c) (pg_k64<__builtin_bit_cast(unsigned long long, (double)(c))>())
#else
#define PG_K(c) (c)
#endif

/* 2^(j/64), j = 0..63, as hi + lo (hi the nearest double, |lo| < ulp(hi)/2) */
PG_TABLE double kPgExp2Tbl[128] = {
    1.0, 0.0,
    1.0108892860517005, -1.5234778603368577e-17,
    1.0218971486541166, 5.109225028973444e-17,
    1.0330248790212284, 7.600838874027088e-18,
    1.0442737824274138, 8.551889705537965e-17,
    1.0556451783605572, 1.759325738772092e-18,
    1.0671404006768237, -7.899853966841582e-17,
    1.0787607977571199, -6.656660436056593e-17,
    1.0905077326652577, -3.046782079812471e-17,
    1.102382583307841, 5.2660368715706944e-17,
    1.1143867425958924, 1.0410278456845571e-16,
    1.1265216186082418, 5.165856758795457e-17,
    1.1387886347566916, 8.912812676025408e-17,
    1.1511892299529827, 3.250710218863827e-17,
    1.1637248587775775, 3.8292048369240935e-17,
    1.1763969916502812, 5.554203254218079e-17,
    1.189207115002721, 3.982015231465646e-17,
    1.202156731452703, 6.644981499252301e-17,
    1.215247359980469, -7.712630692681488e-17,
    1.22848053610687, -1.89878163130253e-17,
    1.241857812073484, 4.658027591836937e-17,
    1.255380757024691, -6.7113898212968784e-18,
    1.2690509571917332, 2.667932131342186e-18,
    1.2828700160787783, 1.713594918243561e-17,
    1.2968395546510096, 2.5382502794888315e-17,
    1.3109612115247644, -7.181536135519454e-17,
    1.3252366431597413, -2.8587312100388614e-17,
    1.339667524053303, 8.927282594831732e-17,
    1.3542555469368927, 7.70094837980299e-17,
    1.3690024229745905, 9.593797919118849e-17,
    1.383909881963832, -6.770511658794786e-17,
    1.3989796725383112, -9.614213209051323e-17,
    1.4142135623730951, -9.667293313452913e-17,
    1.42961333839197, -1.2031642489053655e-17,
    1.4451808069770467, -3.0237581349939873e-17,
    1.460917794180647, -5.600377186075216e-17,
    1.4768261459394993, -3.483994556892796e-17,
    1.4929077282912648, 1.4192920154284036e-17,
    1.5091644275934228, -1.016455327754295e-16,
    1.5255981507445384, -1.1024941712342561e-16,
    1.5422108254079407, 7.949834809697621e-17,
    1.559004400237837, 3.7812070533575275e-17,
    1.5759808451078865, -1.0136916471278304e-17,
    1.593142151342267, -1.0094406542311964e-16,
    1.6104903319492543, 2.4707192569797888e-17,
    1.6280274218573478, -6.712955084707084e-17,
    1.645755478153965, -1.0125679913674773e-16,
    1.6636765803267364, 5.8909926967131e-17,
    1.681792830507429, 8.199010020581497e-17,
    1.7001063537185235, -8.0237193703977e-18,
    1.718619298122478, -1.851380418263111e-17,
    1.7373338352737062, 3.164389299292957e-17,
    1.7562521603732995, 2.960140695448873e-17,
    1.7753764925265212, 6.429731796556572e-17,
    1.7947090750031072, 1.8227458427912087e-17,
    1.8142521755003989, -9.969531538920349e-17,
    1.8340080864093424, 3.283107224245627e-17,
    1.8539791250833855, 9.761887490727594e-17,
    1.8741676341103, -6.122763413004143e-17,
    1.8945759815869656, 3.4034035352165297e-17,
    1.9152065613971474, -1.0619946056195963e-16,
    1.9360617934922943, 1.0332385960676326e-16,
    1.9571441241754002, 8.960767791036668e-17,
    1.978456026387951, 4.0388753109278167e-17,
};

/* pow(e_d, -z), e_d = np.e */
PG_HD double pg_pow_e_neg(double z) {
  if (z != z) return z;
  if (-z > PG_K(709.782712893384)) return INFINITY;
  if (-z < PG_K(-745.1332191019412)) return 0.0;
  const double kInvL = PG_K(92.33248261689366);            /* 64 / ln 2 */
  const double kLhi = PG_K(0.010830424696223417);          /* ln2/64, 36 significant bits: n * kLhi exact */
  const double kLlo = PG_K(2.572804622327669e-14);         /* ln2/64 - kLhi */
  const double kDelta = PG_K(5.318237706605891e-17);       /* 1 - ln(e_d) */
  const double n = rint(-z * kInvL);
  const double r_hi = fma(-n, kLhi, -z);             /* exact: -z - n kLhi */
  const double r_lo = fma(-n, kLlo, z * kDelta);
  /* (r, re) = two_sum(r_hi, r_lo): r + re = r_hi + r_lo exactly */
  const double r = r_hi + r_lo;
  const double bb = r - r_hi;
  const double re = (r_hi - (r - bb)) + (r_lo - bb);
  /* exp(r + re) = 1 + r + q_lo, q_lo = r^2 P(r) + re (1 + r) */
  double pp = PG_K(1.984126984126984e-04);                 /* 1/5040 */
  pp = fma(pp, r, PG_K(1.388888888888889e-03));            /* 1/720 */
  pp = fma(pp, r, PG_K(8.333333333333333e-03));            /* 1/120 */
  pp = fma(pp, r, PG_K(4.1666666666666664e-02));           /* 1/24 */
  pp = fma(pp, r, PG_K(1.6666666666666666e-01));           /* 1/6 */
  pp = fma(pp, r, 0.5);
  const double q_lo = fma(r * r, pp, re * (1.0 + r));
  const int ni = (int)n;
  const int j = ni & 63;
  const double t_hi = kPgExp2Tbl[2 * j], t_lo = kPgExp2Tbl[2 * j + 1];
  /* T (1 + q) = t_hi + t_hi r + (t_hi q_lo + t_lo (1 + r)) */
  const double a_hi = t_hi * r;
  const double a_lo = fma(t_hi, r, -a_hi);
  const double s_hi = t_hi + a_hi;
  const double sb = s_hi - t_hi;
  const double s_lo = (t_hi - (s_hi - sb)) + (a_hi - sb);
  const double tail = s_lo + (a_lo + fma(t_hi, q_lo, t_lo * (1.0 + r)));
  return ldexp(s_hi + tail, ni >> 6);
}

/* numpy_nn.sigmoid: 1 / (1 + np.e ** -z) */
PG_HD double pg_sigmoid_f64(double z) {
  const double t = pg_pow_e_neg(z);
  return 1.0 / (1.0 + t);
}

/* exp(x) to about 1 ulp, small register footprint (error bounds, plateau tests) */
PG_HD double pg_exp_f64(double x) {
  if (x > PG_K(709.782712893384)) return INFINITY;
  if (x < PG_K(-745.1332191019412)) return 0.0;
  const double n = rint(x * PG_K(1.4426950408889634));
  const double r = fma(-n, PG_K(1.9082149292705877e-10), fma(-n, PG_K(6.93147180369123816490e-01), x));
  double p = PG_K(1.6059043836821613e-10);   /* 1/13! */
  p = fma(p, r, PG_K(2.08767569878681e-09));  /* 1/12! */
  p = fma(p, r, PG_K(2.505210838544172e-08)); /* 1/11! */
  p = fma(p, r, PG_K(2.755731922398589e-07)); /* 1/10! */
  p = fma(p, r, PG_K(2.7557319223985893e-06));
  p = fma(p, r, PG_K(2.48015873015873e-05));
  p = fma(p, r, PG_K(1.984126984126984e-04));
  p = fma(p, r, PG_K(1.388888888888889e-03));
  p = fma(p, r, PG_K(8.333333333333333e-03));
  p = fma(p, r, PG_K(4.1666666666666664e-02));
  p = fma(p, r, PG_K(1.6666666666666666e-01));
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)n);
}

#endif
