// pg_f64math.h -- a compact f64 sigmoid for the rare f64 re-decision path.
//
// numpy_nn's sigmoid is 1 / (1 + np.e ** -z) (numpy_nn.py:22-23), i.e. libm
// pow(e_d, -z) with e_d the double nearest e.  pow(e_d, -z) =
// exp(-z ln e_d) = exp(-z) * exp(z * delta), delta = 1 - ln(e_d)
// = 5.318237706605891e-17, and |z delta| < 4e-14 on exp's range, so
// exp(z delta) = 1 + z delta to f64 precision.  exp is Cody-Waite reduced
// (n = rint(x log2 e), r = x - n ln2) and a degree-13 Taylor polynomial on
// |r| <= ln2/2 (truncation < 2^-60), then scaled by 2^n: about 1 ulp, with a
// small register footprint (the library pow costs ~60 VGPRs inline).
// Plain C/C++: compiled into the HIP library and, for the accuracy test, on
// the host (tests/test_f64math.py).
#ifndef PG_F64MATH_H
#define PG_F64MATH_H

#if defined(__HIPCC__)
#define PG_HD __host__ __device__ inline
#else
#define PG_HD static inline
#endif

#include <math.h>

PG_HD double pg_exp_f64(double x) {
  if (x > 709.782712893384) return INFINITY;
  if (x < -745.1332191019412) return 0.0;
  const double n = rint(x * 1.4426950408889634);
  const double r = fma(-n, 1.9082149292705877e-10, fma(-n, 6.93147180369123816490e-01, x));
  double p = 1.6059043836821613e-10;   /* 1/13! */
  p = fma(p, r, 2.08767569878681e-09);  /* 1/12! */
  p = fma(p, r, 2.505210838544172e-08); /* 1/11! */
  p = fma(p, r, 2.755731922398589e-07); /* 1/10! */
  p = fma(p, r, 2.7557319223985893e-06);
  p = fma(p, r, 2.48015873015873e-05);
  p = fma(p, r, 1.984126984126984e-04);
  p = fma(p, r, 1.388888888888889e-03);
  p = fma(p, r, 8.333333333333333e-03);
  p = fma(p, r, 4.1666666666666664e-02);
  p = fma(p, r, 1.6666666666666666e-01);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)n);
}

/* 1 / (1 + pow(np.e, -z)) */
PG_HD double pg_sigmoid_f64(double z) {
  double t = pg_exp_f64(-z);
  if (t < INFINITY) t = fma(t, z * 5.318237706605891e-17, t);  /* inf * (1 + tiny) stays inf */
  return 1.0 / (1.0 + t);
}

#endif
