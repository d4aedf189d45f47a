/*
 * cvr_detmath.h - deterministic float32 math shared by the gfx950 kernels and
 * the CPU oracle.
 *
 * Why this exists: a volumetric random walk is a chaotic function of its
 * inputs.  One ulp of difference in a logf() flips a Woodcock acceptance test
 * and the path takes a different route.  CUDA's libdevice (what the reference,
 * implementation/src/Utilities.cuh:134-136, HG.h:25-26, GGX.h:95-157, links),
 * AMD's ocml and glibc all round differently in the last ulp, so the only way
 * to make a HIP path bit-identical to its CPU restatement is to evaluate the
 * transcendental functions with the same sequence of correctly-rounded IEEE
 * operations on both sides.  Everything below uses only +,-,*,/, sqrtf, floorf
 * and explicit fmaf (all correctly rounded on x86-64 and on CDNA4), so the
 * result is bit-identical on host and device as long as both are compiled with
 * -ffp-contract=off (no implicit FMA contraction).
 *
 * Accuracy (asserted by tests/test_detmath.py against double libm):
 *   det_logf  <= 2 ulp on [FLT_MIN, FLT_MAX]
 *   det_sinf/det_cosf <= 2 ulp on [-8pi, 8pi]
 *   det_tanf  <= 3 ulp on [0, pi/2)
 *   det_acosf <= 2 ulp, det_atan2f <= 3 ulp
 * Coefficients: tools/fit_detmath.py.
 *
 * This header is plain C99 for the oracle and HIP C++ for the kernels.
 */
#ifndef CVR_DETMATH_H_
#define CVR_DETMATH_H_

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define CVR_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define CVR_HD static inline
#endif

#define CVR_PI_F 3.1415926535897932384626422832795028841971f  /* Defines.h:59 */
#define CVR_TWOPI_F 6.2831853071795864769252867665590057683943f /* Defines.h:60 */
#define CVR_EPSILON_F 0.00001f                                /* Defines.h:61 */

CVR_HD float det_fmaf(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

CVR_HD uint32_t det_f2u(float x) {
  union { float f; uint32_t u; } v;
  v.f = x;
  return v.u;
}
CVR_HD float det_u2f(uint32_t x) {
  union { float f; uint32_t u; } v;
  v.u = x;
  return v.f;
}

/* IEEE minNum/maxNum as CUDA's fminf/fmaxf (one NaN operand -> the other);
 * signed zeros resolve to the first operand on both targets. */
CVR_HD float det_fminf(float a, float b) { return (a != a) ? b : ((b < a) ? b : a); }
CVR_HD float det_fmaxf(float a, float b) { return (a != a) ? b : ((b > a) ? b : a); }
CVR_HD float det_fabsf(float a) { return det_u2f(det_f2u(a) & 0x7fffffffu); }
CVR_HD float det_sqrtf(float a) { return __builtin_sqrtf(a); }
CVR_HD float det_floorf(float a) { return __builtin_floorf(a); }

/* (int)floorf(x) with a defined result everywhere, branch-free: saturating,
 * NaN -> INT_MIN (det_fmaxf returns the non-NaN operand). */
CVR_HD int det_floor_i32(float x) {
  float f = det_fminf(det_fmaxf(__builtin_floorf(x), -2147483648.0f), 2147483520.0f);
  return (int)f;
}

/* ---------------------------------------------------------------- log --- */
CVR_HD float det_logf_core(uint32_t ix, int k) {
  /* reduce x into [sqrt(2)/2, sqrt(2)) */
  ix += 0x3f800000u - 0x3f3504f3u;
  k += (int)(ix >> 23) - 0x7f;
  ix = (ix & 0x007fffffu) + 0x3f3504f3u;
  float f = det_u2f(ix) - 1.0f;
  float p = -0.07362867891788483f;
  p = det_fmaf(p, f, 0.1262032687664032f);
  p = det_fmaf(p, f, -0.13202103972434998f);
  p = det_fmaf(p, f, 0.14227114617824554f);
  p = det_fmaf(p, f, -0.16621370613574982f);
  p = det_fmaf(p, f, 0.19999825954437256f);
  p = det_fmaf(p, f, -0.2500085234642029f);
  p = det_fmaf(p, f, 0.3333335518836975f);
  float f2 = f * f;
  float r = (f2 * f) * p;
  float hfsq = 0.5f * f2;
  float dk = (float)k;
  float y = det_fmaf(dk, 9.058001523953862e-06f, r - hfsq);
  y = y + f;
  return det_fmaf(dk, 0.6931381225585938f, y);
}
/* log(x) for x > 0 (normal or subnormal). */
CVR_HD float det_logf(float x) {
  uint32_t ix = det_f2u(x);
  int k = 0;
  if (ix < 0x00800000u) { /* subnormal: scale by 2^25 */
    ix = det_f2u(x * 33554432.0f);
    k = -25;
  }
  return det_logf_core(ix, k);
}
/* Same result as det_logf for normal x > 0. */
CVR_HD float det_logf_normal(float x) { return det_logf_core(det_f2u(x), 0); }

/* ------------------------------------------------------------ sin/cos --- */
CVR_HD float det_sin_poly(float r, float z) {
  float s = 2.7180080905964132e-06f;
  s = det_fmaf(s, z, -0.0001983929832931608f);
  s = det_fmaf(s, z, 0.008333329111337662f);
  s = det_fmaf(s, z, -0.1666666716337204f);
  return det_fmaf(r * z, s, r);
}
CVR_HD float det_cos_poly(float z) {
  float c = -2.720371981013159e-07f;
  c = det_fmaf(c, z, 2.4799432139843702e-05f);
  c = det_fmaf(c, z, -0.0013888883404433727f);
  c = det_fmaf(c, z, 0.0416666679084301f);
  return det_fmaf(z * z, c, det_fmaf(-0.5f, z, 1.0f));
}
/* Cody-Waite reduction by pi/2 (3-term split; exact enough for |x| < 2^10). */
CVR_HD float det_reduce_pio2(float x, int* q) {
  float kf = __builtin_floorf(det_fmaf(x, 0.6366197466850281f, 0.5f));
  float r = det_fmaf(-kf, 1.5707963705062866f, x);
  r = det_fmaf(-kf, -4.371138828673793e-08f, r);
  r = det_fmaf(-kf, -1.7763568394002505e-15f, r);
  *q = ((int)kf) & 3;
  return r;
}
CVR_HD void det_sincosf(float x, float* sp, float* cp) {
  int q;
  float r = det_reduce_pio2(x, &q);
  float z = r * r;
  float s = det_sin_poly(r, z);
  float c = det_cos_poly(z);
  float so, co;
  if (q == 0) { so = s; co = c; }
  else if (q == 1) { so = c; co = -s; }
  else if (q == 2) { so = -s; co = -c; }
  else { so = -c; co = s; }
  *sp = so;
  *cp = co;
}
CVR_HD float det_sinf(float x) { float s, c; det_sincosf(x, &s, &c); return s; }
CVR_HD float det_cosf(float x) { float s, c; det_sincosf(x, &s, &c); return c; }
CVR_HD float det_tanf(float x) {
  int q;
  float r = det_reduce_pio2(x, &q);
  float z = r * r;
  float s = det_sin_poly(r, z);
  float c = det_cos_poly(z);
  return (q & 1) ? (-c / s) : (s / c);
}

/* ---------------------------------------------------------- asin/acos --- */
CVR_HD float det_asin_poly(float x, float z) { /* x + x^3 A(x^2), |x| <= 0.5 */
  float a = 0.03744102641940117f;
  a = det_fmaf(a, z, 0.014491950161755085f);
  a = det_fmaf(a, z, 0.031793925911188126f);
  a = det_fmaf(a, z, 0.044518522918224335f);
  a = det_fmaf(a, z, 0.07500497251749039f);
  a = det_fmaf(a, z, 0.16666659712791443f);
  return det_fmaf(x * z, a, x);
}
/* Three ranges, evaluated branch-free (one polynomial, selected inputs):
 *   |x| <= 0.5: pi/2 - asin(x)
 *   x > 0.5:    2 asin(sqrt((1 - x)/2))
 *   x < -0.5:   2 (pi/2 - asin(sqrt((1 + x)/2)))
 * (GGX lanes straddle the ranges, so branches would run all of them.) */
CVR_HD float det_acosf(float x) {
  const float pio2_hi = 1.5707963705062866f, pio2_lo = -4.371138828673793e-08f;
  const int mid = det_fabsf(x) <= 0.5f;
  const float zo = (x > 0.0f ? 1.0f - x : 1.0f + x) * 0.5f;
  const float z = mid ? x * x : zo;
  const float so = det_sqrtf(zo);
  const float as = det_asin_poly(mid ? x : so, z);
  const float r = mid ? pio2_hi - (as - pio2_lo) : (x > 0.0f ? 2.0f * as : 2.0f * (pio2_hi - (as - pio2_lo)));
  return (x >= -1.0f && x <= 1.0f) ? r : __builtin_nanf("");
}

/* -------------------------------------------------------------- atan2 --- */
CVR_HD float det_atan_poly(float a) { /* atan(a), 0 <= a <= 1 */
  float z = a * a;
  float t = 0.001083198469132185f;
  t = det_fmaf(t, z, -0.007164361421018839f);
  t = det_fmaf(t, z, 0.022212041541934013f);
  t = det_fmaf(t, z, -0.044302549213171005f);
  t = det_fmaf(t, z, 0.0671394020318985f);
  t = det_fmaf(t, z, -0.08798883110284805f);
  t = det_fmaf(t, z, 0.11054951697587967f);
  t = det_fmaf(t, z, -0.14279332756996155f);
  t = det_fmaf(t, z, 0.19999633729457855f);
  t = det_fmaf(t, z, -0.33333325386047363f);
  return det_fmaf(a * z, t, a);
}
CVR_HD float det_atan2f(float y, float x) {
  const float pio2_hi = 1.5707963705062866f, pio2_lo = -4.371138828673793e-08f;
  const float pi_hi = 3.1415927410125732f, pi_lo = -8.742277657347586e-08f;
  float ax = det_fabsf(x), ay = det_fabsf(y);
  float mx = ay > ax ? ay : ax;
  float mn = ay > ax ? ax : ay;
  float t = (mx == 0.0f) ? 0.0f : det_atan_poly(mn / mx);
  if (ay > ax) t = pio2_hi - (t - pio2_lo);
  if (x < 0.0f) t = pi_hi - (t - pi_lo);
  if (det_f2u(y) >> 31) t = -t;
  return t;
}

#endif /* CVR_DETMATH_H_ */
