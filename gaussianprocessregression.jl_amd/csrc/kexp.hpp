// exp(-dist) scaled by a part's sigma^2 via an LDS table: shared by the K-assembly kernels
// (assembly.hip) and the fused MLL gradient (mll.hip), so both evaluate the kernel with the
// same ~1-ulp exponential.
#pragma once
#include <hip/hip_runtime.h>

#ifndef GPR_EXP32  // 1: 32-entry exp tables (conflict-free LDS gathers, 2 more FMAs)
#define GPR_EXP32 0
#endif
// Tang's reduction with x = -dist (already in range): kf = x 256/ln2 + 1.5 2^52 holds
// n = rint(x 256/ln2) in its low word (magic-constant rounding: no rndne / cvt), r = x -
// n ln2/256 in two Cody-Waite steps, a degree-4 expm1 (truncation < 0.2 ulp), exp(x) =
// 2^(n >> 8) T[n & 255] (1 + expm1(r)) with sigma^2 folded into the table (one rounding of
// s2 * T[j]).
static __device__ __forceinline__ double kexp_core(double x, const double* ts) {
  const double kf = fma(x, 369.3299304675746, 6755399441055744.0);
  const double nf = kf - 6755399441055744.0;
  double r = fma(nf, -0.00270760617331689, x);
  r = fma(nf, -7.453964567463233e-13, r);
  const int ni = (int)(unsigned)__double_as_longlong(kf);
  double p = fma(r, 0.041666666666666664, 0.16666666666666666);
  p = fma(r, p, 0.5);
  p = r * p;
  const double q = fma(r, p, r);  // expm1(r)
  const double t = ts[ni & 255];
  return __builtin_ldexp(fma(t, q, t), ni >> 8);
}

// s2 * exp(-dist) with the part's table ts[j] = s2 * 2^(j/256): x = -dist clamped at -800 (exp
// underflows to 0 long before; a NaN dist fails the compare and propagates).  16 VALU + 1 LDS
// read per element.
static __device__ __forceinline__ double kexp_s2(double dist, const double* ts) {
#ifdef GPR_KBUILD_NOEXP
  return ts[0] * fma(dist, -1e-3, 1.0);
#elif GPR_EXP32
  // 32-entry table 2^(j/32) (every entry in its own LDS bank pair: conflict-free gathers),
  // |r| <= ln2/64, degree-6 expm1 (truncation < 0.03 ulp); tab[j] = ts[8 j]
  const double x = dist > 800.0 ? -800.0 : -dist;
  const double kf = fma(x, 46.16624130844683, 6755399441055744.0);
  const double nf = kf - 6755399441055744.0;
  double r = fma(nf, -0.02166084938653512, x);  // ln2/32 = L1 (32 bits) + L2
  r = fma(nf, -5.9631716539705866e-12, r);
  const int ni = (int)(unsigned)__double_as_longlong(kf);
  double p = fma(r, 1.3888888888888889e-03, 8.3333333333333332e-03);
  p = fma(r, p, 0.041666666666666664);
  p = fma(r, p, 0.16666666666666666);
  p = fma(r, p, 0.5);
  p = r * p;
  const double q = fma(r, p, r);
  const double t = ts[ni & 31];
  return __builtin_ldexp(fma(t, q, t), ni >> 5);
#else
  return kexp_core(dist > 800.0 ? -800.0 : -dist, ts);
#endif
}

// the same without the clamp (3 VALU fewer), for callers that have bounded dist < 5.8e6, so
// that n fits the int32 low word: below -745 the ldexp underflows to 0 as in the clamped form,
// and a NaN propagates
static __device__ __forceinline__ double kexp_s2_nc(double dist, const double* ts) {
#if defined(GPR_KBUILD_NOEXP) || GPR_EXP32
  return kexp_s2(dist, ts);
#else
  return kexp_core(-dist, ts);
#endif
}
