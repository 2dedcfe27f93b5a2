// libm_ref.hpp -- device expf / logf that are BIT-IDENTICAL to the host libm the reference links.
//
// The reference runs in float32 and calls the C library's expf/logf (glibc >= 2.27 on Linux: the
// table-driven algorithms of Szabolcs Nagy, evaluated in double and rounded once).  The device's own
// expf/logf are accurate to ~1 ulp but round differently on a sizeable fraction of inputs, and the SW
// direct beam multiplies ~60 such transmittances per column: 1-ulp differences in exp add up to
// ~1e-3 W/m2 in the broadband fluxes.  These functions evaluate the same algorithm with the same
// constants in double precision (gfx950 FP64 FMA is exact IEEE), so the GPU rounds every call exactly
// as the reference does.  Verified bit-for-bit against glibc 2.35 expf on every 7th float in
// (-110, 89) and logf on every 3rd positive finite float (tools/check_libm_ref.c).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rrtmgpnn {

__device__ __forceinline__ double u64_as_f64(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t f64_as_u64(double d) { return (uint64_t)__double_as_longlong(d); }

// exp2f data: tab[i] = bits(2^(i/32)) - (i << 47)
__device__ __constant__ static const uint64_t kExpTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

// tab: the 32-entry table, in LDS in the hot kernels (a per-lane gather from __constant__ memory is a
// vector memory load with L1/L2 latency; from LDS it is a ds_read_b64).
__device__ __forceinline__ float ref_expf_tab(float x, const uint64_t *tab)
{
  const double InvLn2N = 0x1.71547652b82fep+0 * 32, SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
               C2 = 0x1.62e42ff0c52d6p-1 / 32;
  const uint32_t ux = __float_as_uint(x);
  const uint32_t abstop = (ux >> 20) & 0x7ff;
  if (abstop >= 0x42b) {  // |x| >= 88 or nan
    if (ux == 0xff800000u) return 0.0f;
    if (abstop >= 0x7f8) return x + x;
    if (x > 0x1.62e42ep6f) return __int_as_float(0x7f800000);
    if (x < -0x1.9fe368p6f) return 0.0f;
  }
  const double xd = (double)x;
  double kd = __fma_rn(InvLn2N, xd, SHIFT);
  const uint64_t ki = f64_as_u64(kd);
  kd -= SHIFT;
  const double r = __fma_rn(InvLn2N, xd, -kd);
  const double s = u64_as_f64(tab[ki % 32] + (ki << 47));
  const double z = __fma_rn(C0, r, C1), r2 = r * r;
  double y = __fma_rn(C2, r, 1.0);
  y = __fma_rn(z, r2, y);
  return (float)(y * s);
}

__device__ __forceinline__ float ref_expf(float x) { return ref_expf_tab(x, kExpTab); }

// glibc 2.35 cosf (sysdeps/ieee754/flt-32/s_cosf.c with s_sincosf_data.c's table: a pi/2 reduction and double
// polynomials, rounded once), for |y| < 120 -- the SW boundary's mu0 = cos(sza * deg_to_rad) (rrtmgp_rfmip_sw.F90:431-434;
// zenith angles of [0, 180] degrees).  tools/check_libm_ref_cosf.c checks the restatement against the host's cosf on
// every float of [-4, 4] (both of glibc's builds, with and without FMA contraction, give the same bits there).
__device__ __forceinline__ float ref_cosf(float y)
{
  // {c0, c1, c2, c3, c4} of the cosine polynomial, and of its negation for quadrants 2 and 3; s1..s3 of the sine
  constexpr double c[2][5] = {{0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10,
                               0x1.99343027bf8c3p-16},
                              {-0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10,
                               -0x1.99343027bf8c3p-16}};
  constexpr double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
  constexpr double hpi_inv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
  const uint32_t top = (__float_as_uint(y) >> 20) & 0x7ff;
  double x = (double)y;
  int n = 0, q = 0;
  if (top < ((0x3f490fdbu >> 20) & 0x7ff)) {  // |y| < pi/4
    if (top < ((0x39800000u >> 20) & 0x7ff)) return 1.0f;  // |y| < 2^-12
    n = 1;
  } else {
    const double r = x * hpi_inv;
    q = ((int32_t)r + 0x800000) >> 24;
    x = __fma_rn(-(double)q, hpi, x);
    x = (q & 1) == (q & 2) / 2 ? x : -x;  // sign[q & 3] = {1, -1, -1, 1}
    n = q ^ 1;
  }
  const double x2 = x * x;
  const int t = (q & 2) ? 1 : 0;
  if ((n & 1) == 0) {
    const double x3 = x * x2, sa = __fma_rn(x2, s3, s2), x5 = x3 * x2, s = __fma_rn(x3, s1, x);
    return (float)__fma_rn(x5, sa, s);
  }
  const double x4 = x2 * x2, c2 = __fma_rn(x2, c[t][4], c[t][3]), c1 = __fma_rn(x2, c[t][1], c[t][0]), x6 = x4 * x2;
  const double cc = __fma_rn(x4, c[t][2], c1);
  return (float)__fma_rn(x6, c2, cc);
}

// Branch-free form for the solvers' inner loops: the main path is evaluated for every x and glibc's
// over/underflow cases are applied by selection afterwards (x < -0x1.9fe368p6: 0, including -inf;
// x > 0x1.62e42ep6: +inf).  A nan propagates through the main path (glibc returns x + x: also a nan).
// For every other x, including the |x| >= 88 band glibc also sends through the main path, the
// arithmetic is the same as ref_expf_tab's.  No divergent branch, so the scheduler interleaves
// consecutive exps with the surrounding arithmetic.
__device__ __forceinline__ float ref_expf_nb(float x, const uint64_t *tab)
{
  const double InvLn2N = 0x1.71547652b82fep+0 * 32, SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
               C2 = 0x1.62e42ff0c52d6p-1 / 32;
  const double xd = (double)x;
  double kd = __fma_rn(InvLn2N, xd, SHIFT);
  const uint64_t ki = f64_as_u64(kd);
  kd -= SHIFT;
  const double r = __fma_rn(InvLn2N, xd, -kd);
  const double s = u64_as_f64(tab[ki % 32] + (ki << 47));
  const double z = __fma_rn(C0, r, C1), r2 = r * r;
  double y = __fma_rn(C2, r, 1.0);
  y = __fma_rn(z, r2, y);
  float res = (float)(y * s);
  res = (x < -0x1.9fe368p6f) ? 0.0f : res;
  res = (x > 0x1.62e42ep6f) ? __int_as_float(0x7f800000) : res;
  return res;
}

// Correctly rounded sqrtf for normal positive x (the solvers call it on max(., 1e-4)): the hardware
// estimate corrected by one ulp either way, the same steps the compiler emits for sqrtf minus the
// denormal pre-scaling and the zero/inf class test, which never fire in that range.
__device__ __forceinline__ float sqrt_rn_normal(float x)
{
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float em = fmaf(-sm, s, x), ep = fmaf(-sp, s, x);
  float r = (em <= 0.0f) ? sm : s;
  return (ep > 0.0f) ? sp : r;
}

// Correctly rounded 1/b for b in [2^-60, 2^60] (the solvers' denominators: k(1+e^-2k tau)+... and
// 1 - R_dif*albedo): v_rcp_f32, one Newton step and one residual correction -- the compiler's IEEE division
// sequence minus v_div_scale / v_div_fixup (which leave the operands and the result untouched in that range) and
// minus its second correction.  Equal to 1.0f / b on every float of [2^-60, 2^60], checked on the GPU
// (tools/exhaustive_ops.hip; the sequence with both corrections too).
__device__ __forceinline__ float rcp_rn_normal(float b)
{
  float r = __builtin_amdgcn_rcpf(b);
  r = fmaf(fmaf(-b, r, 1.0f), r, r);
  return fmaf(fmaf(-b, r, 1.0f), r, r);
}

// Correctly rounded a / b for operands and quotient in the normal range (|a| >= 2^-100, |b| and |a/b| in
// [2^-126, 2^126]; a == 0 also gives the IEEE result): the compiler's division sequence -- reciprocal, one Newton
// step, quotient, two residual corrections -- without v_div_scale and v_div_fixup, which leave operands and
// result untouched in that range, so the bits are those of a / b (3 of 11 instructions fewer).
__device__ __forceinline__ float div_rn_normal(float a, float b)
{
  float r = __builtin_amdgcn_rcpf(b);
  r = fmaf(fmaf(-b, r, 1.0f), r, r);
  float q = a * r;
  q = fmaf(fmaf(-b, q, a), r, q);
  return fmaf(fmaf(-b, q, a), r, q);
}

// softsign's quotient x / (|x| + 1) (b = |x| + 1): v_rcp_f32 and two residual corrections, without the Newton step
// on the reciprocal, the residual taken as b*q - x so that a -0 quotient keeps its sign.  Equal to x / b on every
// float |x| < 2^126, -0 included, checked on the GPU (tools/exhaustive_ops.hip; div_rn_normal returned +0 for -0).
__device__ __forceinline__ float div_softsign(float x, float b)
{
  const float r = __builtin_amdgcn_rcpf(b);
  float q = x * r;
  q = fmaf(-fmaf(b, q, -x), r, q);
  return fmaf(-fmaf(b, q, -x), r, q);
}

// ref_expf_nb for x <= 0 (the solvers' exp(-tau*D), exp(-tau/mu0), exp(-k*tau) with tau >= 0): only glibc's
// underflow case can occur, so the overflow select is dropped.  For 0 < x <= 0x1.62e42ep6 the main path is
// still glibc's; only a larger x (a negative tau below -88/D) would return a finite value where glibc gives inf.
__device__ __forceinline__ float ref_expf_neg(float x, const uint64_t *tab)
{
  const double InvLn2N = 0x1.71547652b82fep+0 * 32, SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
               C2 = 0x1.62e42ff0c52d6p-1 / 32;
  const double xd = (double)x;
  double kd = __fma_rn(InvLn2N, xd, SHIFT);
  const uint64_t ki = f64_as_u64(kd);
  kd -= SHIFT;
  const double r = __fma_rn(InvLn2N, xd, -kd);
  const double s = u64_as_f64(tab[ki % 32] + (ki << 47));
  const double z = __fma_rn(C0, r, C1), r2 = r * r;
  double y = __fma_rn(C2, r, 1.0);
  y = __fma_rn(z, r2, y);
  const float res = (float)(y * s);
  return (x < -0x1.9fe368p6f) ? 0.0f : res;
}

// ref_expf_neg of M values with the M table reads issued back to back: the same operations per value, so the same bits,
// but one LDS latency for the batch instead of one per exp (the compiler otherwise waits on each read as it is issued)
template <int M>
__device__ __forceinline__ void ref_expf_neg_batch(const float *x, float *y, const uint64_t *tab)
{
  const double InvLn2N = 0x1.71547652b82fep+0 * 32, SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
               C2 = 0x1.62e42ff0c52d6p-1 / 32;
  double r[M];
  uint64_t ki[M], t[M];
#pragma unroll
  for (int i = 0; i < M; i++) {
    const double xd = (double)x[i];
    double kd = __fma_rn(InvLn2N, xd, SHIFT);
    ki[i] = f64_as_u64(kd);
    kd -= SHIFT;
    r[i] = __fma_rn(InvLn2N, xd, -kd);
  }
  __builtin_amdgcn_sched_barrier(0);  // the M table reads issue together (scheduled apart otherwise, each waited on)
#pragma unroll
  for (int i = 0; i < M; i++) t[i] = tab[ki[i] % 32];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < M; i++) {
    const double s = u64_as_f64(t[i] + (ki[i] << 47));
    const double z = __fma_rn(C0, r[i], C1), r2 = r[i] * r[i];
    double yy = __fma_rn(C2, r[i], 1.0);
    yy = __fma_rn(z, r2, yy);
    const float res = (float)(yy * s);
    y[i] = (x[i] < -0x1.9fe368p6f) ? 0.0f : res;
  }
}

// Copy the exp table into LDS (call with all threads of the block; a __syncthreads() must follow).
__device__ __forceinline__ void load_exp_table(uint64_t *lds_tab)
{
  for (int i = threadIdx.x; i < 32; i += blockDim.x) lds_tab[i] = kExpTab[i];
}

struct LogTab {
  double invc, logc;
};
__device__ __constant__ static const LogTab kLogTab[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611ccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};

__device__ __forceinline__ float ref_logf(float x)
{
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  uint32_t ix = __float_as_uint(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return __int_as_float(0xff800000);       // -inf
    if (ix == 0x7f800000u) return x;                          // +inf
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __int_as_float(0x7fc00000);  // nan
    ix = __float_as_uint(x * 0x1p23f);                        // subnormal: normalise
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16);
  const int k = (int)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const double invc = kLogTab[i].invc, logc = kLogTab[i].logc;
  const double z = (double)__uint_as_float(iz);
  const double r = __fma_rn(z, invc, -1.0);
  const double y0 = __fma_rn((double)k, Ln2, logc);
  const double r2 = r * r;
  double y = __fma_rn(A1, r, A2);
  y = __fma_rn(A0, r2, y);
  y = __fma_rn(y, r2, y0 + r);
  return (float)y;
}

// ref_logf without branches (the fused MLP kernel's input scaling, where a branch would split the tile body): glibc's
// main path on the (normalised) argument, the special cases selected afterwards.  Same result as ref_logf for every
// input.
__device__ __forceinline__ float ref_logf_nb(float x)
{
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  const uint32_t ix0 = __float_as_uint(x);
  const bool special = ix0 - 0x00800000u >= 0x7f800000u - 0x00800000u;
  // a positive subnormal is normalised as glibc does; other specials take the main path on a harmless value
  const uint32_t ixs = __float_as_uint(x * 0x1p23f) - (23u << 23);
  const bool subn = special && !(ix0 & 0x80000000u) && ix0 * 2 != 0 && ix0 < 0x00800000u;
  const uint32_t ix = subn ? ixs : (special ? 0x3f800000u : ix0);
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16);
  const int k = (int)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const double invc = kLogTab[i].invc, logc = kLogTab[i].logc;
  const double z = (double)__uint_as_float(iz);
  const double r = __fma_rn(z, invc, -1.0);
  const double y0 = __fma_rn((double)k, Ln2, logc);
  const double r2 = r * r;
  double y = __fma_rn(A1, r, A2);
  y = __fma_rn(A0, r2, y);
  y = __fma_rn(y, r2, y0 + r);
  float res = (float)y;
  res = ix0 == 0x3f800000u ? 0.0f : res;
  const float sp = ix0 * 2 == 0 ? __int_as_float(0xff800000)
                   : ix0 == 0x7f800000u ? x
                   : ((ix0 & 0x80000000u) || ix0 * 2 >= 0xff000000u) ? __int_as_float(0x7fc00000)
                                                                      : res;
  return special && !subn ? sp : res;
}

}  // namespace rrtmgpnn
