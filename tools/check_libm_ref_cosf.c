// check_libm_ref_cosf.c -- the glibc 2.35 cosf algorithm (sysdeps/ieee754/flt-32/s_cosf.c, s_sincosf_data.c and
// sincosf.h: double-precision polynomials after a pi/2 reduction), restated for the SW boundary kernel's mu0
// (csrc/libm_ref.hpp ref_cosf), checked against the host's libm cosf on every float of [-4, 4] (argv[1] = stride).
// The reference driver forms mu0 = cos(sza * deg_to_rad) in working precision (rrtmgp_rfmip_sw.F90:431-434); with the
// reference built here (amdflang + glibc) that is libm's cosf.  glibc dispatches an FMA build of the same source on
// FMA hardware; both forms are checked.
//   gcc -O2 -ffp-contract=off -o /tmp/cosf tools/check_libm_ref_cosf.c -lm && /tmp/cosf 1
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint32_t asu32(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static inline float asf(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static inline uint32_t abstop12(float x) { return (asu32(x) >> 20) & 0x7ff; }

typedef struct { double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; } sincos_t;
static const sincos_t T[2] = {
  {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
   0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
   0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
  {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
   -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
   0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};

static float poly(double x, double x2, const sincos_t *p, int n, int f)
{
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = f ? fma(x2, p->s3, p->s2) : p->s2 + x2 * p->s3;
    double x5 = x3 * x2;
    double s = f ? fma(x3, p->s1, x) : x + x3 * p->s1;
    return (float)(f ? fma(x5, s1, s) : s + x5 * s1);
  }
  double x4 = x2 * x2;
  double c2 = f ? fma(x2, p->c4, p->c3) : p->c3 + x2 * p->c4;
  double c1 = f ? fma(x2, p->c1, p->c0) : p->c0 + x2 * p->c1;
  double x6 = x4 * x2;
  double c = f ? fma(x4, p->c2, c1) : c1 + x4 * p->c2;
  return (float)(f ? fma(x6, c2, c) : c + x6 * c2);
}

// |y| < 120 (the path the driver's zenith angles take); f: the FMA build
static float my_cosf(float y, int f)
{
  double x = y;
  const sincos_t *p = &T[0];
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return poly(x, x * x, p, 1, f);
  }
  double r = x * p->hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  x = f ? fma(-(double)n, p->hpi, x) : x - n * p->hpi;
  double s = p->sign[n & 3];
  if (n & 2) p = &T[1];
  return poly(x * s, x * x, p, n ^ 1, f);
}

int main(int argc, char **argv)
{
  const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 13;
  long n = 0, bad0 = 0, bad1 = 0;
  for (uint32_t u = 0; u <= asu32(4.0f); u += stride)
    for (int sgn = 0; sgn < 2; sgn++) {
      const float x = asf(u | (sgn ? 0x80000000u : 0u));
      const float a = cosf(x);
      n++;
      bad0 += asu32(a) != asu32(my_cosf(x, 0));
      bad1 += asu32(a) != asu32(my_cosf(x, 1));
    }
  printf("cosf on [-4, 4] (stride %u): n=%ld mismatches nofma=%ld fma=%ld\n", stride, n, bad0, bad1);
  return bad1 == 0 || bad0 == 0 ? 0 : 1;
}
