#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static inline uint64_t asu64(double x){uint64_t u; memcpy(&u,&x,8); return u;}
static inline double asd(uint64_t u){double x; memcpy(&x,&u,8); return x;}
static inline uint32_t asu32(float x){uint32_t u; memcpy(&u,&x,4); return u;}
static inline float asf(uint32_t u){float x; memcpy(&x,&u,4); return x;}
static const uint64_t T[32] = {
0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51,
0x3fef72b83c7d517b, 0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1,
0x3fef06fe0a31b715, 0x3feef1a7373aa9cb, 0x3feedea64c123422, 0x3feece086061892d,
0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429, 0x3feea47eb03a5585,
0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d,
0x3feee89f995ad3ad, 0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069,
0x3fef5818dcfba487, 0x3fef7c97337b9b5f, 0x3fefa4afa2a490da, 0x3fefd0765b6e4540};
#define N 32
static const double InvLn2N = 0x1.71547652b82fep+0 * N, SHIFT = 0x1.8p+52;
static const double C0 = 0x1.c6af84b912394p-5/N/N/N, C1 = 0x1.ebfce50fac4f3p-3/N/N, C2 = 0x1.62e42ff0c52d6p-1/N;
float my_expf(float x, int usefma) {
  double xd = x;
  uint32_t abstop = (asu32(x) >> 20) & 0x7ff;
  if (abstop >= ((asu32(88.0f) >> 20) & 0x7ff)) {
    if (asu32(x) == asu32(-INFINITY)) return 0.0f;
    if (abstop >= ((asu32(INFINITY) >> 20) & 0x7ff)) return x + x;
    if (x > 0x1.62e42ep6f) return INFINITY;
    if (x < -0x1.9fe368p6f) return 0.0f;
  }
  double z, kd, r, y, s, r2; uint64_t ki, t;
  if (usefma) {
    kd = fma(InvLn2N, xd, SHIFT);
    ki = asu64(kd); kd -= SHIFT;
    r = fma(InvLn2N, xd, -kd);
  } else {
    z = InvLn2N * xd;
    kd = z + SHIFT; ki = asu64(kd); kd -= SHIFT;
    r = z - kd;
  }
  t = T[ki % N]; t += ki << (52 - 5); s = asd(t);
  if (usefma) { z = fma(C0, r, C1); r2 = r*r; y = fma(C2, r, 1.0); y = fma(z, r2, y); }
  else { z = C0*r + C1; r2 = r*r; y = C2*r + 1; y = z*r2 + y; }
  y = y*s;
  return (float)y;
}
int main(int argc, char**argv){
  long n = 0, bad0 = 0, bad1 = 0;
  // sweep all floats in [-104, 0] and [0, 89]
  for (uint32_t u = 0; u < 0x42b20000u; u += (argc>1?1:7)) {
    for (int sgn = 0; sgn < 2; sgn++) {
      float x = asf(u | (sgn ? 0x80000000u : 0));
      if (!(x > -110 && x < 89)) continue;
      float a = expf(x);
      n++;
      if (asu32(a) != asu32(my_expf(x,0))) bad0++;
      if (asu32(a) != asu32(my_expf(x,1))) bad1++;
    }
  }
  printf("expf: n=%ld mismatches nofma=%ld fma=%ld\n", n, bad0, bad1);
  return 0;
}
