// exhaustive_ops.hip -- checks shorter correctly-rounded sequences for the solvers' and MLPs' 1-argument operations
// against IEEE results on EVERY float of the domain, on the GPU itself (v_rcp_f32 / v_sqrt_f32 / v_sqrt_f64 are
// hardware approximations that a host cannot emulate bit for bit).  Test tool, not product code.
//
//   rcp  : 1/b, b in [2^-60, 2^60]       current rcp_rn_normal (Newton + 2 corrections) vs candidates
//   sqrt : sqrtf(x), x in [2^-20, 2^20]  current sqrt_rn_normal vs (float)v_sqrt_f64((double)x)
//   soft : x/(|x|+1), every finite x     current div_rn_normal vs the division without the Newton step (and with the
//                                        residual negated, which keeps the sign of a -0 quotient)
//
// reference: the compiler's IEEE sequences (default flags: correctly rounded f32 division and sqrt), cross-checked
// with double-precision evaluations rounded once (innocuous double rounding for / and sqrt).
// Output: one line per (op, variant): mismatches against the reference and the first mismatching input.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

__device__ __forceinline__ float rcp_cur(float b)
{
  float r = __builtin_amdgcn_rcpf(b);
  r = fmaf(fmaf(-b, r, 1.0f), r, r);
  float q = r;
  q = fmaf(fmaf(-b, q, 1.0f), r, q);
  return fmaf(fmaf(-b, q, 1.0f), r, q);
}
// Newton step, one correction
__device__ __forceinline__ float rcp_a(float b)
{
  float r = __builtin_amdgcn_rcpf(b);
  r = fmaf(fmaf(-b, r, 1.0f), r, r);
  return fmaf(fmaf(-b, r, 1.0f), r, r);
}
// no Newton step, two corrections
__device__ __forceinline__ float rcp_b(float b)
{
  const float r = __builtin_amdgcn_rcpf(b);
  float q = fmaf(fmaf(-b, r, 1.0f), r, r);
  return fmaf(fmaf(-b, q, 1.0f), r, q);
}
__device__ __forceinline__ float sqrt_cur(float x)
{
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float em = fmaf(-sm, s, x), ep = fmaf(-sp, s, x);
  float r = (em <= 0.0f) ? sm : s;
  return (ep > 0.0f) ? sp : r;
}
// the hardware estimate alone, and with only one of the two one-ulp corrections
__device__ __forceinline__ float sqrt_raw(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float sqrt_up(float x)
{
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  return (fmaf(-sp, s, x) > 0.0f) ? sp : s;
}
__device__ __forceinline__ float sqrt_dn(float x)
{
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  return (fmaf(-sm, s, x) <= 0.0f) ? sm : s;
}
__device__ __forceinline__ float sqrt_d(float x) { return (float)__builtin_amdgcn_sqrt((double)x); }
__device__ __forceinline__ float div_cur(float a, float b)
{
  float r = __builtin_amdgcn_rcpf(b);
  r = fmaf(fmaf(-b, r, 1.0f), r, r);
  float q = a * r;
  q = fmaf(fmaf(-b, q, a), r, q);
  return fmaf(fmaf(-b, q, a), r, q);
}
__device__ __forceinline__ float div_a(float a, float b)
{
  const float r = __builtin_amdgcn_rcpf(b);
  float q = a * r;
  q = fmaf(fmaf(-b, q, a), r, q);
  return fmaf(fmaf(-b, q, a), r, q);
}

// no Newton step, two corrections on the negated residual (b*q - a): the same arithmetic for nonzero residuals, and
// a -0 quotient keeps its sign
__device__ __forceinline__ float div_b(float a, float b)
{
  const float r = __builtin_amdgcn_rcpf(b);
  float q = a * r;
  q = fmaf(-fmaf(b, q, -a), r, q);
  return fmaf(-fmaf(b, q, -a), r, q);
}

constexpr int kVar = 8;
// one thread per contiguous run of inputs; per-thread mismatch counts and first bad input, stored with vector stores
__global__ void check(int op, uint32_t lo, uint64_t n, uint32_t per, unsigned long long *cnt, uint32_t *first)
{
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c[kVar] = {};
  uint32_t f[kVar] = {};
  for (uint32_t i = 0; i < per; i++) {
    const uint64_t k = t * per + i;
    if (k >= n) break;
    const uint32_t u = lo + (uint32_t)k;
    const float x = __uint_as_float(u);
    float ref = 0.0f, ref2 = 0.0f, v[kVar] = {};
    int nv = 0;
    if (op == 0) {
      ref = 1.0f / x;
      ref2 = (float)(1.0 / (double)x);
      v[0] = rcp_cur(x); v[1] = rcp_a(x); v[2] = rcp_b(x); nv = 3;
    } else if (op == 1) {
      ref = sqrtf(x);
      ref2 = (float)sqrt((double)x);
      v[0] = sqrt_cur(x); v[1] = sqrt_d(x); v[2] = sqrt_raw(x); v[3] = sqrt_up(x); v[4] = sqrt_dn(x); nv = 5;
    } else {
      if (!(fabsf(x) < 3.0e38f)) continue;  // finite x; |x| + 1 below inf
      const float b = fabsf(x) + 1.0f;
      ref = x / b;
      ref2 = (float)((double)x / (double)b);
      v[0] = div_cur(x, b); v[1] = div_a(x, b); v[2] = div_b(x, b); nv = 3;
    }
    // variant kVar-1: the double-precision cross-check of the reference itself
    if (__float_as_uint(ref) != __float_as_uint(ref2)) { if (!c[kVar - 1]) f[kVar - 1] = u; c[kVar - 1]++; }
    for (int j = 0; j < nv; j++)
      if (__float_as_uint(v[j]) != __float_as_uint(ref)) { if (!c[j]) f[j] = u; c[j]++; }
  }
  for (int j = 0; j < kVar; j++) {
    cnt[t * kVar + j] = c[j];
    first[t * kVar + j] = f[j];
  }
}

static void run(int op, const char *name, uint32_t lo, uint32_t hi, const char *const *vnames)
{
  const uint64_t n = (uint64_t)hi - lo + 1;
  const uint32_t per = 256;
  const int threads = 256;
  const uint64_t nthr = (n + per - 1) / per;
  const uint64_t blocks = (nthr + threads - 1) / threads;
  unsigned long long *cnt;
  uint32_t *first;
  hipMalloc(&cnt, sizeof(unsigned long long) * blocks * threads * kVar);
  hipMalloc(&first, sizeof(uint32_t) * blocks * threads * kVar);
  hipLaunchKernelGGL(check, dim3((unsigned)blocks), dim3(threads), 0, 0, op, lo, n, per, cnt, first);
  if (hipDeviceSynchronize() != hipSuccess) { printf("%s: kernel failed\n", name); exit(1); }
  std::vector<unsigned long long> hc(blocks * threads * kVar);
  std::vector<uint32_t> hf(blocks * threads * kVar);
  hipMemcpy(hc.data(), cnt, sizeof(unsigned long long) * hc.size(), hipMemcpyDeviceToHost);
  hipMemcpy(hf.data(), first, sizeof(uint32_t) * hf.size(), hipMemcpyDeviceToHost);
  for (int j = 0; j < kVar; j++) {
    if (!vnames[j]) continue;
    unsigned long long tot = 0;
    uint32_t f = 0;
    for (uint64_t t = 0; t < blocks * threads; t++) {
      if (hc[t * kVar + j] && !tot) f = hf[t * kVar + j];
      tot += hc[t * kVar + j];
    }
    float fx;
    memcpy(&fx, &f, 4);
    printf("%-5s %-24s inputs %llu mismatches %llu first %a\n", name, vnames[j], (unsigned long long)n, tot,
           tot ? (double)fx : 0.0);
  }
  hipFree(cnt);
  hipFree(first);
}

int main()
{
  const char *rv[kVar] = {"current(newton+2corr)", "newton+1corr", "2corr", nullptr, nullptr, nullptr, nullptr,
                          "ref-vs-double"};
  run(0, "rcp", 0x21800000u /* 2^-60 */, 0x5d800000u /* 2^60 */, rv);
  const char *sv[kVar] = {"current", "f64-sqrt", "raw", "up-only", "down-only", nullptr, nullptr, "ref-vs-double"};
  run(1, "sqrt", 0x35800000u /* 2^-20 */, 0x49800000u /* 2^20 */, sv);
  run(1, "sqrt<", 0x38d1b717u /* 1e-4 */, 0x40800000u /* 4 */, sv);
  const char *dv[kVar] = {"current(newton+2corr)", "2corr", "2corr-negres", nullptr, nullptr, nullptr, nullptr,
                          "ref-vs-double"};
  run(2, "soft+", 0x00000000u, 0x7f7fffffu, dv);
  run(2, "soft-", 0x80000000u, 0xff7fffffu, dv);
  // below 2^126 in magnitude (the documented domain)
  run(2, "soft+<", 0x00000000u, 0x7e7fffffu, dv);
  run(2, "soft-<", 0x80000000u, 0xfe7fffffu, dv);
  return 0;
}
