// valu_rates.hip -- issue cost and dependent latency of the VALU instructions the SW solver is made of, on gfx950.
//
// Each kernel runs CHAINS independent chains of one instruction, ITER times, in every wave; the grid puts WAVES waves
// on every SIMD (256 CUs x 4 SIMDs).  cycles per instruction per SIMD = elapsed * clock / (instructions per SIMD).
// With 8 chains and 8 waves per SIMD the figure is the issue cost; with 1 chain and 1 wave it is the dependent latency.
// Build: hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define ITER 2048

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ inline float fst(float x) { return x; }
__device__ inline float fst(double x) { return (float)x; }
__device__ inline float fst(f2 x) { return x.x; }

#define OP_KERNEL(NAME, T, ASM)                                                                 \
  template <int CH>                                                                             \
  __global__ void __launch_bounds__(512) NAME(T *out, T b, T c)                                 \
  {                                                                                             \
    T a[CH];                                                                                    \
    _Pragma("unroll") for (int i = 0; i < CH; i++) a[i] = out[threadIdx.x % 8 + i];             \
    for (int it = 0; it < ITER; it++) {                                                         \
      _Pragma("unroll") for (int i = 0; i < CH; i++) asm volatile(ASM : "+v"(a[i]) : "v"(b), "v"(c)); \
    }                                                                                           \
    T s = a[0];                                                                                 \
    _Pragma("unroll") for (int i = 1; i < CH; i++) s += a[i];                                   \
    if (fst(s) == 12345.0f) out[blockIdx.x] = s;                                                \
  }

OP_KERNEL(k_fma_f32, float, "v_fma_f32 %0, %1, %2, %0")
OP_KERNEL(k_add_f32, float, "v_add_f32 %0, %1, %0")
OP_KERNEL(k_exp_f32, float, "v_exp_f32 %0, %0")
OP_KERNEL(k_rcp_f32, float, "v_rcp_f32 %0, %0")
OP_KERNEL(k_sqrt_f32, float, "v_sqrt_f32 %0, %0")
OP_KERNEL(k_pk_fma_f32, f2, "v_pk_fma_f32 %0, %1, %2, %0")
OP_KERNEL(k_pk_mul_f32, f2, "v_pk_mul_f32 %0, %1, %0")
OP_KERNEL(k_pk_add_f32, f2, "v_pk_add_f32 %0, %1, %0")
OP_KERNEL(k_fma_f64, double, "v_fma_f64 %0, %1, %2, %0")
OP_KERNEL(k_mul_f64, double, "v_mul_f64 %0, %1, %0")
OP_KERNEL(k_add_f64, double, "v_add_f64 %0, %1, %0")
OP_KERNEL(k_cndmask, float, "v_cndmask_b32 %0, %1, %0, vcc")
OP_KERNEL(k_mov_b64, double, "v_mov_b64 %0, %1")
OP_KERNEL(k_lshl_add_u64, double, "v_lshl_add_u64 %0, %0, 3, %1")

// conversions change the register width, so they run in pairs (f32 -> f64 -> f32)
template <int CH>
__global__ void __launch_bounds__(512) k_cvt_pair(float *out, float b, float c)
{
  float a[CH];
#pragma unroll
  for (int i = 0; i < CH; i++) a[i] = out[threadIdx.x % 8 + i];
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      double d;
      asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d) : "v"(a[i]));
      asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(a[i]) : "v"(d));
    }
  }
  float s = a[0];
#pragma unroll
  for (int i = 1; i < CH; i++) s += a[i];
  if (s == 12345.f) out[blockIdx.x] = s;
}

// ds_read_b64 of a per-lane table index (the exp table gather), dependent: the index comes from the last value
template <int CH>
__global__ void __launch_bounds__(512) k_lds_gather(double *out, double b, double c)
{
  __shared__ double tab[32];
  if (threadIdx.x < 32) tab[threadIdx.x] = (double)threadIdx.x;
  __syncthreads();
  unsigned idx[CH];
#pragma unroll
  for (int i = 0; i < CH; i++) idx[i] = (threadIdx.x + i) % 32;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      double v = tab[idx[i]];
      idx[i] = ((unsigned)__double2hiint(v) + idx[i] + 1) & 31;
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < CH; i++) s += idx[i];
  if (s == 12345u) out[blockIdx.x] = s;
}

template <typename T, typename K>
static void run(const char *name, K kern8, K kern1, int instr_per_iter)
{
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev);
  T *out;
  hipMalloc(&out, sizeof(T) * 65536);
  hipMemset(out, 0, sizeof(T) * 65536);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("%-16s", name);
  // (chains, waves per SIMD)
  const int cfg[4][2] = {{8, 8}, {8, 2}, {1, 8}, {1, 1}};
  for (auto &c : cfg) {
    const int chains = c[0], waves = c[1];
    // blocks of 4 waves (one per SIMD), `waves` blocks per CU
    const dim3 grid(cus * waves), block(256);
    K k = chains == 8 ? kern8 : kern1;
    hipLaunchKernelGGL(k, grid, block, 0, 0, out, (T)1, (T)0);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, grid, block, 0, 0, out, (T)1, (T)0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double instr_per_simd = 5.0 * waves * chains * (double)ITER * instr_per_iter;
    const double cyc = ms * 1e-3 * clk_khz * 1e3 / instr_per_simd;
    printf("  ch%d/w%d %6.2f", chains, waves, cyc);
  }
  printf("   cycles per instruction per SIMD (clock %d MHz)\n", clk_khz / 1000);
  hipFree(out);
}

#define RUN(K, T, N) run<T>(#K, K<8>, K<1>, N)

int main()
{
  RUN(k_fma_f32, float, 1);
  RUN(k_add_f32, float, 1);
  RUN(k_pk_fma_f32, f2, 1);
  RUN(k_pk_mul_f32, f2, 1);
  RUN(k_pk_add_f32, f2, 1);
  RUN(k_fma_f64, double, 1);
  RUN(k_mul_f64, double, 1);
  RUN(k_add_f64, double, 1);
  RUN(k_exp_f32, float, 1);
  RUN(k_rcp_f32, float, 1);
  RUN(k_sqrt_f32, float, 1);
  RUN(k_cndmask, float, 1);
  RUN(k_mov_b64, double, 1);
  RUN(k_lshl_add_u64, double, 1);
  RUN(k_cvt_pair, float, 2);
  RUN(k_lds_gather, double, 1);
  return 0;
}
