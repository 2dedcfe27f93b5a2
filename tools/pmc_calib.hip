// Calibration kernels for the rocprofv3 FETCH_SIZE / WRITE_SIZE counters at the access widths the solvers use
// (MI355X_MICROARCH.md: only 16-B-per-lane streaming accesses are calibrated there).  Each kernel moves a known
// byte count through HBM: tools/pmc_calib.py runs them under --pmc and prints counter bytes / true bytes.
// Tool code, not part of librrtmgpnn.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int W>
struct Vec;
template <>
struct Vec<4> { typedef float T; };
template <>
struct Vec<8> { typedef float2 T; };
template <>
struct Vec<16> { typedef float4 T; };

template <typename T>
__device__ __forceinline__ float fold(T v);
template <>
__device__ __forceinline__ float fold(float v) { return v; }
template <>
__device__ __forceinline__ float fold(float2 v) { return v.x + v.y; }
template <>
__device__ __forceinline__ float fold(float4 v) { return v.x + v.y + v.z + v.w; }

// grid-stride streaming read, W bytes per lane
template <int W>
__global__ void __launch_bounds__(256) read_kernel(const void *__restrict__ in, size_t n, float *__restrict__ out)
{
  typedef typename Vec<W>::T T;
  const T *p = (const T *)in;
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += fold(p[i]);
  if (s == 12345.678f) out[0] = s;  // keeps the loads; never true for the zero-filled input
}

// grid-stride streaming write, W bytes per lane
template <int W>
__global__ void __launch_bounds__(256) write_kernel(void *__restrict__ outp, size_t n)
{
  typedef typename Vec<W>::T T;
  T *p = (T *)outp;
  T v;
  __builtin_memset(&v, 0, sizeof(v));
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// the solvers' pattern: one block per column, one lane per g-point (W=4) or g-point pair (W=8), a row of
// ngpt floats per level read (or written) with raw buffer loads/stores at a scalar level offset
template <int W, bool kStore>
__global__ void __launch_bounds__(256) column_kernel(float *__restrict__ a, int ngpt, int nlev, float *__restrict__ out)
{
  const uint32_t row = 4u * (uint32_t)ngpt;
  const size_t col = (size_t)ngpt * nlev * blockIdx.x;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a + col), 0, (int)(row * nlev), 0x00020000);
  const int lanes = ngpt * 4 / W;
  if ((int)threadIdx.x >= lanes) return;
  const uint32_t v = (uint32_t)W * threadIdx.x;
  float s = 0.0f;
  for (int l = 0; l < nlev; l++) {
    if (kStore) {
      if (W == 4)
        __builtin_amdgcn_raw_buffer_store_b32(0u, r, v, row * l, 0);
      else {
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64((u2){0u, 0u}, r, v, row * l, 0);
      }
    } else {
      if (W == 4)
        s += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, v, row * l, 0));
      else {
        const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, v, row * l, 0);
        s += __uint_as_float(x[0]) + __uint_as_float(x[1]);
      }
    }
  }
  if (s == 12345.678f) out[0] = s;
}

// VALU issue calibration: 8 independent fma chains per lane, NIT iterations (8 * NIT v_fma per wave, no memory).
// Built with -fno-slp-vectorize so float stays v_fma_f32; pk2 (two floats per value) is v_pk_fma_f32.
typedef float pk2 __attribute__((ext_vector_type(2)));
template <typename T, typename S>
__global__ void __launch_bounds__(256) fma_kernel(S *__restrict__ out, int nit, S a_, S b_)
{
  const T a = a_, b = b_;
  T x0 = (S)threadIdx.x, x1 = x0 + (S)1, x2 = x0 + (S)2, x3 = x0 + (S)3, x4 = x0 + (S)4, x5 = x0 + (S)5,
    x6 = x0 + (S)6, x7 = x0 + (S)7;
  for (int i = 0; i < nit; i++) {
    x0 = x0 * a + b; x1 = x1 * a + b; x2 = x2 * a + b; x3 = x3 * a + b;
    x4 = x4 * a + b; x5 = x5 * a + b; x6 = x6 * a + b; x7 = x7 * a + b;
  }
  const T s = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
  if constexpr (sizeof(T) == sizeof(S)) {
    if (s == (S)12345.678) out[0] = s;
  } else {
    if (s.x == (S)12345.678) out[0] = s.x + s.y;
  }
}

extern "C" {
// returns the kernel time in ms (hipEvents); dbl: v_fma_f64 instead of v_fma_f32
// returns the kernel time in ms (hipEvents); kind 0 v_fma_f32, 1 v_fma_f64, 2 v_pk_fma_f32
float calib_fma(int kind, void *out, int blocks, int nit)
{
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  if (kind == 1)
    hipLaunchKernelGGL((fma_kernel<double, double>), dim3(blocks), dim3(256), 0, 0, (double *)out, nit, 0.999, 1e-3);
  else if (kind == 2)
    hipLaunchKernelGGL((fma_kernel<pk2, float>), dim3(blocks), dim3(256), 0, 0, (float *)out, nit, 0.999f, 1e-3f);
  else
    hipLaunchKernelGGL((fma_kernel<float, float>), dim3(blocks), dim3(256), 0, 0, (float *)out, nit, 0.999f, 1e-3f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return ms;
}

int calib_read(int width, const void *in, size_t bytes, float *out)
{
  const dim3 grid(4096), block(256);
  if (width == 4) hipLaunchKernelGGL(read_kernel<4>, grid, block, 0, 0, in, bytes / 4, out);
  else if (width == 8) hipLaunchKernelGGL(read_kernel<8>, grid, block, 0, 0, in, bytes / 8, out);
  else hipLaunchKernelGGL(read_kernel<16>, grid, block, 0, 0, in, bytes / 16, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
int calib_write(int width, void *p, size_t bytes)
{
  const dim3 grid(4096), block(256);
  if (width == 4) hipLaunchKernelGGL(write_kernel<4>, grid, block, 0, 0, p, bytes / 4);
  else if (width == 8) hipLaunchKernelGGL(write_kernel<8>, grid, block, 0, 0, p, bytes / 8);
  else hipLaunchKernelGGL(write_kernel<16>, grid, block, 0, 0, p, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
// ngpt <= 256 (W=4) or <= 512 (W=8); a holds ngpt * nlev * ncol floats
int calib_column(int width, int store, float *a, int ngpt, int nlev, int ncol, float *out)
{
  const dim3 grid(ncol), block(256);
  if (width == 4 && store) hipLaunchKernelGGL((column_kernel<4, true>), grid, block, 0, 0, a, ngpt, nlev, out);
  else if (width == 4) hipLaunchKernelGGL((column_kernel<4, false>), grid, block, 0, 0, a, ngpt, nlev, out);
  else if (store) hipLaunchKernelGGL((column_kernel<8, true>), grid, block, 0, 0, a, ngpt, nlev, out);
  else hipLaunchKernelGGL((column_kernel<8, false>), grid, block, 0, 0, a, ngpt, nlev, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}
