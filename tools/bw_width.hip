// Streaming-read bandwidth against the access width per lane and the bytes each wave keeps in flight, at the
// solvers' occupancies -- does the SW solver's 8-byte-per-lane plane traffic cap its passes near 5 TB/s?
// Tool code, not part of librrtmgpnn.  Build: hipcc -O3 --offload-arch=gfx950 tools/bw_width.hip -o tools/bw_width
// Run: tools/bw_width  ->  one line per (width, loads in flight per lane, waves per SIMD): TB/s over a 2 GiB array.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int W> struct V;
template <> struct V<4> { typedef uint32_t T; };
template <> struct V<8> { typedef uint2 T; };
template <> struct V<16> { typedef uint4 T; };

__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// every wave sweeps its own contiguous slab; U independent loads per lane per step (U * W * 64 bytes in flight per
// wave), like a solver layer step loading U planes' rows of one column
template <int W, int U>
__global__ void __launch_bounds__(256) sweep(const void *__restrict__ in, size_t nvec, uint32_t *__restrict__ out)
{
  typedef typename V<W>::T T;
  const T *p = (const T *)in;
  const size_t waves = (size_t)gridDim.x * (blockDim.x / 64);
  const size_t wave = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const size_t per = nvec / waves / 64 / U * 64 * U;  // vectors per wave, a multiple of 64 U
  const T *q = p + wave * per + (threadIdx.x & 63);
  uint32_t s = 0;
  for (size_t i = 0; i < per; i += 64 * U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = q[i + 64 * u];
#pragma unroll
    for (int u = 0; u < U; u++) s ^= fold(v[u]);
  }
  if (s == 0x12345678u) out[0] = s;
}

template <int W, int U>
static float run(const void *buf, size_t bytes, uint32_t *out, int blocks)
{
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((sweep<W, U>), dim3(blocks), dim3(256), 0, 0, buf, bytes / W, out);  // warm
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((sweep<W, U>), dim3(blocks), dim3(256), 0, 0, buf, bytes / W, out);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  const int waves = blocks * 4;
  const size_t per = bytes / W / waves / 64 / U * 64 * U;
  return (float)((double)per * W * waves / (best * 1e-3) / 1e12);
}

int main()
{
  const size_t bytes = 2ull << 30;
  void *buf = nullptr;
  uint32_t *out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("width_B loads_in_flight_per_lane waves_per_simd TB/s\n");
  for (int wps : {2, 3, 4, 8}) {
    const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD each
#define R(W, U) printf("%d %d %d %.3f\n", W, U, wps, run<W, U>(buf, bytes, out, blocks))
    R(4, 1); R(4, 2); R(4, 4); R(4, 8);
    R(8, 1); R(8, 2); R(8, 3); R(8, 4); R(8, 6); R(8, 8);
    R(16, 1); R(16, 2); R(16, 4);
  }
  hipFree(buf);
  hipFree(out);
  return 0;
}
