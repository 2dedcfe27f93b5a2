// hostcopy_rates.cpp -- host memcpy bandwidth into pinned staging memory of different kinds (the Fortran drop-in's
// per-call state copies go through a pinned ring): plain malloc, hipHostMalloc default / non-coherent /
// write-combined, and pageable memory registered with hipHostRegister; 1 and 4 threads.
// Build: hipcc -O2 tools/hostcopy_rates.cpp -o tools/hostcopy_rates -lpthread
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double rate(void *dst, const void *src, size_t bytes, int nthr, int reps)
{
  std::vector<std::thread> th;
  auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < nthr; t++)
    th.emplace_back([=] {
      const size_t per = bytes / nthr;
      for (int r = 0; r < reps; r++) std::memcpy((char *)dst + t * per, (const char *)src + t * per, per);
    });
  for (auto &x : th) x.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return (double)bytes * reps / s / 1e9;
}

int main()
{
  const size_t bytes = 8u << 20;
  char *src = (char *)std::malloc(bytes);
  std::memset(src, 1, bytes);
  struct K { const char *name; unsigned flags; int kind; } kinds[] = {
      {"malloc", 0, 0}, {"malloc", 0, 0}, {"hipHostMalloc default", hipHostMallocDefault, 1},
      {"hipHostMalloc noncoherent", hipHostMallocNonCoherent, 1}, {"hipHostMalloc coherent", hipHostMallocCoherent, 1},
      {"hipHostMalloc writecombined", hipHostMallocWriteCombined, 1}, {"malloc + hipHostRegister", 0, 2},
      {"hipHostMalloc default", hipHostMallocDefault, 1}};
  void *dev = nullptr;
  (void)hipMalloc(&dev, bytes);
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  for (auto &k : kinds) {
    void *dst = nullptr;
    if (k.kind == 0 || k.kind == 2) {
      dst = std::aligned_alloc(4096, bytes);
      if (k.kind == 2 && hipHostRegister(dst, bytes, hipHostRegisterDefault) != hipSuccess) { printf("register failed\n"); continue; }
    } else if (hipHostMalloc(&dst, bytes, k.flags) != hipSuccess) {
      printf("%-30s alloc failed\n", k.name);
      continue;
    }
    std::memset(dst, 0, bytes);
    printf("%-30s 1 thread %6.1f GB/s   4 threads %6.1f GB/s\n", k.name, rate(dst, src, bytes, 1, 20),
           rate(dst, src, bytes, 4, 20));
    // and the other direction (D2H staging -> user array)
    printf("%-30s read back: 1 thread %6.1f GB/s\n", "", rate(src, dst, bytes, 1, 20));
    if (k.kind != 0) {  // DMA rates from / to this memory (hipMemcpyAsync on a stream)
      for (int dir = 0; dir < 2; dir++) {
        for (int w = 0; w < 2; w++) {
          auto t0 = std::chrono::steady_clock::now();
          for (int r = 0; r < 20; r++)
            (void)(dir ? hipMemcpyAsync(dst, dev, bytes, hipMemcpyDeviceToHost, st)
                       : hipMemcpyAsync(dev, dst, bytes, hipMemcpyHostToDevice, st));
          (void)hipStreamSynchronize(st);
          const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
          if (w) printf("%-30s DMA %s %6.1f GB/s\n", "", dir ? "D2H" : "H2D", (double)bytes * 20 / s / 1e9);
        }
      }
    }
    if (k.kind == 1) (void)hipHostFree(dst);
    else { if (k.kind == 2) (void)hipHostUnregister(dst); std::free(dst); }
  }
  return 0;
}
