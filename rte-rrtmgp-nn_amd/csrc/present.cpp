// present.cpp -- a context's device data environment: the pool of device buffers and the host -> device map the
// Fortran drop-in keeps its optical properties, sources and gas concentrations in between calls (the reference's
// GPU build does the same with OpenACC `enter data` / `update host` / `exit data`, include/rrtmgpnn.h).
//
// Pool: buffers are cached by capacity and handed out again for any request between half and all of it, so the
// steady state of a block loop allocates nothing.  Every use of a buffer is ordered on the context's one stream,
// so a buffer released after enqueueing its last kernel can be handed to the next request at once: the next user's
// work is enqueued behind it.
//
// Present map: one per context (each OpenMP thread of the Fortran drop-in has its own), but the invalidations are
// process-wide, as the reference's single OpenACC data environment is.  `update_device` and `delete` of a host array
// bump that array's generation in a process-wide table; a context's copy made at an older generation is taken as
// "host newer" on its next READ, in every context.  So a host array shared by the worker threads (a gas
// concentration set_vmr re-sets from the serial region between parallel block loops: drop, deallocate, allocate at
// the same address) is uploaded again by every worker instead of being served from its stale cached copy.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <unordered_map>

#include "internal.hpp"

using namespace rrtmgpnn;

namespace {
constexpr size_t kPoolGrain = 256;  // bytes; capacities are rounded up to this

std::mutex g_gen_mu;
std::unordered_map<const void *, uint64_t> g_gen;  // host array -> generation (absent: 0)

uint64_t generation(const void *host)
{
  std::lock_guard<std::mutex> lk(g_gen_mu);
  auto it = g_gen.find(host);
  return it == g_gen.end() ? 0 : it->second;
}

void invalidate_everywhere(const void *host)
{
  std::lock_guard<std::mutex> lk(g_gen_mu);
  ++g_gen[host];
}

int check(rrtmgpnn_context *ctx)
{
  if (!ctx) return fail(RRTMGPNN_ERR_ARGUMENT, "null context");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return fail(RRTMGPNN_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return RRTMGPNN_OK;
}
}  // namespace

int rrtmgpnn_context::pool_get(size_t bytes, void **out)
{
  const size_t cap = (std::max<size_t>(bytes, 1) + kPoolGrain - 1) / kPoolGrain * kPoolGrain;
  auto it = pool_free.lower_bound(cap);
  if (it != pool_free.end() && it->first <= 2 * cap) {
    *out = it->second;
    pool_live[it->second] = it->first;
    pool_free.erase(it);
    return RRTMGPNN_OK;
  }
  void *p = nullptr;
  hipError_t e = hipMalloc(&p, cap);
  if (e != hipSuccess) {
    // give the cached buffers back and try once more
    (void)hipStreamSynchronize(stream);
    for (auto &f : pool_free) (void)hipFree(f.second);
    pool_free.clear();
    (void)hipGetLastError();
    e = hipMalloc(&p, cap);
    if (e != hipSuccess) return fail(RRTMGPNN_ERR_DEVICE, std::string("pool hipMalloc: ") + hipGetErrorString(e));
  }
  pool_live[p] = cap;
  *out = p;
  return RRTMGPNN_OK;
}

void rrtmgpnn_context::pool_put(void *p)
{
  auto it = pool_live.find(p);
  if (it == pool_live.end()) return;
  pool_free.emplace(it->second, p);
  pool_live.erase(it);
}

namespace {
constexpr size_t kPinMin = 32u << 20;   // initial pinned staging ring
constexpr size_t kPinMax = 256u << 20;  // copies larger than this go straight from pageable memory
}  // namespace

// a slice of the pinned ring (nullptr: the copy is too large for it)
static void *pin_slice(rrtmgpnn_context *c, size_t bytes)
{
  const size_t b = (bytes + kPoolGrain - 1) / kPoolGrain * kPoolGrain;
  if (b > kPinMax) return nullptr;
  if (c->pin_head + b > c->pin_cap) {
    if (c->sync()) return nullptr;  // every queued copy is done: the whole ring is free
    if (b > c->pin_cap) {
      if (c->pin) (void)hipHostFree(c->pin);
      c->pin = nullptr;
      c->pin_cap = 0;
      size_t cap = std::max(kPinMin, 2 * b);
      // default flags: non-coherent and coherent allocations measured the same in the Fortran block loop
      if (hipHostMalloc(&c->pin, cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        c->pin = nullptr;
        return nullptr;
      }
      c->pin_cap = cap;
    }
  }
  void *p = (char *)c->pin + c->pin_head;
  c->pin_head += b;
  return p;
}

int rrtmgpnn_context::h2d(void *dst, const void *host, size_t bytes)
{
  if (!bytes) return RRTMGPNN_OK;
  if (void *p = pin_slice(this, bytes)) {
    std::memcpy(p, host, bytes);
    RRTMGPNN_HIP(hipMemcpyAsync(dst, p, bytes, hipMemcpyHostToDevice, stream));
  } else {
    RRTMGPNN_HIP(hipMemcpyAsync(dst, host, bytes, hipMemcpyHostToDevice, stream));
  }
  return RRTMGPNN_OK;
}

int rrtmgpnn_context::d2h(void *host, const void *dev, size_t bytes)
{
  if (!bytes) return RRTMGPNN_OK;
  if (void *p = pin_slice(this, bytes)) {
    RRTMGPNN_HIP(hipMemcpyAsync(p, dev, bytes, hipMemcpyDeviceToHost, stream));
    pending_d2h.push_back({host, p, bytes});
  } else {
    RRTMGPNN_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, stream));
  }
  return RRTMGPNN_OK;
}

int rrtmgpnn_context::sync()
{
  RRTMGPNN_HIP(hipStreamSynchronize(stream));
  for (const auto &d : pending_d2h) std::memcpy(d.dst, d.src, d.bytes);
  pending_d2h.clear();
  pin_head = 0;
  return RRTMGPNN_OK;
}

void rrtmgpnn_context::pool_clear()
{
  (void)sync();
  if (pin) (void)hipHostFree(pin);
  pin = nullptr;
  pin_cap = 0;
  for (auto &f : pool_free) (void)hipFree(f.second);
  for (auto &l : pool_live) (void)hipFree(l.first);
  pool_free.clear();
  pool_live.clear();
  present.clear();
}

extern "C" {

int rrtmgpnn_context_create_owned(int device, rrtmgpnn_context **ctx)
{
  if (int rc = rrtmgpnn_context_create(device, nullptr, ctx)) return rc;
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) {
    rrtmgpnn_context_destroy(*ctx);
    *ctx = nullptr;
    return fail(RRTMGPNN_ERR_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  (*ctx)->stream = s;
  (*ctx)->own_stream = true;
  return RRTMGPNN_OK;
}

int rrtmgpnn_present(rrtmgpnn_context *ctx, const void *host, long long bytes, int mode, void **dptr)
{
  if (int rc = check(ctx)) return rc;
  if (!host || !dptr || bytes <= 0 || !(mode & (RRTMGPNN_PRESENT_READ | RRTMGPNN_PRESENT_WRITE)))
    return fail(RRTMGPNN_ERR_ARGUMENT, "present: needs a host array, a positive size and a READ/WRITE mode");
  auto &m = ctx->present;
  auto it = m.find(host);
  if (it != m.end() && it->second.bytes != (size_t)bytes) {  // same address, another array: start over
    ctx->pool_put(it->second.dev);
    m.erase(it);
    it = m.end();
  }
  if (it == m.end()) {
    rrtmgpnn_context::Present p;
    if (int rc = ctx->pool_get((size_t)bytes, &p.dev)) return rc;
    p.bytes = (size_t)bytes;
    p.state = 0;
    it = m.emplace(host, p).first;
  }
  auto &p = it->second;
  const uint64_t gen = generation(host);
  if (p.gen != gen) {  // updated or deleted through some context since this copy was made: the host copy is newer
    // (also over a device-newer copy of this context: the host wins, include/rrtmgpnn.h)
    p.state = 0;
    p.gen = gen;
  }
  if ((mode & RRTMGPNN_PRESENT_READ) && p.state == 0) {
    if (int rc = ctx->h2d(p.dev, host, p.bytes)) return rc;
    p.state = 1;
  }
  if (mode & RRTMGPNN_PRESENT_WRITE) p.state = 2;
  *dptr = p.dev;
  return RRTMGPNN_OK;
}

int rrtmgpnn_present_update_host(rrtmgpnn_context *ctx, void *host)
{
  if (int rc = check(ctx)) return rc;
  auto it = ctx->present.find(host);
  if (it == ctx->present.end() || it->second.state != 2) return RRTMGPNN_OK;
  if (int rc = ctx->d2h(host, it->second.dev, it->second.bytes)) return rc;
  if (int rc = ctx->sync()) return rc;
  it->second.state = 1;
  return RRTMGPNN_OK;
}

int rrtmgpnn_present_update_device(rrtmgpnn_context *ctx, const void *host)
{
  if (int rc = check(ctx)) return rc;
  invalidate_everywhere(host);  // every context's copy (this one's too) is reloaded on its next READ
  auto it = ctx->present.find(host);
  if (it != ctx->present.end()) it->second.state = 0;
  return RRTMGPNN_OK;
}

int rrtmgpnn_present_delete(rrtmgpnn_context *ctx, const void *host)
{
  if (int rc = check(ctx)) return rc;
  invalidate_everywhere(host);  // other contexts keep their buffers, but their copies are stale from here on
  auto it = ctx->present.find(host);
  if (it == ctx->present.end()) return RRTMGPNN_OK;
  ctx->pool_put(it->second.dev);
  ctx->present.erase(it);
  return RRTMGPNN_OK;
}

int rrtmgpnn_stage_h2d(rrtmgpnn_context *ctx, const void *host, long long bytes, void **dptr)
{
  if (int rc = check(ctx)) return rc;
  if (!host || !dptr || bytes <= 0) return fail(RRTMGPNN_ERR_ARGUMENT, "stage_h2d: bad arguments");
  if (int rc = ctx->pool_get((size_t)bytes, dptr)) return rc;
  return ctx->h2d(*dptr, host, (size_t)bytes);
}

int rrtmgpnn_scratch(rrtmgpnn_context *ctx, long long bytes, void **dptr)
{
  if (int rc = check(ctx)) return rc;
  if (!dptr || bytes <= 0) return fail(RRTMGPNN_ERR_ARGUMENT, "scratch: bad arguments");
  return ctx->pool_get((size_t)bytes, dptr);
}

int rrtmgpnn_release(rrtmgpnn_context *ctx, void *dptr)
{
  if (int rc = check(ctx)) return rc;
  if (dptr) ctx->pool_put(dptr);
  return RRTMGPNN_OK;
}

int rrtmgpnn_copy_d2h(rrtmgpnn_context *ctx, void *host, const void *dptr, long long bytes)
{
  if (int rc = check(ctx)) return rc;
  if (!host || !dptr || bytes < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "copy_d2h: bad arguments");
  return ctx->d2h(host, dptr, (size_t)bytes);
}

int rrtmgpnn_copy_h2d(rrtmgpnn_context *ctx, void *dptr, const void *host, long long bytes)
{
  if (int rc = check(ctx)) return rc;
  if (!host || !dptr || bytes < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "copy_h2d: bad arguments");
  return ctx->h2d(dptr, host, (size_t)bytes);
}

int rrtmgpnn_copy_d2d(rrtmgpnn_context *ctx, void *dst, const void *src, long long bytes)
{
  if (int rc = check(ctx)) return rc;
  if (!dst || !src || bytes < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "copy_d2d: bad arguments");
  if (bytes) RRTMGPNN_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return RRTMGPNN_OK;
}

int rrtmgpnn_memset_async(rrtmgpnn_context *ctx, void *dptr, int value, long long bytes)
{
  if (int rc = check(ctx)) return rc;
  if (!dptr || bytes < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "memset: bad arguments");
  if (bytes) RRTMGPNN_HIP(hipMemsetAsync(dptr, value, (size_t)bytes, ctx->stream));
  return RRTMGPNN_OK;
}

}  // extern "C"
