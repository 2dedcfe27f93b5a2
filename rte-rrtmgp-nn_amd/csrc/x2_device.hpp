// x2_device.hpp -- two g-points per lane: packed-fp32 helpers shared by the two-per-lane solvers
// (kernels_sw_x2.hip).  A lane carries g-points g and g+1 as a float2, so products, sums and fma
// chains issue as v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32 -- two IEEE operations each, the same bits as two
// scalar ones -- while the glibc-exact exps (double precision), reciprocals' v_rcp and selects stay per element.
#pragma once
#include "rte_device.hpp"

namespace rrtmgpnn {
namespace x2 {

typedef float f2 __attribute__((ext_vector_type(2)));

// vfma / vmax / vmin take f2 or float (the checkpointed kernel's one-g-point-per-lane instances)
template <class V> __device__ __forceinline__ V vfma(V a, V b, V c) { return __builtin_elementwise_fma(a, b, c); }
template <class V> __device__ __forceinline__ V vmax(V a, V b) { return __builtin_elementwise_max(a, b); }
template <class V> __device__ __forceinline__ V vmin(V a, V b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ f2 splat(float x) { return (f2){x, x}; }

// x <= 0 everywhere it is called (exp of -tau*k and -tau/mu0)
__device__ __forceinline__ f2 exp2v(f2 x, const uint64_t *etab)
{
  return (f2){solver_exp_neg(x.x, etab), solver_exp_neg(x.y, etab)};
}
// the direct-beam transmittance exp(-tau/mu0) (solver_exp_beam)
__device__ __forceinline__ f2 exp2v_beam(f2 x, const uint64_t *etab)
{
  return (f2){solver_exp_beam(x.x, etab), solver_exp_beam(x.y, etab)};
}

// sqrt_rn_normal (libm_ref.hpp) with the correction fmas paired
__device__ __forceinline__ f2 sqrt2(f2 x)
{
  const f2 s = (f2){__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
  const f2 sm = (f2){__uint_as_float(__float_as_uint(s.x) - 1u), __uint_as_float(__float_as_uint(s.y) - 1u)};
  const f2 sp = (f2){__uint_as_float(__float_as_uint(s.x) + 1u), __uint_as_float(__float_as_uint(s.y) + 1u)};
  const f2 em = vfma(-sm, s, x), ep = vfma(-sp, s, x);
  f2 r;
  r.x = (ep.x > 0.0f) ? sp.x : ((em.x <= 0.0f) ? sm.x : s.x);
  r.y = (ep.y > 0.0f) ? sp.y : ((em.y <= 0.0f) ? sm.y : s.y);
  return r;
}

// rcp_rn_normal (libm_ref.hpp) with the Newton fmas paired
__device__ __forceinline__ f2 rcp2(f2 b)
{
  f2 r = (f2){__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  const f2 one = splat(1.0f);
  r = vfma(vfma(-b, r, one), r, r);
  return vfma(vfma(-b, r, one), r, r);
}

// solver_div (rte_device.hpp) with the Newton fmas paired
__device__ __forceinline__ f2 div2(f2 a, f2 b)
{
  f2 r = (f2){__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  r = vfma(vfma(-b, r, splat(1.0f)), r, r);
  f2 q = a * r;
  q = vfma(vfma(-b, q, a), r, q);
  return vfma(vfma(-b, q, a), r, q);
}

// The same helpers for one g-point per lane: the scalar functions they pair (same bits element by element)
__device__ __forceinline__ float exp2v(float x, const uint64_t *etab) { return solver_exp_neg(x, etab); }
__device__ __forceinline__ float exp2v_beam(float x, const uint64_t *etab) { return solver_exp_beam(x, etab); }
__device__ __forceinline__ float sqrt2(float x) { return sqrt_rn_normal(x); }
__device__ __forceinline__ float rcp2(float b) { return rcp_rn_normal(b); }
__device__ __forceinline__ float div2(float a, float b) { return solver_div(a, b); }

// exps of N lane values (f2 or float) with the table reads batched (ref_expf_neg_batch); exp_neg_batch follows
// solver_exp_neg (the tolerance build keeps its per-element hardware exp), exp_beam_batch solver_exp_beam
template <int N, class V>
__device__ __forceinline__ void exp_neg_batch(const V (&x)[N], V (&y)[N], const uint64_t *etab)
{
#if !RRTMGPNN_FAST_LIBM
  constexpr int L = sizeof(V) / sizeof(float);
  float xs[N * L], ys[N * L];
#pragma unroll
  for (int i = 0; i < N; i++) __builtin_memcpy(&xs[i * L], &x[i], sizeof(V));
  ref_expf_neg_batch<N * L>(xs, ys, etab);
#pragma unroll
  for (int i = 0; i < N; i++) __builtin_memcpy(&y[i], &ys[i * L], sizeof(V));
#else
#pragma unroll
  for (int i = 0; i < N; i++) y[i] = exp2v(x[i], etab);
#endif
}
template <int N, class V>
__device__ __forceinline__ void exp_beam_batch(const V (&x)[N], V (&y)[N], const uint64_t *etab)
{
  constexpr int L = sizeof(V) / sizeof(float);
  float xs[N * L], ys[N * L];
#pragma unroll
  for (int i = 0; i < N; i++) __builtin_memcpy(&xs[i * L], &x[i], sizeof(V));
  ref_expf_neg_batch<N * L>(xs, ys, etab);
#pragma unroll
  for (int i = 0; i < N; i++) __builtin_memcpy(&y[i], &ys[i * L], sizeof(V));
}

// 8-byte column-local loads and stores (g-point pair at byte offset voff, layer at soff)
struct ColArr2 {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ ColArr2(const float *base, size_t col_off, uint32_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc((void *)(base + col_off), 0, (int)bytes, 0x00020000)) {}
  __device__ __forceinline__ f2 ld(uint32_t voff, uint32_t soff) const
  {
    return __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  }
  __device__ __forceinline__ float ld1(uint32_t voff, uint32_t soff) const
  {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  }
  __device__ __forceinline__ void st(f2 v, uint32_t voff, uint32_t soff) const
  {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, voff, soff, 0);
  }
};

// column-local loads and stores of one lane's g-points: V = f2 (8 bytes, ColArr2) or float (4 bytes)
template <class V>
struct ColArrV : ColArr2 {
  __device__ __forceinline__ ColArrV(const float *base, size_t col_off, uint32_t bytes) : ColArr2(base, col_off, bytes) {}
  __device__ __forceinline__ V ldv(uint32_t voff, uint32_t soff) const
  {
    if constexpr (sizeof(V) == 8) return ld(voff, soff);
    else return ld1(voff, soff);
  }
  __device__ __forceinline__ void stv(V v, uint32_t voff, uint32_t soff) const
  {
    if constexpr (sizeof(V) == 8) st(v, voff, soff);
    else __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, 0);
  }
};

}  // namespace x2
}  // namespace rrtmgpnn
