// rte_device.hpp -- device-side pieces shared by the RTE solver kernels (kernels_rte.hip,
// kernels_lw_scat.hip): constants, band lookup, the ordered broadband reduction and column-local
// buffer addressing.
#pragma once
#include "internal.hpp"
#include "libm_ref.hpp"

#include <cfloat>
#include <cmath>

namespace rrtmgpnn {

static constexpr float kPi = 3.14159265358979323846f;


__device__ __forceinline__ int band_of(const BandArgs &b, int g)
{
  for (int i = 0; i < b.nbnd; i++)
    if (g >= b.lims[2 * i] - 1 && g < b.lims[2 * i + 1]) return i;
  return 0;
}

static constexpr int kExpTabOff = 0, kExpTabFloats = 64;  // exp table (32 x u64) at the front of LDS

// The solvers' divisions whose operands stay in the normal range use div_rn_normal, and their exps of non-positive
// arguments ref_expf_neg (libm_ref.hpp): the bits of a / b and of glibc's expf, in fewer instructions.
__device__ __forceinline__ float solver_div(float a, float b) { return div_rn_normal(a, b); }
// RRTMGPNN_FAST_LIBM (opt-in tolerance build, librrtmgpnn_fastlibm.so; never the default): the solvers' exps of
// non-positive arguments use the hardware exponential (v_exp_f32, a few ulp) instead of glibc's algorithm
// evaluated in double.  Fluxes then differ from the reference's in the last bits; tests/test_gpu_tolerance.py holds
// them to the north star's 1e-3 W/m2 RMS.
#ifndef RRTMGPNN_FAST_LIBM
#define RRTMGPNN_FAST_LIBM 0
#endif
// The direct-beam transmittance exp(-tau/mu0) multiplies down every layer of a column, so its rounding errors compound:
// it keeps glibc's algorithm in the tolerance build too (with the hardware exp there, C3 SW down-flux errors reached
// 1.0e-3 W/m2 RMS, the north star's bar itself).
__device__ __forceinline__ float solver_exp_beam(float x, const uint64_t *tab) { return ref_expf_neg(x, tab); }
__device__ __forceinline__ float solver_exp_neg(float x, const uint64_t *tab)
{
#if RRTMGPNN_FAST_LIBM
  // 2^(x log2 e) on the hardware exp2 (v_exp_f32, ~1 ulp), with the product x*log2(e) carried in two parts (hi by
  // the rounded product, lo by fma residual + x*(log2(e) - hi constant)) so its rounding does not scale with |x|;
  // the lo part enters as the first-order factor (1 + lo*ln2).
  (void)tab;
  const float L = 1.44269502162933349609375f, L_lo = 1.925963033500011079E-8f, LN2 = 0.693147180559945f;
  const float t = x * L;
  float e = fmaf(x, L, -t);
  e = fmaf(x, L_lo, e);
  const float r = __builtin_amdgcn_exp2f(t);
  return (x < -0x1.9fe368p6f) ? 0.0f : fmaf(r, e * LN2, r);
#else
  return ref_expf_neg(x, tab);
#endif
}


// interpolate1D of compute_Planck_source_nn (rrtmgp/kernels/mo_gas_optics_kernels.F90:1024-1043)
__device__ __forceinline__ float interp1d(float val, float offset, float delta, int ntemp, const float *__restrict__ t)
{
  float val0 = (val - offset) / delta;
  int iv = (int)val0;  // Fortran int(): truncation
  float frac = val0 - (float)iv;
  int index = min(ntemp - 1, max(1, iv + 1));
  float lo = t[index - 1], hi = t[index];
  return lo + frac * (hi - lo);
}

// Planck inputs of the LW solvers that form the sources in-kernel from the Planck fraction
struct LwPlanck {
  const float *tlay, *tlev, *tsfc, *totplnk;
  int ntemp, sfc_lay;
  int emis_by_band;  // sfc_emis is (nbnd, ncol) and expanded in-kernel (rte_lw's expand)
  float tmin, tdelta;
};

// fused Planck table size in floats, padded so the ring that follows stays 16-byte aligned
__host__ __device__ constexpr size_t lw_btab_floats(int nbnd, int nlay) { return ((size_t)nbnd * (2 * nlay + 2) + 3) & ~(size_t)3; }

// Gauss-Jacobi quadrature of the LW no-scattering solvers (secants and weights, nmus <= 4)
struct LwAngles {
  float D[4], w[4];
  int nmus;
  const float *Dg;  // rte_lw's lw_Ds: per-(g-point, column) secants D(igpt, icol), one angle (nullptr: Gauss D)
  int rad;          // kMulti with one angle (g-point outputs): store radiances, reduce with fac as lw_solver_noscat
};

// ------------------------------------------------------------------------------------------
// Ordered broadband reduction.  The reference sums g-points into 4 interleaved partial sums,
// partial j accumulating g = j, j+4, j+8, ... in increasing g, then ((p0+p1)+p2)+p3
// (rte/kernels/mo_rte_solver_kernels.F90:296-318 LW, :643-686 SW).  A float32 tree reduction
// differs from that by several ulp of the broadband flux (~1e-3 W/m2 at SW magnitudes), so the
// kernels reproduce the reference's order exactly: each level's per-g values are staged in an
// LDS ring of R levels; when it fills, one thread per (quantity, level) walks them sequentially.
// ------------------------------------------------------------------------------------------
// Flush `n` staged levels.  ring: [nq][R][ngpt], slot c holds level lev0 + c*dl; part: [nq][nlev][4].
// One thread per (quantity, level) walks the level's g-points with 16-byte LDS reads: element k of
// the float4 at m is g = 4m + k, so the 4 interleaved partials advance together, each in g order.
// dn_mode (SW): quantity 1 is accumulated as (s + ring1) + ring2, i.e. sums_dn + radn_dn + radn_dir.
// ngpt % 4 != 0, or seq: the reference uses sum(radn, 1) instead (one sequential sum, kept in partial 0).
// slot0: the first staged slot (the levels sit in slots slot0 .. slot0 + n - 1)
template <int R>
__device__ __forceinline__ void ring_flush(const float *ring, float *part, int nq, int n, int lev0, int dl, int ngpt,
                                           int nlev, bool dn_mode, bool seq = false, int slot0 = 0)
{
  __syncthreads();
  const int t = threadIdx.x;
  if (t < nq * n) {
    const int q = t / n, c = t - q * n;
    const float *r = ring + ((size_t)q * R + slot0 + c) * ngpt;
    const float *r2 = ring + ((size_t)2 * R + slot0 + c) * ngpt;
    const bool dn = dn_mode && q == 1;
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    if ((ngpt & 3) == 0 && !seq) {
      const float4 *r4 = (const float4 *)r, *q4 = (const float4 *)r2;
      const int n4 = ngpt >> 2;
      if (dn) {
#pragma unroll 4
        for (int m = 0; m < n4; m++) {
          const float4 a = r4[m], b = q4[m];
          s0 = (s0 + a.x) + b.x; s1 = (s1 + a.y) + b.y; s2 = (s2 + a.z) + b.z; s3 = (s3 + a.w) + b.w;
        }
      } else {
#pragma unroll 4
        for (int m = 0; m < n4; m++) {
          const float4 a = r4[m];
          s0 = s0 + a.x; s1 = s1 + a.y; s2 = s2 + a.z; s3 = s3 + a.w;
        }
      }
    } else {
      if (dn) for (int i = 0; i < ngpt; i++) s0 = s0 + (r[i] + r2[i]);  // radn_dn = radn_dn + radn_dir; sum
      else    for (int i = 0; i < ngpt; i++) s0 = s0 + r[i];
    }
    float4 *p = (float4 *)(part + ((size_t)q * nlev + lev0 + c * dl) * 4);
    *p = make_float4(s0, s1, s2, s3);
  }
  __syncthreads();
}

// ring_flush of one quantity (nq = 1, no dn_mode) for ngpt % 4 == 0 with one lane per partial: lane (s, j) walks
// partial j of slot s (ring rows `stride` floats apart) and stores it to part[lev][j] -- the same partial sums as
// ring_flush's float4 walk, in the same order, with a quarter of its instructions on the flushing wave.  With rows
// padded to stride = ngpt + 4 the lanes' rows start in different LDS banks.
// slot0: the first staged slot (the levels sit in slots slot0 .. slot0 + n - 1)
__device__ __forceinline__ void ring_flush_lanes(const float *ring, int stride, float *part, int n, int lev0, int dl,
                                                 int ngpt, int slot0 = 0)
{
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 4 * n) {
    const int sl = t >> 2, j = t & 3;
    const float *r = ring + (size_t)(slot0 + sl) * stride + j;
    const int n4 = ngpt >> 2;
    float sum = 0.0f;
#pragma unroll 8
    for (int m = 0; m < n4; m++) sum = sum + r[4 * m];
    part[(size_t)(lev0 + sl * dl) * 4 + j] = sum;
  }
  __syncthreads();
}

__device__ __forceinline__ float combine4(const float *p) { return ((p[0] + p[1]) + p[2]) + p[3]; }

// The SW solvers' flush for blocks that hold `ncb` columns: ring [ncb][3][R][ngpt] (up, dif, dir of column c at
// ring + c*3*R*ngpt).  Each (column, quantity, level) thread forms the level's complete ordered sum -- the same
// partials and the same ((p0 + p1) + p2) + p3 as ring_flush + combine4 -- and stores it straight to the flux
// array: up, dn (= dif + dir, dn_mode) and dir.  Columns at or past ncol (the grid's last block) store nothing.
// kTotal: the down slot already holds the total (diffuse + direct) g-point flux, as sw_solver_2stream forms it when it
// saves g-point fluxes (:660-670): the down sum is s + total instead of (s + diffuse) + direct
// stride: floats per ring row (ngpt, or ngpt padded so that the rows the flush threads walk together fall in different
// LDS banks)
template <int R, bool kTotal = false>
__device__ __forceinline__ void ring_flush_sw(const float *ring, int ncb, int n, int lev0, int dl, int ngpt, int nlev,
                                              int icol0, int ncol, float *o_up, float *o_dn, float *o_dir,
                                              int stride = 0, int slot0 = 0)
{
  __syncthreads();
  const int t = threadIdx.x;
  const int rs = stride ? stride : ngpt;
  if (t < 3 * ncb * n) {
    const int c = t / (3 * n), rem = t - c * 3 * n, q = rem / n, s = rem - q * n;
    const float *rc = ring + (size_t)c * 3 * R * rs;
    const float *r = rc + ((size_t)q * R + slot0 + s) * rs;
    const float *r2 = rc + ((size_t)2 * R + slot0 + s) * rs;
    const bool dn = q == 1;
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    if ((ngpt & 3) == 0) {
      const float4 *r4 = (const float4 *)r, *q4 = (const float4 *)r2;
      const int n4 = ngpt >> 2;
      if (dn && !kTotal) {
#pragma unroll 4
        for (int m = 0; m < n4; m++) {
          const float4 a = r4[m], b = q4[m];
          s0 = (s0 + a.x) + b.x; s1 = (s1 + a.y) + b.y; s2 = (s2 + a.z) + b.z; s3 = (s3 + a.w) + b.w;
        }
      } else {
#pragma unroll 4
        for (int m = 0; m < n4; m++) {
          const float4 a = r4[m];
          s0 = s0 + a.x; s1 = s1 + a.y; s2 = s2 + a.z; s3 = s3 + a.w;
        }
      }
    } else {
      if (dn && !kTotal) for (int i = 0; i < ngpt; i++) s0 = s0 + (r[i] + r2[i]);
      else    for (int i = 0; i < ngpt; i++) s0 = s0 + r[i];
    }
    const int icol = icol0 + c;
    if (icol < ncol) {
      float *o = q == 0 ? o_up : (q == 1 ? o_dn : o_dir);
      o[lev0 + s * dl + (size_t)nlev * icol] = ((s0 + s1) + s2) + s3;
    }
  }
  __syncthreads();
}

// The same sums with one lane per partial (ngpt % 4 == 0): lane (q, c, s, j) walks partial j of quantity q, column c,
// ring slot slot0 + s -- 4 words per step instead of a float4 per (q, c, s) -- and the four partials of a row are then
// combined ((p0 + p1) + p2) + p3 by the row's lane j = 0 (partials fetched from lanes j = 1..3 of its quad).  Lanes
// are ordered quantity-major, so with 64 lanes per (quantity) group a wave walks one quantity only: the down sums (two
// adds per step) and the others do not share a wave's instruction stream.  Same partials, same additions, same order,
// same bits as ring_flush_sw; about a quarter of its instructions on the critical wave.
// ring_flush_sw_lanes maps a lane's row to its column with three comparisons: at most this many columns per block
// (the SW launchers refuse more before launching)
constexpr int kFlushLanesMaxCols = 4;

template <int R, bool kTotal = false>
__device__ __forceinline__ void ring_flush_sw_lanes(const float *ring, int ncb, int n, int lev0, int dl, int ngpt,
                                                    int nlev, int icol0, int ncol, float *o_up, float *o_dn,
                                                    float *o_dir, int stride, int slot0 = 0)
{
  __syncthreads();
  const int t = threadIdx.x;
  const int per_q = ncb * n * 4;  // lanes per quantity
  if (t < 3 * per_q) {  // idle lanes of the last wave walk nothing (the branch is per lane only in that wave)
    // the lane's (quantity, column, slot, partial) by comparisons and 24-bit products: integer division by the
    // runtime per_q and n took ~40 dependent VALU ops (quarter-rate multiplies among them) before every flush
    const int q = (t >= per_q) + (t >= 2 * per_q);  // three quantities
    const int rem = t - (int)__umul24((unsigned)q, (unsigned)per_q), row = rem >> 2, j = rem & 3;
    const int c = (ncb > 1 && row >= n) + (ncb > 2 && row >= 2 * n) + (ncb > 3 && row >= 3 * n);  // ncb <= kFlushLanesMaxCols
    const int sl = row - (int)__umul24((unsigned)c, (unsigned)n);
    // LDS offsets (well under 2^24 floats)
    const int rc = (int)__umul24((unsigned)c, (unsigned)(3 * R * stride)) + j;
    const float *r = ring + rc + (int)__umul24((unsigned)(q * R + slot0 + sl), (unsigned)stride);
    const float *r2 = ring + rc + (int)__umul24((unsigned)(2 * R + slot0 + sl), (unsigned)stride);
    const int n4 = ngpt >> 2;
    float sum = 0.0f;
    if (q == 1 && !kTotal) {
#pragma unroll 8
      for (int m = 0; m < n4; m++) sum = (sum + r[4 * m]) + r2[4 * m];
    } else {
#pragma unroll 8
      for (int m = 0; m < n4; m++) sum = sum + r[4 * m];
    }
    // the quad's partials p0..p3 sit in lanes j = 0..3 of consecutive threads (per_q is a multiple of 4)
    const float p1 = __shfl_down(sum, 1, 4), p2 = __shfl_down(sum, 2, 4), p3 = __shfl_down(sum, 3, 4);
    const int icol = icol0 + c;
    if (j == 0 && icol < ncol) {
      float *o = q == 0 ? o_up : (q == 1 ? o_dn : o_dir);
      o[lev0 + (dl > 0 ? sl : -sl) + (size_t)nlev * icol] = ((sum + p1) + p2) + p3;  // dl = +-1
    }
  }
  __syncthreads();
}

// Columns per block for a solver whose column occupies `lanes` lanes: the count (1, 2 or 4, at most 512 lanes)
// that leaves the fewest idle lanes in the block's last wave -- the two-per-lane SW kernel's 112 lanes per column
// (224 g-points): 4 columns = 448 lanes = 7 full waves instead of 2 waves with 16 idle lanes each (C4 -5 %).
inline int columns_per_block(int lanes)
{
  int best = 1;
  double best_waste = 1e30;
  for (int k = 1; k <= 4; k *= 2) {
    if (k * lanes > 512) break;
    const double waste = (double)((k * lanes + 63) / 64 * 64) / (k * lanes);
    if (waste < best_waste - 1e-9) { best = k; best_waste = waste; }
  }
  return best;
}

// ------------------------------------------------------------------------------------------
// Column-local addressing.  Every solver array is (ngpt, n, ncol) with the column block uniform per
// workgroup, so each array gets a per-column buffer descriptor built from wave-uniform values: a
// load is `buffer_load v, voff=g*4, s_rsrc, soff=layer*ngpt*4` -- no per-lane 64-bit address math,
// the layer offset lives in an SGPR.
// ------------------------------------------------------------------------------------------
// A buffer offset past every solver array's range: raw buffer stores there are dropped, loads return 0 (the
// range check covers the VGPR offset; the SGPR layer offset is added past it), so idle lanes and padding steps
// can issue the same stores as the others without a branch.
static constexpr uint32_t kBufOOB = 0x7ffff000u;

struct ColArr {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ ColArr() = default;
  __device__ __forceinline__ ColArr(const float *base, size_t col_off, uint32_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc((void *)(base + col_off), 0, (int)bytes, 0x00020000)) {}  __device__ __forceinline__ float ld(uint32_t voff, uint32_t soff) const
  {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  }
  __device__ __forceinline__ void st(float v, uint32_t voff, uint32_t soff) const
  {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, 0);
  }
};

}  // namespace rrtmgpnn
