// kernels_clouds.hip -- all-sky additions for gfx950.
//
//  * cloud_optics_kernel : ty_cloud_optics%cloud_optics, LUT (compute_all_from_table) and Pade
//                          (compute_all_from_pade) forms, liquid + ice combined into 1scl or 2str
//                          by band (extensions/cloud_optics/mo_cloud_optics.F90:354-535, 603-775)
//  * increment_bybnd     : ty_optical_props_arry%increment of g-point properties by band-resolved
//                          ones (rte/mo_optical_props.F90:882-1023, kernels :358-484)
//  * delta_scale_2str    : delta_scale with f = g**2 (rte/kernels/mo_optical_props_kernels.F90:72-92)
//
// All three are elementwise: one thread per output element, the band (or g-point) index fastest so
// a wave's loads and stores are contiguous.  Expressions follow the reference term by term and the
// file is compiled with -ffp-contract=off, so results are bit-identical to the oracle/reference.
#include "internal.hpp"

#include <cfloat>
#include <cmath>

namespace rrtmgpnn {

struct CloudTab {
  // LUT: (nsize, nband) liquid, (nsize, nband) ice (already offset to the roughness in use)
  const float *lut[6];
  // Pade: (nband, nsizereg, ncoef) liquid / ice (offset to the roughness), bounds [nsizereg+1] x 6
  const float *pade[6];
  const float *sizreg[6];
  int lut_mode, nband, nsize_liq, nsize_ice, nsizereg;
  float radliq_lwr, radice_lwr, liq_step, ice_step;
};

// compute_all_from_table (:603-645) for one value
__device__ __forceinline__ void from_table(float lwp, float re, int nsteps, float step, float offset,
                                           const float *__restrict__ tt, const float *__restrict__ st,
                                           const float *__restrict__ at, int b, float &t, float &ts, float &tsg)
{
  int index = (int)floorf((re - offset) / step) + 1;
  index = min(index, nsteps - 1);
  const float fint = (re - offset) / step - (float)(index - 1);
  const int i = index - 1 + nsteps * b;
  t = lwp * (tt[i] + fint * (tt[i + 1] - tt[i]));
  ts = t * (st[i] + fint * (st[i + 1] - st[i]));
  tsg = ts * (at[i] + fint * (at[i + 1] - at[i]));
}

// pade_eval_1 (:750-775): c(nbnd, nrads, 0:m+n), irad 1-based
template <int M, int N>
__device__ __forceinline__ float pade_eval(int b, int nbnd, int nrads, int irad, float re, const float *__restrict__ c)
{
  auto C = [&](int i) { return c[b + nbnd * ((irad - 1) + nrads * i)]; };
  float denom = C(N + M);
#pragma unroll
  for (int i = N - 1 + M; i >= 1 + M; i--) denom = C(i) + re * denom;
  denom = 1.0f + re * denom;
  float numer = C(M);
#pragma unroll
  for (int i = M - 1; i >= 1; i--) numer = C(i) + re * numer;
  numer = C(0) + re * numer;
  return numer / denom;
}

// size regime of compute_all_from_pade (:684-697): min(floor((re - b(2))/b(3)) + 2, 3)
__device__ __forceinline__ int pade_irad(float re, const float *__restrict__ bounds)
{
  return min((int)floorf((re - bounds[1]) / bounds[2]) + 2, 3);
}

__device__ __forceinline__ void from_pade(float wp, float re, const CloudTab &c, int k, int b, float &t, float &ts,
                                          float &tsg)
{
  t = wp * pade_eval<2, 3>(b, c.nband, c.nsizereg, pade_irad(re, c.sizreg[3 * k]), re, c.pade[3 * k]);
  // Pade approximants for co-albedo can sometimes be negative (:690-692)
  ts = t * (1.0f - fmaxf(0.0f, pade_eval<2, 2>(b, c.nband, c.nsizereg, pade_irad(re, c.sizreg[3 * k + 1]), re,
                                                c.pade[3 * k + 1])));
  tsg = ts * pade_eval<2, 2>(b, c.nband, c.nsizereg, pade_irad(re, c.sizreg[3 * k + 2]), re, c.pade[3 * k + 2]);
}

// block = rpb (lay, col) rows x nband bands; a thread keeps its band and strides over rows
__global__ void cloud_optics_kernel(long long nrow, int rpb, CloudTab c, const float *__restrict__ clwp,
                                    const float *__restrict__ ciwp, const float *__restrict__ reliq,
                                    const float *__restrict__ reice, float *__restrict__ tau, float *__restrict__ ssa,
                                    float *__restrict__ g)
{
  const int b = threadIdx.x % c.nband, r0 = threadIdx.x / c.nband;
  if (r0 >= rpb) return;
  for (long long s = (long long)blockIdx.x * rpb + r0; s < nrow; s += (long long)gridDim.x * rpb) {
    const long long i = b + (long long)c.nband * s;
    float lt = 0.0f, lts = 0.0f, ltsg = 0.0f, it = 0.0f, its = 0.0f, itsg = 0.0f;
    const float lw = clwp[s], iw = ciwp[s];
    if (lw > 0.0f) {
      if (c.lut_mode) from_table(lw, reliq[s], c.nsize_liq, c.liq_step, c.radliq_lwr, c.lut[0], c.lut[1], c.lut[2], b, lt, lts, ltsg);
      else from_pade(lw, reliq[s], c, 0, b, lt, lts, ltsg);
    }
    if (iw > 0.0f) {
      if (c.lut_mode) from_table(iw, reice[s], c.nsize_ice, c.ice_step, c.radice_lwr, c.lut[3], c.lut[4], c.lut[5], b, it, its, itsg);
      else from_pade(iw, reice[s], c, 1, b, it, its, itsg);
    }
    if (!ssa) {
      tau[i] = (lt - lts) + (it - its);  // absorption optical depth (1scl, :497-505)
    } else {                             // 2str (:507-520)
      const float t = lt + it, ts = lts + its;
      g[i] = (ltsg + itsg) / fmaxf(FLT_EPSILON, ts);
      ssa[i] = ts / fmaxf(FLT_EPSILON, t);
      tau[i] = t;
    }
  }
}

static unsigned grid_for(rrtmgpnn_context *ctx, long long n, int threads)
{
  long long want = (n + threads - 1) / threads, cap = (long long)ctx->num_cus * 8;
  return (unsigned)(want < cap ? (want > 0 ? want : 1) : cap);
}

int launch_cloud_optics(rrtmgpnn_context *ctx, const rrtmgpnn_cloud_optics *co, int ncol, int nlay, const float *clwp,
                        const float *ciwp, const float *reliq, const float *reice, float *tau, float *ssa, float *g)
{
  const long long n = (long long)co->nband * nlay * ncol;
  if (n == 0) return RRTMGPNN_OK;
  CloudTab c{};
  const int r = co->icergh - 1;
  c.lut_mode = co->lut_mode;
  c.nband = co->nband;
  c.nsize_liq = co->nsize_liq;
  c.nsize_ice = co->nsize_ice;
  c.nsizereg = co->nsizereg;
  c.radliq_lwr = co->radliq_lwr;
  c.radice_lwr = co->radice_lwr;
  c.liq_step = co->liq_step;
  c.ice_step = co->ice_step;
  if (co->lut_mode) {
    for (int k = 0; k < 3; k++) c.lut[k] = co->d_tab + co->off[k];
    const size_t ice_stride = (size_t)co->nsize_ice * co->nband;
    for (int k = 3; k < 6; k++) c.lut[k] = co->d_tab + co->off[k] + ice_stride * r;
  } else {
    const size_t stride_ext = (size_t)co->nband * co->nsizereg * co->ncoef_ext;
    const size_t stride_ssa = (size_t)co->nband * co->nsizereg * co->ncoef_ssa;
    for (int k = 0; k < 3; k++) c.pade[k] = co->d_tab + co->off[k];
    c.pade[3] = co->d_tab + co->off[3] + stride_ext * r;
    c.pade[4] = co->d_tab + co->off[4] + stride_ssa * r;
    c.pade[5] = co->d_tab + co->off[5] + stride_ssa * r;
    for (int k = 0; k < 6; k++) c.sizreg[k] = co->d_tab + co->off[6 + k];
  }
  const long long nrow = (long long)nlay * ncol;
  const int rpb = 256 / co->nband;
  const long long want = (nrow + rpb - 1) / rpb, cap = (long long)ctx->num_cus * 8;
  hipLaunchKernelGGL(cloud_optics_kernel, dim3((unsigned)(want < cap ? want : cap)), dim3(rpb * co->nband), 0,
                     ctx->stream, nrow, rpb, c, clwp, ciwp, reliq, reice, tau, ssa, g);
  RRTMGPNN_LAUNCH_CHECK("cloud_optics_kernel");
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// increment by band (:358-484).  nstr_io / nstr_in: 1 (tau) or 2 (tau, ssa, g).
// ------------------------------------------------------------------------------------------
// One thread per g-point (block = ngpt rounded up to a wave), blocks striding over (lay, col) rows: the
// g-point's band is looked up once per thread and every row is a contiguous load/store of ngpt values.
template <int IO, int IN, bool kSame>
__global__ void increment_bybnd_kernel(long long nrow, int ngpt, int nbnd, BandArgs bands, float *__restrict__ tau1,
                                       float *__restrict__ ssa1, float *__restrict__ g1,
                                       const float *__restrict__ tau2, const float *__restrict__ ssa2,
                                       const float *__restrict__ g2)
{
  const float eps = 3.0f * FLT_MIN;  // 3*tiny(1.0_wp) (mo_optical_props_kernels.F90:31)
  const int igpt = threadIdx.x;
  if (igpt >= ngpt) return;
  int b = igpt;  // kSame: both sets at the same g-point resolution (increment_*_by_*, :109-219)
  if constexpr (!kSame) {
    b = -1;  // lims 1-based; a g-point in no band is left untouched
    for (int k = 0; k < bands.nbnd && b < 0; k++)
      if (igpt >= bands.lims[2 * k] - 1 && igpt < bands.lims[2 * k + 1]) b = k;
    if (b < 0) return;
  }
  const int nin = kSame ? ngpt : nbnd;
  for (long long r = blockIdx.x; r < nrow; r += gridDim.x) {
    const long long i = igpt + (long long)ngpt * r, ib = b + (long long)nin * r;
    if constexpr (IO == 1) {
      tau1[i] = IN == 1 ? tau1[i] + tau2[ib] : tau1[i] + tau2[ib] * (1.0f - ssa2[ib]);
    } else if constexpr (IN == 1) {
      const float tau12 = tau1[i] + tau2[ib];
      ssa1[i] = tau1[i] * ssa1[i] / fmaxf(eps, tau12);
      tau1[i] = tau12;
    } else {
      const float t1 = tau1[i], w1 = ssa1[i];
      const float tau12 = t1 + tau2[ib];
      const float tauscat12 = t1 * w1 + tau2[ib] * ssa2[ib];
      g1[i] = (t1 * w1 * g1[i] + tau2[ib] * ssa2[ib] * g2[ib]) / fmaxf(eps, tauscat12);
      ssa1[i] = tauscat12 / fmaxf(eps, tau12);
      tau1[i] = tau12;
    }
  }
}

template <bool kSame>
static void launch_inc(rrtmgpnn_context *ctx, long long nrow, int ngpt, const BandArgs &bands, float *tau1, float *ssa1,
                       float *g1, const float *tau2, const float *ssa2, const float *g2)
{
  const int threads = (ngpt + 63) / 64 * 64;
  const long long cap = (long long)ctx->num_cus * (2048 / threads);
  const dim3 grid((unsigned)(nrow < cap ? nrow : cap)), block(threads);
  const int nb = bands.nbnd;
  if (!ssa1 && !ssa2)
    hipLaunchKernelGGL((increment_bybnd_kernel<1, 1, kSame>), grid, block, 0, ctx->stream, nrow, ngpt, nb, bands, tau1, ssa1, g1, tau2, ssa2, g2);
  else if (!ssa1)
    hipLaunchKernelGGL((increment_bybnd_kernel<1, 2, kSame>), grid, block, 0, ctx->stream, nrow, ngpt, nb, bands, tau1, ssa1, g1, tau2, ssa2, g2);
  else if (!ssa2)
    hipLaunchKernelGGL((increment_bybnd_kernel<2, 1, kSame>), grid, block, 0, ctx->stream, nrow, ngpt, nb, bands, tau1, ssa1, g1, tau2, ssa2, g2);
  else
    hipLaunchKernelGGL((increment_bybnd_kernel<2, 2, kSame>), grid, block, 0, ctx->stream, nrow, ngpt, nb, bands, tau1, ssa1, g1, tau2, ssa2, g2);
}

// bands == nullptr: both sets at the same resolution (ngpt values per layer each)
int launch_increment_bybnd(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, const BandArgs *bands, float *tau1,
                           float *ssa1, float *g1, const float *tau2, const float *ssa2, const float *g2)
{
  const long long nrow = (long long)nlay * ncol;
  if (nrow == 0) return RRTMGPNN_OK;
  if (ngpt > 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "increment: more than 1024 g-points");
  if (bands) launch_inc<false>(ctx, nrow, ngpt, *bands, tau1, ssa1, g1, tau2, ssa2, g2);
  else launch_inc<true>(ctx, nrow, ngpt, BandArgs{}, tau1, ssa1, g1, tau2, ssa2, g2);
  RRTMGPNN_LAUNCH_CHECK("increment_bybnd_kernel");
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// delta_scale_2str_k (:72-92), f = g*g; delta_scale_2str_f_k (:41-70) when fwd is given
// ------------------------------------------------------------------------------------------
__global__ void delta_scale_kernel(long long n, float *__restrict__ tau, float *__restrict__ ssa, float *__restrict__ g,
                                   const float *__restrict__ fwd)
{
  const float eps = 3.0f * FLT_MIN;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float gi = g[i], si = ssa[i];
    const float f = fwd ? fwd[i] : gi * gi, wf = si * f;
    tau[i] = (1.0f - wf) * tau[i];
    ssa[i] = (si - wf) / fmaxf(eps, 1.0f - wf);
    g[i] = (gi - f) / fmaxf(eps, 1.0f - f);
  }
}

int launch_delta_scale(rrtmgpnn_context *ctx, long long n, float *tau, float *ssa, float *g, const float *fwd)
{
  if (n == 0) return RRTMGPNN_OK;
  hipLaunchKernelGGL(delta_scale_kernel, dim3(grid_for(ctx, n, 256)), dim3(256), 0, ctx->stream, n, tau, ssa, g, fwd);
  RRTMGPNN_LAUNCH_CHECK("delta_scale_kernel");
  return RRTMGPNN_OK;
}

}  // namespace rrtmgpnn
