// kernels_rte.hip -- Planck source and RTE solvers for gfx950 (MI355X).
//
// Layout: g-point fastest, exactly the reference's (ngpt, nlay[+1], ncol) arrays.  One block per
// column, one lane per g-point: every layer step of a wave reads 64 consecutive g-points
// (256 B, coalesced), and the vertical recurrence runs in registers.  Broadband fluxes are
// reduced in-kernel (wave shuffle -> per-wave LDS partials -> fixed-order sum: deterministic).
//
//  * planck_source_kernel : compute_Planck_source_nn (rrtmgp/kernels/mo_gas_optics_kernels.F90:615-683)
//  * lw_noscat_kernel     : lw_solver_noscat[_GaussQuad] (rte/kernels/mo_rte_solver_kernels.F90:119-415)
//  * sw_2stream kernels   : sw_solver_2stream + sw_two_stream_source + adding (:541-692, :1366-1637)
#include "internal.hpp"
#include "libm_ref.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>

namespace rrtmgpnn {

static constexpr float kPi = 3.14159265358979323846f;

// Ablation switches for tools/ablate_solvers.sh (never set in the product build): they break parity
// on purpose to attribute solver time.  RRTMGPNN_ABL_NATIVE_EXP: device expf instead of ref_expf;
// RRTMGPNN_ABL_NO_REDUCE: skip the ordered broadband reduction (barriers kept);
// RRTMGPNN_ABL_NO_BARRIER: skip staging and flushing entirely.
#ifdef RRTMGPNN_ABL_NATIVE_EXP
#define ref_expf_tab(x, t) __expf(x)
#endif

__device__ __forceinline__ float wave_sum(float v)
{
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ------------------------------------------------------------------------------------------
// Planck source.  grid (nlay, ncol), block >= ngpt.  The block of layer `ilay` owns pfrac(:,ilay)
// and also writes lev_source(:,nlay+1) (ilay == nlay-1) and the surface sources (ilay == sfc_lay-1)
// from its in-register pfrac, before pfrac is overwritten with lay_source (no cross-block race).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float interp1d(float val, float offset, float delta, int ntemp, const float *__restrict__ t)
{
  float val0 = (val - offset) / delta;
  int iv = (int)val0;  // Fortran int(): truncation
  float frac = val0 - (float)iv;
  int index = min(ntemp - 1, max(1, iv + 1));
  float lo = t[index - 1], hi = t[index];
  return lo + frac * (hi - lo);
}

__device__ __forceinline__ int band_of(const BandArgs &b, int g)
{
  for (int i = 0; i < b.nbnd; i++)
    if (g >= b.lims[2 * i] - 1 && g < b.lims[2 * i + 1]) return i;
  return 0;
}

constexpr int kPlanckLayers = 4;  // layers per block: independent loads in flight per lane

__global__ void planck_source_kernel(int ncol, int nlay, int ngpt, int ntemp, const float *__restrict__ tlay,
                                     const float *__restrict__ tlev, const float *__restrict__ tsfc, int sfc_lay,
                                     BandArgs bands, float tmin, float tdelta, const float *__restrict__ totplnk,
                                     float *__restrict__ sfc_src, float *__restrict__ sfc_jac, float *__restrict__ pfrac,
                                     float *__restrict__ lev_src)
{
  const int l0 = blockIdx.x * kPlanckLayers, icol = blockIdx.y, g = threadIdx.x;
  if (g >= ngpt) return;
  const int b = band_of(bands, g);
  const float *tab = totplnk + (size_t)ntemp * b;
  const float *tl = tlev + (size_t)(nlay + 1) * icol;
  float pf[kPlanckLayers];
#pragma unroll
  for (int k = 0; k < kPlanckLayers; k++) {
    const int ilay = min(l0 + k, nlay - 1);
    pf[k] = pfrac[(size_t)g + (size_t)ngpt * (ilay + (size_t)nlay * icol)];
  }
#pragma unroll
  for (int k = 0; k < kPlanckLayers; k++) {
    const int ilay = l0 + k;
    if (ilay >= nlay) break;
    const size_t il = (size_t)g + (size_t)ngpt * (ilay + (size_t)nlay * icol);
    const size_t iv = (size_t)g + (size_t)ngpt * (ilay + (size_t)(nlay + 1) * icol);
    lev_src[iv] = pf[k] * interp1d(tl[ilay], tmin, tdelta, ntemp, tab);
    if (ilay == nlay - 1) lev_src[iv + ngpt] = pf[k] * interp1d(tl[nlay], tmin, tdelta, ntemp, tab);
    if (ilay == sfc_lay - 1) {
      float ts = tsfc[icol];
      float ps = interp1d(ts, tmin, tdelta, ntemp, tab);
      float pj = interp1d(ts + 1.0f, tmin, tdelta, ntemp, tab);
      sfc_src[g + (size_t)ngpt * icol] = pf[k] * ps;
      sfc_jac[g + (size_t)ngpt * icol] = pf[k] * (pj - ps);
    }
    pfrac[il] = pf[k] * interp1d(tlay[ilay + (size_t)nlay * icol], tmin, tdelta, ntemp, tab);
  }
}

int launch_planck_source(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ntemp, const float *tlay,
                         const float *tlev, const float *tsfc, int sfc_lay, const BandArgs &bands, float temp_ref_min,
                         float totplnk_delta, const float *totplnk, float *sfc_source, float *sfc_source_Jac,
                         float *pfrac, float *lev_source)
{
  if (ncol == 0 || nlay == 0) return RRTMGPNN_OK;
  if (ngpt > 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "planck source: ngpt > 1024");
  int threads = (ngpt + 63) / 64 * 64;
  hipLaunchKernelGGL(planck_source_kernel, dim3((nlay + kPlanckLayers - 1) / kPlanckLayers, ncol), dim3(threads), 0, ctx->stream, ncol, nlay, ngpt, ntemp,
                     tlay, tlev, tsfc, sfc_lay, bands, temp_ref_min, totplnk_delta, totplnk, sfc_source,
                     sfc_source_Jac, pfrac, lev_source);
  RRTMGPNN_LAUNCH_CHECK("planck_source_kernel");
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// Ordered broadband reduction.  The reference sums g-points into 4 interleaved partial sums,
// partial j accumulating g = j, j+4, j+8, ... in increasing g, then ((p0+p1)+p2)+p3
// (rte/kernels/mo_rte_solver_kernels.F90:296-318 LW, :643-686 SW).  A float32 tree reduction
// differs from that by several ulp of the broadband flux (~1e-3 W/m2 at SW magnitudes), so the
// kernels reproduce the reference's order exactly: each level's per-g values are staged in an
// LDS ring of kRing levels; when it fills, 4*kRing*NQ threads each walk one (quantity, level,
// partial) sequentially.  Deterministic and order-identical to the reference.
// ------------------------------------------------------------------------------------------
static constexpr int kRing = 8;
static constexpr int kPF = 4;
static constexpr int kExpTabOff = 0, kExpTabFloats = 64;  // exp table (32 x u64) at the front of LDS  // layers of inputs kept in flight per lane (software prefetch)

// Flush `nfill` staged levels.  ring: [nq][kRing][ngpt]; part: [nq][nlev][4]; slot_lev[c] = level.
// One thread per (quantity, level) walks the level's g-points with 16-byte LDS reads: element k of
// the float4 at m is g = 4m + k, so the 4 interleaved partials advance together, each in g order.
// dn_mode (SW): quantity 1 is accumulated as (s + ring1) + ring2, i.e. sums_dn + radn_dn + radn_dir.
// ngpt % 4 != 0: the reference uses sum(radn, 1) instead (one sequential sum, kept in partial 0).
__device__ __forceinline__ void ring_flush(const float *ring, float *part, const int *slot_lev, int nq, int nfill,
                                           int ngpt, int nlev, bool accumulate, bool dn_mode)
{
  __syncthreads();
  const int t = threadIdx.x;
#ifdef RRTMGPNN_ABL_NO_REDUCE
  if (false) {
#else
  if (t < nq * nfill) {
#endif
    const int q = t / nfill, c = t % nfill;
    const float *r = ring + ((size_t)q * kRing + c) * ngpt;
    const float *r2 = ring + ((size_t)2 * kRing + c) * ngpt;
    const bool dn = dn_mode && q == 1;
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    if ((ngpt & 3) == 0) {
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
    float *p = part + ((size_t)q * nlev + slot_lev[c]) * 4;
    if (accumulate) { p[0] += s0; p[1] += s1; p[2] += s2; p[3] += s3; }
    else { p[0] = s0; p[1] = s1; p[2] = s2; p[3] = s3; }
  }
  __syncthreads();
}

__device__ __forceinline__ float combine4(const float *p) { return ((p[0] + p[1]) + p[2]) + p[3]; }

// ------------------------------------------------------------------------------------------
// LW no-scattering solver.  block = one column, lane = g-point.  The down pass stores nothing: the
// up pass re-reads tau/lay/lev for its layer (L2/MALL-hot) and recomputes trans and the source,
// bitwise identical to the down pass' values.  Source indexing follows lw_source_noscat
// (:742-776): source_dn uses lev(l+1), source_up uses lev(l) for EVERY orientation (quirk B-1).
// LDS: ring [kRing][ngpt], part [2][nlev][4], slot_lev [kRing].
// ------------------------------------------------------------------------------------------
struct LwAngles {
  float D[4], w[4];
  int nmus;
};

__global__ void lw_noscat_kernel(int ngpt, int nlay, int ncol, int top_at_1, LwAngles ang,
                                 const float *__restrict__ inc_flux, const float *__restrict__ tau,
                                 const float *__restrict__ lay, const float *__restrict__ lev,
                                 const float *__restrict__ emis, const float *__restrict__ sfc,
                                 float *__restrict__ ws, float *__restrict__ flux_up, float *__restrict__ flux_dn)
{
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int icol = blockIdx.x, g = threadIdx.x;
  const bool on = g < ngpt;
  const int gc = on ? g : ngpt - 1;  // clamped g-point for unconditional loads
  const int nlev = nlay + 1;
  // nmus > 1 (lw_solver_noscat_GaussQuad :383-412): g-point fluxes are summed over angles first, then
  // reduced with sum_broadband's plain sequential sum; ws holds the per-g accumulators (2, nlev, ngpt).
  const bool multi = ang.nmus > 1;
  float *wcol = multi ? ws + (size_t)2 * nlev * ngpt * icol : nullptr;
  float *ring = smem + kExpTabFloats;            // [kRing][ngpt]
  float *part = ring + (size_t)kRing * ngpt;     // [2][nlev][4]: 0 = dn, 1 = up
  int *slot_lev = (int *)(part + (size_t)2 * nlev * 4);
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);  // 16-byte aligned slot at the front
  load_exp_table(etab);
  __syncthreads();
  const float tau_thresh = sqrtf(FLT_EPSILON);
  const size_t cl = (size_t)ngpt * nlay * icol, cv = (size_t)ngpt * nlev * icol;
  const float e = on ? emis[g + (size_t)ngpt * icol] : 0.0f;
  const float ss = on ? sfc[g + (size_t)ngpt * icol] : 0.0f;
  const float inc = (on && inc_flux) ? inc_flux[g + (size_t)ngpt * icol] : 0.0f;
  const int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0;
  int nfill = 0;
  auto stage = [&](float v, int level, float *pq, bool acc) {
    if (multi) {
      if (on) {
        float *w = wcol + (size_t)(pq == part ? 0 : nlev) * ngpt + (size_t)level * ngpt + g;
        *w = acc ? *w + v : v;
      }
      return;
    }
    if (on) ring[(size_t)nfill * ngpt + g] = v;
    if (g == 0) slot_lev[nfill] = level;
#ifdef RRTMGPNN_ABL_NO_BARRIER
    return;
#endif
    if (++nfill == kRing) {
      ring_flush(ring, pq, slot_lev, 1, nfill, ngpt, nlev, acc, false);
      nfill = 0;
    }
  };
  auto drain = [&](float *pq, bool acc) {
    if (multi) return;
    if (nfill) ring_flush(ring, pq, slot_lev, 1, nfill, ngpt, nlev, acc, false);
    nfill = 0;
  };
  float *pdn = part, *pup = part + (size_t)nlev * 4;

  for (int imu = 0; imu < ang.nmus; imu++) {
    const float D = ang.D[imu];
    // radiance -> flux factor inside the broadband sum; with nmus == 1 and ngpt % 4 != 0 the reference
    // sums plain radiances (quirk B-5, mo_rte_solver_kernels.F90:287-320)
    const float fac = (multi || (ngpt & 3) == 0) ? 2.0f * kPi * ang.w[imu] : 1.0f;
    const bool acc = imu > 0;
    float I = inc / (2.0f * kPi * ang.w[imu]);
    stage(fac * I, top, pdn, acc);
    // downward: lw_transport_noscat_dn (:982-1009).  Inputs of layer step j+kPF are loaded while step
    // j computes (loads are unconditional on clamped indices: no branch around a load).
    {
      float pt[kPF], py[kPF], pv[kPF];
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int l = top_at_1 ? min(p, nlay - 1) : max(nlay - 1 - p, 0);
        const size_t i = (size_t)gc + (size_t)ngpt * l;
        pt[p] = tau[cl + i]; py[p] = lay[cl + i]; pv[p] = lev[cv + i + ngpt];
      }
      for (int j0 = 0; j0 < nlay; j0 += kPF) {
#pragma unroll
        for (int p = 0; p < kPF; p++) {
          const int j = j0 + p;
          if (j < nlay) {
            const int l = top_at_1 ? j : nlay - 1 - j;
            const float t = pt[p] * D, ly = py[p], lvdn = pv[p];
            {
              const int jn = min(j + kPF, nlay - 1), ln = top_at_1 ? jn : nlay - 1 - jn;
              const size_t i = (size_t)gc + (size_t)ngpt * ln;
              pt[p] = tau[cl + i]; py[p] = lay[cl + i]; pv[p] = lev[cv + i + ngpt];
            }
            float T = ref_expf_tab(-t, etab);
            float fact = (t > tau_thresh) ? (1.0f - T) / t - T : t * (0.5f - 1.0f / 3.0f * t);
            float S = (1.0f - T) * lvdn + 2.0f * fact * (ly - lvdn);
            I = T * I + S;
            stage(fac * I, top_at_1 ? l + 1 : l, pdn, acc);
          }
        }
      }
    }
    drain(pdn, acc);
    // surface reflection and emission (:269)
    float U = I * (1.0f - e) + e * ss;
    stage(fac * U, sfcl, pup, acc);
    // upward: lw_transport_noscat_up (:950-980)
    {
      float pt[kPF], py[kPF], pv[kPF];
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int l = top_at_1 ? max(nlay - 1 - p, 0) : min(p, nlay - 1);
        const size_t i = (size_t)gc + (size_t)ngpt * l;
        pt[p] = tau[cl + i]; py[p] = lay[cl + i]; pv[p] = lev[cv + i];
      }
      for (int j0 = 0; j0 < nlay; j0 += kPF) {
#pragma unroll
        for (int p = 0; p < kPF; p++) {
          const int j = j0 + p;
          if (j < nlay) {
            const int l = top_at_1 ? nlay - 1 - j : j;
            const float t = pt[p] * D, ly = py[p], lvup = pv[p];
            {
              const int jn = min(j + kPF, nlay - 1), ln = top_at_1 ? nlay - 1 - jn : jn;
              const size_t i = (size_t)gc + (size_t)ngpt * ln;
              pt[p] = tau[cl + i]; py[p] = lay[cl + i]; pv[p] = lev[cv + i];
            }
            float T = ref_expf_tab(-t, etab);
            float fact = (t > tau_thresh) ? (1.0f - T) / t - T : t * (0.5f - 1.0f / 3.0f * t);
            float S = (1.0f - T) * lvup + 2.0f * fact * (ly - lvup);
            U = T * U + S;
            stage(fac * U, top_at_1 ? l : l + 1, pup, acc);
          }
        }
      }
    }
    drain(pup, acc);
  }
  if (multi) {
    __syncthreads();
    for (int t = g; t < 2 * nlev; t += blockDim.x) {
      const float *w = wcol + (size_t)t * ngpt;
      float s = 0.0f;
      for (int i = 0; i < ngpt; i++) s = s + w[i];  // sum_broadband: sequential over g
      const int l = t % nlev;
      (t < nlev ? flux_dn : flux_up)[l + (size_t)nlev * icol] = s;
    }
    return;
  }
  for (int l = g; l < nlev; l += blockDim.x) {
    flux_dn[l + (size_t)nlev * icol] = combine4(pdn + 4 * l);
    flux_up[l + (size_t)nlev * icol] = combine4(pup + 4 * l);
  }
}

int launch_lw_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus, const float *Ds,
                     const float *wts, const float *inc_flux, const float *tau, const float *lay_source,
                     const float *lev_source, const float *sfc_emis, const float *sfc_source, float *flux_up,
                     float *flux_dn)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (nmus < 1 || nmus > 4) return fail(RRTMGPNN_ERR_ARGUMENT, "lw solver: nmus must be 1..4");
  if (ngpt > 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw solver: ngpt > 1024");
  LwAngles a{};
  a.nmus = nmus;
  for (int i = 0; i < nmus; i++) { a.D[i] = Ds[i]; a.w[i] = wts[i]; }
  int threads = (ngpt + 63) / 64 * 64;
  size_t lds = sizeof(float) * (kExpTabFloats + (size_t)kRing * ngpt + (size_t)2 * (nlay + 1) * 4) + sizeof(int) * kRing;
  if (lds > 64 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw solver: too many layers for LDS partials");
  void *ws = nullptr;
  if (nmus > 1) {
    int rc = ctx->workspace(sizeof(float) * 2 * (size_t)ngpt * (nlay + 1) * ncol, &ws);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(lw_noscat_kernel, dim3(ncol), dim3(threads), lds, ctx->stream, ngpt, nlay, ncol, top_at_1, a,
                     inc_flux, tau, lay_source, lev_source, sfc_emis, sfc_source, (float *)ws, flux_up, flux_dn);
  RRTMGPNN_LAUNCH_CHECK("lw_noscat_kernel");
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// SW two-stream solver.  block = one column, lane = g-point.
//   pass 1 (top->bottom): direct beam F_dir per level -> workspace
//   pass 2 (bottom->top): sw_two_stream_source coefficients (Tnoscat recomputed bit-identically
//          from tau and mu0), adding's albedo/src/denom (Shonk & Hogan Eqs 9-11); stores per level
//          alpha and src only
//   pass 3 (top->bottom): recomputes the layer coefficients (same bits as pass 2: memory traffic is
//          the bound, arithmetic is spare) and runs Eqs 12-13 with the reference's exact expression
//          order; direct beam recomputed; ordered broadband sums of up, dif+dir, dir.
// Workspace ws: 2 arrays (ngpt, nlay+1, ncol): [F_dir -> alpha], src.
// ------------------------------------------------------------------------------------------
struct SwCoef {
  float Rdif, Tdif, Sup, Sdn, Tnoscat;
};

__device__ __forceinline__ SwCoef sw_two_stream(float tau, float w0, float g, float mu0, float mu0_inv, float dir_inc,
                                               const uint64_t *etab)
{
  const float k_min = 1.e-4f, eps = FLT_EPSILON;
  SwCoef c;
  float Tnoscat = ref_expf_tab(-tau * mu0_inv, etab);
  float gamma1 = (8.0f - w0 * (5.0f + 3.0f * g)) * .25f;
  float gamma2 = 3.0f * (w0 * (1.0f - g)) * .25f;
  float gamma3 = (2.0f - 3.0f * mu0 * g) * .25f;
  float gamma4 = 1.0f - gamma3;
  float alpha1 = gamma1 * gamma4 + gamma2 * gamma3;
  float alpha2 = gamma1 * gamma3 + gamma2 * gamma4;
  float k = sqrtf(fmaxf((gamma1 - gamma2) * (gamma1 + gamma2), k_min));
  float emk = ref_expf_tab(-tau * k, etab);
  float em2k = emk * emk;
  float k2e = 2.0f * k * emk;
  float RT = 1.0f / (k * (1.0f + em2k) + gamma1 * (1.0f - em2k));
  c.Rdif = RT * gamma2 * (1.0f - em2k);
  c.Tdif = RT * 2.0f * k * emk;
  float k_mu = k * mu0, k_mu2 = k_mu * k_mu, k_g3 = k * gamma3, k_g4 = k * gamma4;
  float dd = (fabsf(1.0f - k_mu2) >= eps) ? (1.0f - k_mu2) : eps;
  RT = w0 * RT / dd;
  float Rdir = RT * ((1.0f - k_mu) * (alpha2 + k_g3) - (1.0f + k_mu) * (alpha2 - k_g3) * em2k -
                     k2e * (gamma3 - alpha2 * mu0) * Tnoscat);
  float Tdir = RT * (k2e * (gamma4 + alpha1 * mu0) -
                     Tnoscat * ((1.0f + k_mu) * (alpha1 + k_g4) - (1.0f - k_mu) * (alpha1 - k_g4) * em2k));
  Rdir = fmaxf(0.0f, fminf(Rdir, (1.0f - Tnoscat)));
  Tdir = fmaxf(0.0f, fminf(Tdir, (1.0f - Tnoscat - Rdir)));
  c.Sup = Rdir * dir_inc;
  c.Sdn = Tdir * dir_inc;
  c.Tnoscat = Tnoscat;
  return c;
}

__global__ void sw_2stream_kernel(int ngpt, int nlay, int ncol, int top_at_1, const float *__restrict__ inc_flux,
                                  const float *__restrict__ inc_dif, const float *__restrict__ tau,
                                  const float *__restrict__ ssa, const float *__restrict__ gg,
                                  const float *__restrict__ mu0p, const float *__restrict__ alb_dir,
                                  const float *__restrict__ alb_dif, float *__restrict__ ws,
                                  float *__restrict__ flux_up, float *__restrict__ flux_dn, float *__restrict__ flux_dir)
{
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int icol = blockIdx.x, g = threadIdx.x;
  const bool on = g < ngpt;
  const int nlev = nlay + 1;
  float *ring = smem + kExpTabFloats;              // [3][kRing][ngpt]: up, dif, dir
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  load_exp_table(etab);
  __syncthreads();
  float *part = ring + (size_t)3 * kRing * ngpt;   // [3][nlev][4]: up, dn, dir
  int *slot_lev = (int *)(part + (size_t)3 * nlev * 4);
  const size_t cl = (size_t)ngpt * nlay * icol, cv = (size_t)ngpt * nlev * icol;
  const size_t plane = (size_t)ngpt * nlev * ncol;
  float *wA = ws + cv, *wS = ws + plane + cv;
  const float mu0 = mu0p[icol], mu0_inv = 1.0f / mu0;
  // "layer l spans levels l (top side) and l+1" when top_at_1, else l+1 (top) and l
  auto lev_above = [&](int l) { return top_at_1 ? l : l + 1; };
  auto lev_below = [&](int l) { return top_at_1 ? l + 1 : l; };
  auto lay_of_down = [&](int j) { return top_at_1 ? j : nlay - 1 - j; };  // j-th layer from the top
  auto lay_of_up = [&](int j) { return top_at_1 ? nlay - 1 - j : j; };    // j-th layer from the surface
  const int gc = on ? g : ngpt - 1;  // clamped g-point for unconditional loads
  const int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0;
  const float Ftop = on ? inc_flux[g + (size_t)ngpt * icol] * mu0 : 0.0f;

  // ---- pass 1: direct beam (only tau is read) ----
  float Fd = Ftop;
  if (on) wA[(size_t)g + (size_t)ngpt * top] = Fd;
  {
    float pt[kPF];
#pragma unroll
    for (int p = 0; p < kPF; p++) pt[p] = tau[cl + (size_t)gc + (size_t)ngpt * lay_of_down(min(p, nlay - 1))];
    for (int j0 = 0; j0 < nlay; j0 += kPF) {
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int j = j0 + p;
        if (j < nlay) {
          const int l = lay_of_down(j);
          const float t = pt[p];
          pt[p] = tau[cl + (size_t)gc + (size_t)ngpt * lay_of_down(min(j + kPF, nlay - 1))];
          Fd = ref_expf_tab(-t * mu0_inv, etab) * Fd;
          if (on) wA[(size_t)g + (size_t)ngpt * lev_below(l)] = Fd;
        }
      }
    }
  }
  // ---- pass 2: bottom -> top adding (albedo, src) ----
  float alb_b = on ? alb_dif[g + (size_t)ngpt * icol] : 0.0f;  // albedo at the level below
  float src_b = on ? Fd * alb_dir[g + (size_t)ngpt * icol] : 0.0f;
  if (on) {
    wA[(size_t)g + (size_t)ngpt * sfcl] = alb_b;
    wS[(size_t)g + (size_t)ngpt * sfcl] = src_b;
  }
  {
    float pt[kPF], pw[kPF], pg[kPF];
#pragma unroll
    for (int p = 0; p < kPF; p++) {
      const size_t i = cl + (size_t)gc + (size_t)ngpt * lay_of_up(min(p, nlay - 1));
      pt[p] = tau[i]; pw[p] = ssa[i]; pg[p] = gg[i];
    }
    for (int j0 = 0; j0 < nlay; j0 += kPF) {
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int j = j0 + p;
        if (j < nlay) {
          const int l = lay_of_up(j);
          const float t = pt[p], w0 = pw[p], g0 = pg[p];
          {
            const size_t i = cl + (size_t)gc + (size_t)ngpt * lay_of_up(min(j + kPF, nlay - 1));
            pt[p] = tau[i]; pw[p] = ssa[i]; pg[p] = gg[i];
          }
          const size_t ia = (size_t)gc + (size_t)ngpt * lev_above(l);
          const float Fin = wA[ia];
          SwCoef c = sw_two_stream(t, w0, g0, mu0, mu0_inv, Fin, etab);
          float denom = 1.0f / (1.0f - c.Rdif * alb_b);
          float alb = c.Rdif + c.Tdif * c.Tdif * alb_b * denom;
          float src = c.Sup + c.Tdif * denom * (src_b + alb_b * c.Sdn);
          if (on) {
            wA[ia] = alb;
            wS[ia] = src;
          }
          alb_b = alb;
          src_b = src;
        }
      }
    }
  }
  // ---- pass 3: top -> bottom fluxes + ordered broadband sums ----
  int nfill = 0;
  auto stage = [&](float up, float dif, float dir, int level) {
    if (on) {
      ring[(size_t)nfill * ngpt + g] = up;
      ring[((size_t)kRing + nfill) * ngpt + g] = dif;
      ring[((size_t)2 * kRing + nfill) * ngpt + g] = dir;
    }
    if (g == 0) slot_lev[nfill] = level;
#ifdef RRTMGPNN_ABL_NO_BARRIER
    return;
#endif
    if (++nfill == kRing) {
      ring_flush(ring, part, slot_lev, 3, nfill, ngpt, nlev, false, true);
      nfill = 0;
    }
  };
  float Fdn = (on && inc_dif) ? inc_dif[g + (size_t)ngpt * icol] : 0.0f;
  Fd = Ftop;
  stage(Fdn * alb_b + src_b, Fdn, Fd, top);  // Eq 12 at the top; alb_b/src_b hold the top level's values
  {
    float pt[kPF], pw[kPF], pg[kPF], pa[kPF], ps[kPF];
#pragma unroll
    for (int p = 0; p < kPF; p++) {
      const int l = lay_of_down(min(p, nlay - 1));
      const size_t i = cl + (size_t)gc + (size_t)ngpt * l, ib = (size_t)gc + (size_t)ngpt * lev_below(l);
      pt[p] = tau[i]; pw[p] = ssa[i]; pg[p] = gg[i]; pa[p] = wA[ib]; ps[p] = wS[ib];
    }
    for (int j0 = 0; j0 < nlay; j0 += kPF) {
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int j = j0 + p;
        if (j < nlay) {
          const int l = lay_of_down(j);
          const float t = pt[p], w0 = pw[p], g0 = pg[p], alb = pa[p], src = ps[p];
          {
            const int ln = lay_of_down(min(j + kPF, nlay - 1));
            const size_t i = cl + (size_t)gc + (size_t)ngpt * ln, ib = (size_t)gc + (size_t)ngpt * lev_below(ln);
            pt[p] = tau[i]; pw[p] = ssa[i]; pg[p] = gg[i]; pa[p] = wA[ib]; ps[p] = wS[ib];
          }
          // recompute the layer's coefficients exactly as pass 2 did (same inputs, same F_dir -> same bits)
          SwCoef c = sw_two_stream(t, w0, g0, mu0, mu0_inv, Fd, etab);
          const float denom = 1.0f / (1.0f - c.Rdif * alb);
          Fdn = (c.Tdif * Fdn + c.Rdif * src + c.Sdn) * denom;  // Eq 13 (adding :1583-1591)
          const float up = Fdn * alb + src;                      // Eq 12
          Fd = c.Tnoscat * Fd;
          stage(up, Fdn, Fd, lev_below(l));
        }
      }
    }
  }
  if (nfill) ring_flush(ring, part, slot_lev, 3, nfill, ngpt, nlev, false, true);
  for (int l = g; l < nlev; l += blockDim.x) {
    flux_up[l + (size_t)nlev * icol] = combine4(part + 4 * l);
    flux_dn[l + (size_t)nlev * icol] = combine4(part + (size_t)nlev * 4 + 4 * l);
    flux_dir[l + (size_t)nlev * icol] = combine4(part + (size_t)2 * nlev * 4 + 4 * l);
  }
}

int launch_sw_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                      const float *inc_flux_dif, const float *tau, const float *ssa, const float *g, const float *mu0,
                      const float *alb_dir, const float *alb_dif, float *flux_up, float *flux_dn, float *flux_dir)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (ngpt > 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: ngpt > 1024");
  void *ws = nullptr;
  int rc = ctx->workspace(sizeof(float) * 2 * (size_t)ngpt * (nlay + 1) * ncol, &ws);
  if (rc) return rc;
  int threads = (ngpt + 63) / 64 * 64;
  size_t lds = sizeof(float) * (kExpTabFloats + (size_t)3 * kRing * ngpt + (size_t)3 * (nlay + 1) * 4) + sizeof(int) * kRing;
  if (lds > 64 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: too many layers for LDS partials");
  hipLaunchKernelGGL(sw_2stream_kernel, dim3(ncol), dim3(threads), lds, ctx->stream, ngpt, nlay, ncol, top_at_1,
                     inc_flux, inc_flux_dif, tau, ssa, g, mu0, alb_dir, alb_dif, (float *)ws, flux_up, flux_dn,
                     flux_dir);
  RRTMGPNN_LAUNCH_CHECK("sw_2stream_kernel");
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// expand band -> g-point (rte/mo_rte_lw.F90:429-447)
// ------------------------------------------------------------------------------------------
__global__ void expand_kernel(int nband, int ngpt, int ncol, BandArgs b, const float *__restrict__ in,
                              float *__restrict__ out)
{
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)ngpt * ncol) return;
  int g = (int)(i % ngpt), icol = (int)(i / ngpt);
  int bd = -1;
  for (int k = 0; k < b.nbnd; k++)
    if (g >= b.lims[2 * k] - 1 && g < b.lims[2 * k + 1]) { bd = k; break; }
  if (bd >= 0) out[i] = in[bd + (size_t)nband * icol];
}

int launch_expand(rrtmgpnn_context *ctx, int nband, int ngpt, int ncol, const BandArgs &bands, const float *in,
                  float *out)
{
  long long n = (long long)ngpt * ncol;
  if (n == 0) return RRTMGPNN_OK;
  hipLaunchKernelGGL(expand_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, nband, ngpt, ncol,
                     bands, in, out);
  RRTMGPNN_LAUNCH_CHECK("expand_kernel");
  return RRTMGPNN_OK;
}

}  // namespace rrtmgpnn
