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
#include "rte_device.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>

namespace rrtmgpnn {

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
// Solver tuning (the ordered broadband reduction and buffer addressing live in rte_device.hpp).
// ------------------------------------------------------------------------------------------
// Solver constants (each chosen by A/B on one box, rounds 1-3):
//   kRing / kRingSw : levels staged in LDS per ordered flush (LW, one-g-point-per-lane SW);
//   k*Pf            : layers of inputs kept in flight per lane (software prefetch) -- LW, fused LW, SW;
//   __launch_bounds__(256, 8): 8 waves per SIMD, blocks of at most 256 threads (one column, lane = g-point).
#define LW_BOUNDS __launch_bounds__(256, 8)
#define SW_BOUNDS __launch_bounds__(256, 8)
static constexpr int kRing = 8, kRingSw = 6;
static constexpr int kLwPf = 4, kLwfPf = 2, kSwPf = 2;
// ring_flush_lanes walks slot s's 4 partials with lanes 4s .. 4s+3: a flush of kRing slots needs 4 * kRing lanes, and
// the smallest LW block (ngpt <= 64) has 64
static_assert(4 * kRing <= 64, "the LW ring's lane-per-partial flush needs 4 lanes per slot within one wave");
// LW no-scattering flush: one lane per partial sum over ring rows padded by 4 floats when ngpt % 4 == 0 (the float4
// walk of ring_flush over unpadded rows otherwise)
__host__ __device__ constexpr int lw_ring_stride(int ngpt) { return (ngpt & 3) == 0 ? ngpt + 4 : ngpt; }
static constexpr int kLwMaxG = 256, kSwMaxG = 256;  // g-points per column block
// ------------------------------------------------------------------------------------------
// LW no-scattering solver.  block = one column, lane = g-point.  The down pass stores nothing: the
// up pass re-reads its layer's inputs (L2/MALL-hot) and recomputes trans and the source, bitwise
// identical to the down pass' values.  Source indexing follows lw_source_noscat (:742-776):
// source_dn uses lev(l+1), source_up uses lev(l) for EVERY orientation (quirk B-1).
//
// Layers are walked in chunks of kRing: each chunk's levels are staged in LDS slots with static
// indices (the chunk loop is unrolled) and reduced by one ring_flush at the chunk end, so the
// recurrence never branches around a flush.  Inputs run kPF layers ahead of the recurrence.
//
// kFused: the Planck sources are not read from lay_source/lev_source but formed in-kernel from the
// Planck fraction exactly as compute_Planck_source_nn (mo_gas_optics_kernels.F90:615-683) forms
// them -- lay(g,l) = pfrac(g,l)*B_b(tlay(l)), lev(g,l) = pfrac(g,min(l,nlay-1))*B_b(tlev(l)),
// sfc(g) = pfrac(g,sfc_lay)*B_b(tsfc) -- with the band Planck values B_b interpolated once per
// column into LDS.  Same products, same bits; the source arrays never touch HBM.
// LDS: etab | [fused: B [nbnd][2*nlay+1], Bsfc[nbnd]] | ring [kRing][ngpt] | part [2][nlev][4]
// ------------------------------------------------------------------------------------------


// kInc: tau is incremented by a band-resolved absorption optical depth tau_bnd (nbnd, nlay, ncol) as it is
// read -- inc_1scalar_by_1scalar_bybnd (rte/kernels/mo_optical_props_kernels.F90:358-372), tau + tau_bnd(band),
// the same single add -- so clouds%increment(atmos) never makes a pass over the g-point array.
template <bool kFused, bool kInc, int kPF, bool kMulti>
__global__ void LW_BOUNDS lw_noscat_kernel(int ngpt, int nlay, int ncol, int top_at_1, LwAngles ang,
                                           const float *__restrict__ inc_flux, const float *__restrict__ tau,
                                           const float *__restrict__ lay, const float *__restrict__ lev,
                                           const float *__restrict__ emis, const float *__restrict__ sfc,
                                           LwPlanck pl, BandArgs bands, const float *__restrict__ tau_bnd,
                                           float *__restrict__ gdn, float *__restrict__ gup, long long gcs,
                                           float *__restrict__ flux_up, float *__restrict__ flux_dn)
{
  static_assert(kRing % kPF == 0, "prefetch depth must divide the ring");
  // the fused down pass takes lev(l+1)'s Planck fraction from the neighbouring prefetch slot, py[(r+1) % kPF]: with
  // one slot that would be the layer's own pfrac
  static_assert(!kFused || kPF >= 2, "the fused down pass needs at least two prefetch slots");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int icol = blockIdx.x, g = threadIdx.x;
  const bool on = g < ngpt;
  const int gc = on ? g : ngpt - 1;  // clamped g-point for unconditional loads
  const int nlev = nlay + 1;
  const uint32_t vg = 4u * (uint32_t)gc, row = 4u * (uint32_t)ngpt;
  // kMulti (nmus > 1, lw_solver_noscat_GaussQuad :383-412): g-point fluxes are summed over angles first, then
  // reduced with sum_broadband's plain sequential sum; gdn / gup (column stride gcs) hold the per-g accumulators,
  // (nlev, ngpt) per column: the context workspace, or the caller's g-point flux arrays (ty_fluxes_flexible).  With
  // ang.rad (g-point outputs at one angle) they receive the radiances and the fluxes are reduced as lw_solver_noscat
  // reduces them (quirk B-5).  A template parameter, so the nmus = 1 kernel's layer loop holds no global memory
  // access besides its loads and the compiler's vmcnt waits keep the prefetch distance (a runtime branch merged both
  // paths into vmcnt(0)).
  float *wdn = kMulti ? gdn + gcs * icol : nullptr, *wup = kMulti ? gup + gcs * icol : nullptr;
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  float *btab = smem + kExpTabFloats;                        // fused: [nbnd][2*nlay+1] + [nbnd]
  const int brow = 2 * nlay + 1;
  // [kRing][rs]: rows of ngpt floats, padded by 4 when the flush walks one lane per partial (rows in different banks)
  const int rs = lw_ring_stride(ngpt);
  float *ring = btab + (kFused ? lw_btab_floats(bands.nbnd, nlay) : 0);
  float *part = ring + (size_t)kRing * rs;                   // [2][nlev][4]: 0 = dn, 1 = up
  load_exp_table(etab);
  const ColArr Ttau(tau, (size_t)ngpt * nlay * icol, row * nlay);
  const ColArr Tlay(lay, (size_t)ngpt * nlay * icol, row * nlay);  // lay_source, or pfrac when fused
  const ColArr Tlev(lev, (size_t)ngpt * nlev * icol, row * nlev);
  const float *bl = btab;  // this lane's band row
  // kInc: this lane's band-resolved increment, one value per layer at stride nbnd
  const uint32_t irow = 4u * (uint32_t)bands.nbnd, vb = kInc ? 4u * (uint32_t)band_of(bands, gc) : 0u;
  const ColArr Tinc(kInc ? tau_bnd : tau, kInc ? (size_t)bands.nbnd * nlay * icol : 0, irow * nlay);
  auto ld_inc = [&](int l) { return kInc ? Tinc.ld(vb, irow * (uint32_t)l) : 0.0f; };
  auto tau_of = [&](float t, float ti) { return kInc ? t + ti : t; };
  // the value to load for lev index li: lev_source(li), or pfrac(min(li, nlay-1)) when fused
  auto lev_ld = [&](int li) {
    return kFused ? Tlay.ld(vg, row * (uint32_t)min(li, nlay - 1)) : Tlev.ld(vg, row * (uint32_t)li);
  };
  // j-th layer from the top is l = lay_dn(j)
  auto lay_dn = [&](int j) { return top_at_1 ? j : nlay - 1 - j; };
  // The first angle's first kPF layers, the surface Planck fraction, the emissivity and the incident flux are loaded
  // here, ahead of the prologue's barriers (which would hold the loads back until the Planck table is built).  Only in
  // the fused clear-sky instance: in the others the early layers' registers spill (64 VGPRs, the 8-wave bound).
  constexpr bool kEarly = kFused && !kInc;
  float pt0[kPF], py0[kPF], pv0[kPF], pi0[kPF];
#pragma unroll
  for (int p = 0; p < kPF; p++) {
    const int l = lay_dn(min(p, nlay - 1));
    pt0[p] = kEarly ? Ttau.ld(vg, row * l) : 0.0f;
    py0[p] = kEarly ? Tlay.ld(vg, row * l) : 0.0f;
    pi0[p] = 0.0f;
    pv0[p] = (kEarly && !kFused) ? lev_ld(l + 1) : 0.0f;
  }
  const float ysfc = kFused ? Tlay.ld(vg, row * (uint32_t)(pl.sfc_lay - 1)) : 0.0f;
  // emissivity per g-point, or (fused, emis_by_band) the band value rte_lw's expand would copy there
  const float e = !on ? 0.0f
                      : (kFused && pl.emis_by_band ? emis[band_of(bands, g) + (size_t)bands.nbnd * icol]
                                                   : emis[g + (size_t)ngpt * icol]);
  const float inc = (on && inc_flux) ? inc_flux[g + (size_t)ngpt * icol] : 0.0f;
  float ss;
  if constexpr (kFused) {
    // band Planck values for this column: B_b(tlay(l)) at [b][l], B_b(tlev(l)) at [b][nlay+l], B_b(tsfc) at
    // [nbnd*brow + b]; interpolate1D of compute_Planck_source_nn
    const float *tl = pl.tlay + (size_t)nlay * icol, *tv = pl.tlev + (size_t)nlev * icol;
    // kBtabU entries per thread per round, their loads issued together: the temperatures, then the table pairs (a
    // loop of one entry per round waits out two dependent load latencies per entry, ~16 per block at C3)
    constexpr int kBtabU = 8;
    const int ntab = bands.nbnd * (brow + 1), nrow = bands.nbnd * brow;
    for (int i0 = threadIdx.x; i0 < ntab; i0 += kBtabU * (int)blockDim.x) {
      float T[kBtabU];
      int bb[kBtabU];
#pragma unroll
      for (int u = 0; u < kBtabU; u++) {
        const int i = min(i0 + u * (int)blockDim.x, ntab - 1);  // clamped: past-the-end entries are not stored
        const int b = i < nrow ? i / brow : i - nrow;
        const int k = i < nrow ? i - b * brow : -1;
        bb[u] = b;
        const float *p = k < 0 ? pl.tsfc + icol : (k < nlay ? tl + k : tv + (k - nlay));  // one load, no branch
        T[u] = *p;
      }
      float v[kBtabU];
#pragma unroll
      for (int u = 0; u < kBtabU; u++)
        v[u] = interp1d(T[u], pl.tmin, pl.tdelta, pl.ntemp, pl.totplnk + (size_t)pl.ntemp * bb[u]);
#pragma unroll
      for (int u = 0; u < kBtabU; u++) {
        const int i = i0 + u * (int)blockDim.x;
        if (i < ntab) btab[i] = v[u];
      }
    }
    const int b = band_of(bands, gc);
    bl = btab + (size_t)b * brow;
    __syncthreads();
    ss = ysfc * btab[(size_t)bands.nbnd * brow + b];
  } else {
    __syncthreads();
    ss = on ? sfc[g + (size_t)ngpt * icol] : 0.0f;
  }
  const float tau_thresh = sqrtf(FLT_EPSILON);
  const int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0;
  // stage one level's value v = fac * radiance: slot r of the ring, or (kMulti) the per-g accumulator of plane q
  // (the radiance itself with ang.rad)
  auto put = [&](float v, float rad, int r, int q, int level, bool acc) {
    if constexpr (kMulti) {
      if (on) {
        float *w = (q == 0 ? wdn : wup) + (size_t)level * ngpt + g;
        const float x = ang.rad ? rad : v;
        *w = acc ? *w + x : x;
      }
    } else if (on) {
      ring[(size_t)r * rs + g] = v;
    }
  };
  auto flush = [&](float *pq, int n, int lev0, int dl) {
    if constexpr (!kMulti) {
      if (rs != ngpt)
        ring_flush_lanes(ring, rs, pq, n, lev0, dl, ngpt);
      else
        ring_flush<kRing>(ring, pq, 1, n, lev0, dl, ngpt, nlev, false);
    }
  };
  // layer source and the level source on the side given by `li` (lev index, 0..nlay)
  auto lay_src = [&](float y, int l) { return kFused ? y * bl[l] : y; };
  auto lev_src = [&](float v, int li) { return kFused ? v * bl[nlay + li] : v; };
  float *pdn = part, *pup = part + (size_t)nlev * 4;
  const int dl_dn = top_at_1 ? 1 : -1;  // level index step going down

  for (int imu = 0; imu < ang.nmus; imu++) {
    // lw_Ds (rte/mo_rte_lw.F90:329-341): the kernel's D(igpt, icol), one angle
    const float D = ang.Dg ? ang.Dg[gc + (size_t)ngpt * icol] : ang.D[imu];
    // radiance -> flux factor inside the broadband sum; with nmus == 1 and ngpt % 4 != 0 the reference
    // sums plain radiances (quirk B-5, mo_rte_solver_kernels.F90:287-320)
    const float fac = (kMulti || (ngpt & 3) == 0) ? 2.0f * kPi * ang.w[imu] : 1.0f;
    const bool acc = imu > 0;
    float I = inc / (2.0f * kPi * ang.w[imu]);
    put(fac * I, I, 0, 0, top, acc);
    flush(pdn, 1, top, 1);
    // downward: lw_transport_noscat_dn (:982-1009)
    {
      float pt[kPF], py[kPF], pv[kPF], pi[kPF];
      if (kEarly && imu == 0) {  // loaded ahead of the prologue
#pragma unroll
        for (int p = 0; p < kPF; p++) {
          pt[p] = pt0[p]; py[p] = py0[p]; pi[p] = pi0[p]; pv[p] = pv0[p];
        }
      } else {
#pragma unroll
        for (int p = 0; p < kPF; p++) {
          const int l = lay_dn(min(p, nlay - 1));
          pt[p] = Ttau.ld(vg, row * l); py[p] = Tlay.ld(vg, row * l); pi[p] = ld_inc(l);
          if constexpr (!kFused) pv[p] = lev_ld(l + 1);
        }
      }
      // fused: lev(l+1)'s Planck fraction pfrac(min(l+1, nlay-1)) is a neighbour's in walk order, already loaded --
      // the next layer's (top_at_1: in the other prefetch slot) or the previous one's (bottom first) -- and the
      // layer's own at the clamped end; kept here instead of loaded a second time
      float py_prev = 0.0f;
      // Every step issues its prefetch loads unconditionally (clamped to the last layer); only the arithmetic of
      // the last chunk's steps past nlay is skipped, by a uniform branch holding no memory access, so the
      // compiler's vmcnt waits see the same loads on every path and keep the prefetch distance.
      auto step = [&](int j, int r) {
        const int p = r % kPF, l = lay_dn(min(j, nlay - 1));
        const float y_next = py[(r + 1) % kPF], y_own = py[p];
        const float v = kFused ? (top_at_1 ? y_next : (j == 0 ? y_own : py_prev)) : pv[p];
        const float t = tau_of(pt[p], pi[p]) * D, ly = lay_src(y_own, l), lvdn = lev_src(v, l + 1);
        py_prev = y_own;
        {
          const int ln = lay_dn(min(j + kPF, nlay - 1));
          pt[p] = Ttau.ld(vg, row * ln); py[p] = Tlay.ld(vg, row * ln);
          if constexpr (!kFused) pv[p] = lev_ld(ln + 1);
          pi[p] = ld_inc(ln);
        }
        if (j < nlay) {
          const float T = solver_exp_neg(-t, etab);
          const float fact = (t > tau_thresh) ? solver_div(1.0f - T, t) - T : t * (0.5f - 1.0f / 3.0f * t);
          const float S = (1.0f - T) * lvdn + 2.0f * fact * (ly - lvdn);
          I = T * I + S;
          put(fac * I, I, r, 0, top_at_1 ? l + 1 : l, acc);
        }
      };
      for (int j0 = 0; j0 < nlay; j0 += kRing) {
#pragma unroll
        for (int r = 0; r < kRing; r++) step(j0 + r, r);
        flush(pdn, min(kRing, nlay - j0), top + dl_dn * (j0 + 1), dl_dn);
      }
    }
    // upward: lw_transport_noscat_up (:950-980); j-th layer from the surface is l = lay_up(j).  With one angle its first
    // kPF layers are loaded before the surface level's flush, whose barrier would otherwise hold the loads back (with
    // several angles there is no flush, and the registers would spill)
    auto lay_up = [&](int j) { return top_at_1 ? nlay - 1 - j : j; };
    float ptu[kPF], pyu[kPF], pvu[kPF], piu[kPF];
    if constexpr (!kMulti) {
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int l = lay_up(min(p, nlay - 1));
        ptu[p] = Ttau.ld(vg, row * l); pyu[p] = Tlay.ld(vg, row * l); piu[p] = ld_inc(l);
        pvu[p] = kFused ? 0.0f : Tlev.ld(vg, row * l);
      }
    }
    // surface reflection and emission (:269)
    float U = I * (1.0f - e) + e * ss;
    put(fac * U, U, 0, 1, sfcl, acc);
    flush(pup, 1, sfcl, 1);
    {
      float pt[kPF], py[kPF], pv[kPF], pi[kPF];
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        if constexpr (!kMulti) {
          pt[p] = ptu[p]; py[p] = pyu[p]; pi[p] = piu[p]; pv[p] = pvu[p];
        } else {
          const int l = lay_up(min(p, nlay - 1));
          pt[p] = Ttau.ld(vg, row * l); py[p] = Tlay.ld(vg, row * l); pi[p] = ld_inc(l);
          if constexpr (!kFused) pv[p] = Tlev.ld(vg, row * l);
        }
      }
      auto step = [&](int j, int r) {
        const int p = r % kPF, l = lay_up(min(j, nlay - 1));
        // fused: lev(l) = pfrac(l) * B(tlev(l)) (l < nlay), from the layer's own pfrac
        const float t = tau_of(pt[p], pi[p]) * D, ly = lay_src(py[p], l);
        const float lvup = lev_src(kFused ? py[p] : pv[p], l);
        {
          const int ln = lay_up(min(j + kPF, nlay - 1));
          pt[p] = Ttau.ld(vg, row * ln); py[p] = Tlay.ld(vg, row * ln); pi[p] = ld_inc(ln);
          if constexpr (!kFused) pv[p] = Tlev.ld(vg, row * ln);
        }
        if (j < nlay) {
          const float T = solver_exp_neg(-t, etab);
          const float fact = (t > tau_thresh) ? solver_div(1.0f - T, t) - T : t * (0.5f - 1.0f / 3.0f * t);
          const float S = (1.0f - T) * lvup + 2.0f * fact * (ly - lvup);
          U = T * U + S;
          put(fac * U, U, r, 1, top_at_1 ? l : l + 1, acc);
        }
      };
      for (int j0 = 0; j0 < nlay; j0 += kRing) {
#pragma unroll
        for (int r = 0; r < kRing; r++) step(j0 + r, r);
        flush(pup, min(kRing, nlay - j0), sfcl - dl_dn * (j0 + 1), -dl_dn);
      }
    }
  }
  if constexpr (kMulti) {
    __syncthreads();
    for (int t = g; t < 2 * nlev; t += blockDim.x) {
      const int l = t % nlev;
      const float *w = (t < nlev ? wdn : wup) + (size_t)l * ngpt;
      float s = 0.0f;
      if (ang.rad && (ngpt & 3) == 0) {
        // one angle: lw_solver_noscat's inline reduction of fac * radiance in 4 partial sums (:296-318)
        const float fac = 2.0f * kPi * ang.w[0];
        float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int i = 0; i < ngpt; i += 4)
          for (int k = 0; k < 4; k++) s4[k] = s4[k] + fac * w[i + k];
        s = ((s4[0] + s4[1]) + s4[2]) + s4[3];
      } else {
        for (int i = 0; i < ngpt; i++) s = s + w[i];  // sum_broadband (or, one angle, ngpt % 4 != 0: quirk B-5)
      }
      (t < nlev ? flux_dn : flux_up)[l + (size_t)nlev * icol] = s;
    }
    return;
  }
  for (int l = g; l < nlev; l += blockDim.x) {
    flux_dn[l + (size_t)nlev * icol] = combine4(pdn + 4 * l);
    flux_up[l + (size_t)nlev * icol] = combine4(pup + 4 * l);
  }
}

template <bool kFused, bool kInc>
static int launch_lw_impl(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                          const float *Ds, const float *wts, const float *inc_flux, const float *tau,
                          const float *lay_or_pfrac, const float *lev_source, const float *sfc_emis,
                          const float *sfc_source, const LwPlanck &pl, const BandArgs &bands, const float *tau_bnd,
                          float *flux_up, float *flux_dn)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (nmus < 1 || nmus > 4) return fail(RRTMGPNN_ERR_ARGUMENT, "lw solver: nmus must be 1..4");
  if (ngpt > kLwMaxG) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw solver: too many g-points");
  const auto &ex = ctx->extras;
  if (ex.lw_Ds && nmus != 1) return fail(RRTMGPNN_ERR_ARGUMENT, "rte_lw: providing lw_Ds incompatible with specifying n_gauss_angles");
  if ((ex.gpt_up == nullptr) != (ex.gpt_dn == nullptr))
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw solver: g-point outputs need both gpt_flux_up and gpt_flux_dn");
  const bool gpt = ex.gpt_up != nullptr;
  LwAngles a{};
  a.nmus = nmus;
  a.Dg = ex.lw_Ds;
  a.rad = gpt && nmus == 1;
  for (int i = 0; i < nmus; i++) { a.D[i] = Ds[i]; a.w[i] = wts[i]; }
  int threads = (ngpt + 63) / 64 * 64;
  size_t lds = sizeof(float) * (kExpTabFloats + (size_t)kRing * lw_ring_stride(ngpt) + (size_t)2 * (nlay + 1) * 4);
  if (kFused) lds += sizeof(float) * lw_btab_floats(bands.nbnd, nlay);
  if (lds > 64 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw solver: too many layers for LDS partials");
  // per-g accumulators: the caller's g-point arrays, or (several angles) the context workspace
  float *gdn = ex.gpt_dn, *gup = ex.gpt_up;
  const long long nv = (long long)ngpt * (nlay + 1);
  long long gcs = nv;
  if (!gpt && nmus > 1) {
    void *ws = nullptr;
    int rc = ctx->workspace(sizeof(float) * 2 * (size_t)nv * ncol, &ws);
    if (rc) return rc;
    gdn = (float *)ws;
    gup = gdn + nv;
    gcs = 2 * nv;
  }
  constexpr int PF = kFused ? kLwfPf : kLwPf;
  if (nmus > 1 || gpt)
    hipLaunchKernelGGL((lw_noscat_kernel<kFused, kInc, PF, true>), dim3(ncol), dim3(threads), lds, ctx->stream, ngpt,
                       nlay, ncol, top_at_1, a, inc_flux, tau, lay_or_pfrac, kFused ? lay_or_pfrac : lev_source,
                       sfc_emis, sfc_source, pl, bands, tau_bnd, gdn, gup, gcs, flux_up, flux_dn);
  else
    hipLaunchKernelGGL((lw_noscat_kernel<kFused, kInc, PF, false>), dim3(ncol), dim3(threads), lds, ctx->stream, ngpt,
                       nlay, ncol, top_at_1, a, inc_flux, tau, lay_or_pfrac, kFused ? lay_or_pfrac : lev_source,
                       sfc_emis, sfc_source, pl, bands, tau_bnd, gdn, gup, gcs, flux_up, flux_dn);
  RRTMGPNN_LAUNCH_CHECK("lw_noscat_kernel");
  return RRTMGPNN_OK;
}

int launch_lw_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus, const float *Ds,
                     const float *wts, const float *inc_flux, const float *tau, const float *lay_source,
                     const float *lev_source, const float *sfc_emis, const float *sfc_source, float *flux_up,
                     float *flux_dn)
{
  LwPlanck pl{};
  BandArgs b{};
  return launch_lw_impl<false, false>(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, wts, inc_flux, tau, lay_source,
                                      lev_source, sfc_emis, sfc_source, pl, b, nullptr, flux_up, flux_dn);
}

int launch_lw_noscat_planck(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                            const float *Ds, const float *wts, const float *inc_flux, const float *tau,
                            const float *pfrac, int ntemp, const float *tlay, const float *tlev, const float *tsfc,
                            int sfc_lay, const BandArgs &bands, float temp_ref_min, float totplnk_delta,
                            const float *totplnk, bool emis_by_band, const float *sfc_emis, const float *tau_bnd,
                            float *flux_up, float *flux_dn)
{
  LwPlanck pl{tlay, tlev, tsfc, totplnk, ntemp, sfc_lay, emis_by_band ? 1 : 0, temp_ref_min, totplnk_delta};
  if (tau_bnd)
    return launch_lw_impl<true, true>(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, wts, inc_flux, tau, pfrac, nullptr,
                                      sfc_emis, nullptr, pl, bands, tau_bnd, flux_up, flux_dn);
  return launch_lw_impl<true, false>(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, wts, inc_flux, tau, pfrac, nullptr,
                                     sfc_emis, nullptr, pl, bands, nullptr, flux_up, flux_dn);
}

// ------------------------------------------------------------------------------------------
// SW two-stream solver.  block = one column, lane = g-point.
//   pass 1 (top->bottom): direct beam F_dir per level -> WA
//   pass 2 (bottom->top): sw_two_stream_source coefficients (Tnoscat recomputed bit-identically
//          from tau and mu0) and adding's albedo/src (Shonk & Hogan Eqs 9-11) -> WB, WS per level;
//          the layer's direct-beam source S_dn -> WD
//   pass 3 (top->bottom): Eqs 12-13 with the reference's exact expression order.  Only R_dif and
//          T_dif are recomputed (same expressions, same bits as pass 2); S_dn, albedo, src and the
//          direct beam are read back.  Ordered broadband sums of up, dif+dir, dir, staged per chunk
//          of kRingSw levels as in the LW solver.
// The split between recomputing and storing balances the kernel's two bounds: recomputing all of
// sw_two_stream in pass 3 made it VALU-bound (~400 VALU ops per layer and g-point), storing every
// coefficient would make it HBM-bound; this form is ~250 ops and 4 workspace planes.
// Workspace ws: 4 arrays (ngpt, nlay+1, ncol): WA = F_dir, WB = albedo, WS = src, WD = S_dn.
// kHasG = false: g == NULL means g == 0 everywhere (the NN path zero-fills g, quirk B-6); the
// coefficient expressions then evaluate with a literal 0 -- identical bits, one array less to read.
// ------------------------------------------------------------------------------------------
struct SwDif {
  float gamma1, gamma2, k, emk, em2k, RT, Rdif, Tdif;
};

// diffuse reflectance/transmittance of sw_two_stream (mo_rte_solver_kernels.F90:1366-1480)
__device__ __forceinline__ SwDif sw_dif(float tau, float w0, float g, const uint64_t *etab)
{
  const float k_min = 1.e-4f;
  SwDif d;
  d.gamma1 = (8.0f - w0 * (5.0f + 3.0f * g)) * .25f;
  d.gamma2 = 3.0f * (w0 * (1.0f - g)) * .25f;
  d.k = sqrt_rn_normal(fmaxf((d.gamma1 - d.gamma2) * (d.gamma1 + d.gamma2), k_min));
  d.emk = solver_exp_neg(-tau * d.k, etab);
  d.em2k = d.emk * d.emk;
  d.RT = rcp_rn_normal(d.k * (1.0f + d.em2k) + d.gamma1 * (1.0f - d.em2k));
  d.Rdif = d.RT * d.gamma2 * (1.0f - d.em2k);
  d.Tdif = d.RT * 2.0f * d.k * d.emk;
  return d;
}

struct SwCoef {
  float Rdif, Tdif, Sup, Sdn, Tnoscat;
};

// kG0: g is the literal 0 (the NN path), so gamma3 = (2 - 3 mu0 0)/4 = 0.5 and gamma4 = 0.5 exactly (mu0 finite).
template <bool kG0 = false>
__device__ __forceinline__ SwCoef sw_two_stream(float tau, float w0, float g, float mu0, float mu0_inv, float dir_inc,
                                               const uint64_t *etab)
{
  const float eps = FLT_EPSILON;
  SwCoef c;
  const SwDif d = sw_dif(tau, w0, g, etab);
  const float gamma1 = d.gamma1, gamma2 = d.gamma2, k = d.k, emk = d.emk, em2k = d.em2k;
  float Tnoscat = solver_exp_beam(-tau * mu0_inv, etab);
  float gamma3 = kG0 ? 0.5f : (2.0f - 3.0f * mu0 * g) * .25f;
  float gamma4 = 1.0f - gamma3;
  float alpha1 = gamma1 * gamma4 + gamma2 * gamma3;
  float alpha2 = gamma1 * gamma3 + gamma2 * gamma4;
  float k2e = 2.0f * k * emk;
  c.Rdif = d.Rdif;
  c.Tdif = d.Tdif;
  float k_mu = k * mu0, k_mu2 = k_mu * k_mu, k_g3 = k * gamma3, k_g4 = k * gamma4;
  float dd = (fabsf(1.0f - k_mu2) >= eps) ? (1.0f - k_mu2) : eps;
  float RT = solver_div(w0 * d.RT, dd);
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

// inc_2stream_by_2stream_bybnd (rte/kernels/mo_optical_props_kernels.F90:430-463) for one g-point: the
// same expressions as increment_bybnd_kernel, so the incremented properties are bit-identical.
__device__ __forceinline__ void inc_2str(float &t1, float &w1, float &g1, float t2, float w2, float g2)
{
  const float eps = 3.0f * FLT_MIN;
  const float tau12 = t1 + t2;
  const float tauscat12 = t1 * w1 + t2 * w2;
  g1 = (t1 * w1 * g1 + t2 * w2 * g2) / fmaxf(eps, tauscat12);
  w1 = tauscat12 / fmaxf(eps, tau12);
  t1 = tau12;
}

// kInc: the atmosphere is incremented by band-resolved two-stream properties (tau, ssa, g)_bnd as it is read
// (clouds%increment(atmos) fused).  Pass 1 needs only tau + tau_bnd; pass 2 forms the full increment and
// parks (tau, ssa, g) in three workspace planes that pass 3 reads in place of the inputs.
//
// One column per block: packing two 224-g-point columns into 7 full waves (as the two-per-lane kernel does) was
// measured slower here (C3 0.312 vs 0.288 ms): its 72 VGPRs allow 7 waves per SIMD, and this kernel wants 8.
//
// kGpt: also store the g-point fluxes (ty_fluxes_flexible; (ngpt, nlay+1, ncol) each): up, the total down flux
// (diffuse + direct, rounded once: "adding computes only diffuse flux; flux_dn is total", :665-666, and for ngpt not
// a multiple of 4 radn_dn = radn_dn + radn_dir, :682) and direct, with the broadband down flux summed from the
// total as sw_solver_2stream does when it saves them (:660-684).  This is the g-point kernel for odd ngpt; even ngpt
// takes the checkpointed kernel's g-point instance.
template <bool kHasG, bool kInc, int kPF, bool kGpt = false>
__global__ void SW_BOUNDS sw_2stream_kernel(int ngpt, int nlay, int ncol, int top_at_1,
                                            const float *__restrict__ inc_flux, const float *__restrict__ inc_dif,
                                            const float *__restrict__ tau, const float *__restrict__ ssa,
                                            const float *__restrict__ gg, const float *__restrict__ mu0p,
                                            const float *__restrict__ alb_dir, const float *__restrict__ alb_dif,
                                            BandArgs bands, const float *__restrict__ tau_bnd,
                                            const float *__restrict__ ssa_bnd, const float *__restrict__ g_bnd,
                                            float *__restrict__ ws, float *__restrict__ flux_up,
                                            float *__restrict__ flux_dn, float *__restrict__ flux_dir,
                                            float *__restrict__ gpt_up, float *__restrict__ gpt_dn,
                                            float *__restrict__ gpt_dir)
{
  static_assert(kRingSw % kPF == 0, "prefetch depth must divide the ring");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nlev = nlay + 1;
  const int icol = blockIdx.x, g = threadIdx.x;
  const bool on = g < ngpt;
  const int gc = on ? g : ngpt - 1;  // clamped g-point for unconditional loads
  float *ring = smem + kExpTabFloats;                // [3][kRingSw][ngpt]: up, dif, dir
  float *part = ring + (size_t)3 * kRingSw * ngpt;   // [3][nlev][4]: up, dn, dir
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  load_exp_table(etab);
  __syncthreads();
  const uint32_t row = 4u * (uint32_t)ngpt;
  const uint32_t vL = 4u * (uint32_t)gc, vV = vL;  // g-point in the VGPR offset (layer and level arrays alike)
  const size_t cl = (size_t)ngpt * nlay * icol, cv = (size_t)ngpt * nlev * icol, plane = (size_t)ngpt * nlev * ncol;
  const uint32_t bL = row * nlay, bV = row * nlev;
  const ColArr Ttau(tau, cl, bL), Tssa(ssa, cl, bL), Tg(kHasG ? gg : tau, cl, bL);
  const ColArr WA(ws, cv, bV), WB(ws + plane, cv, bV), WS(ws + 2 * plane, cv, bV), WD(ws + 3 * plane, cv, bV);
  // kInc: incremented (tau, ssa, g) planes (ngpt, nlay, ncol) after the four level planes
  const size_t lplane = (size_t)ngpt * nlay * ncol;
  float *wi = ws + 4 * plane;
  const ColArr WT(wi, cl, bL), WW(wi + lplane, cl, bL), WG(wi + 2 * lplane, cl, bL);
  // band-resolved increments: this lane's band in the VGPR offset, the layer in the SGPR offset
  const size_t cb = (size_t)bands.nbnd * nlay * icol;
  const uint32_t brow = 4u * (uint32_t)bands.nbnd;
  const uint32_t vb = kInc ? 4u * (uint32_t)band_of(bands, gc) : 0u;
  const uint32_t bB = kInc ? brow * nlay : 0u;
  const ColArr Bt(kInc ? tau_bnd : tau, kInc ? cb : 0, bB), Bw(kInc ? ssa_bnd : tau, kInc ? cb : 0, bB),
      Bg(kInc ? g_bnd : tau, kInc ? cb : 0, bB);
  auto ld_bnd = [&](const ColArr &a, int l) { return kInc ? a.ld(vb, brow * (uint32_t)l) : 0.0f; };
  const float mu0 = mu0p[icol], mu0_inv = 1.0f / mu0;
  // "layer l spans levels l (top side) and l+1" when top_at_1, else l+1 (top) and l
  auto lev_above = [&](int l) { return top_at_1 ? l : l + 1; };
  auto lev_below = [&](int l) { return top_at_1 ? l + 1 : l; };
  auto lay_of_down = [&](int j) { return top_at_1 ? j : nlay - 1 - j; };  // j-th layer from the top
  auto lay_of_up = [&](int j) { return top_at_1 ? nlay - 1 - j : j; };    // j-th layer from the surface
  auto ld_g = [&](uint32_t soff) { return kHasG ? Tg.ld(vL, soff) : 0.0f; };
  const size_t gcol = (size_t)gc + (size_t)ngpt * icol;  // this lane's (g, col) in (ngpt, ncol) arrays
  const int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0;
  const float Ftop = on ? inc_flux[gcol] * mu0 : 0.0f;

  // ---- pass 1: direct beam (only tau is read) ----
  // Straight-line layer steps: the prefetch loads and the stores are issued on every step, the stores of idle
  // lanes (g >= ngpt) and of the steps past nlay at an out-of-range buffer offset (dropped by the hardware), and
  // only arithmetic sits under the uniform `j < nlay` branch.  So every path issues the same memory operations and
  // the compiler's vmcnt waits (loads and stores share the counter) keep the prefetch distance instead of
  // draining to vmcnt(0) at each merge.
  const uint32_t vVs = on ? vV : kBufOOB, vLs = on ? vL : kBufOOB;
  float Fd = Ftop;
  WA.st(Fd, vVs, row * top);
  {
    float pt[kPF], pi[kPF];
#pragma unroll
    for (int p = 0; p < kPF; p++) {
      const int l = lay_of_down(min(p, nlay - 1));
      pt[p] = Ttau.ld(vL, row * l);
      pi[p] = ld_bnd(Bt, l);
    }
    for (int j0 = 0; j0 < nlay; j0 += kPF) {
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int j = j0 + p;
        const int l = lay_of_down(min(j, nlay - 1));
        const float t = kInc ? pt[p] + pi[p] : pt[p];  // tau12 of the increment
        {
          const int ln = lay_of_down(min(j + kPF, nlay - 1));
          pt[p] = Ttau.ld(vL, row * ln);
          pi[p] = ld_bnd(Bt, ln);
        }
        if (j < nlay) Fd = solver_exp_beam(-t * mu0_inv, etab) * Fd;
        WA.st(Fd, j < nlay ? vVs : kBufOOB, row * lev_below(l));
      }
    }
  }
  // ---- pass 2: bottom -> top adding (albedo, src) ----
  float alb_b = on ? alb_dif[gcol] : 0.0f;  // albedo at the level below
  float src_b = on ? Fd * alb_dir[gcol] : 0.0f;
  WB.st(alb_b, vVs, row * sfcl);
  WS.st(src_b, vVs, row * sfcl);
  {
    float pt[kPF], pw[kPF], pg[kPF], pf[kPF], qt[kPF], qw[kPF], qg[kPF];
    auto load2 = [&](int p, int l) {
      const uint32_t s = row * l;
      pt[p] = Ttau.ld(vL, s); pw[p] = Tssa.ld(vL, s); pg[p] = ld_g(s); pf[p] = WA.ld(vV, row * lev_above(l));
      if constexpr (kInc) {
        qt[p] = ld_bnd(Bt, l); qw[p] = ld_bnd(Bw, l); qg[p] = ld_bnd(Bg, l);
      }
    };
#pragma unroll
    for (int p = 0; p < kPF; p++) load2(p, lay_of_up(min(p, nlay - 1)));
    for (int j0 = 0; j0 < nlay; j0 += kPF) {
#pragma unroll
      for (int p = 0; p < kPF; p++) {
        const int j = j0 + p;
        const int l = lay_of_up(min(j, nlay - 1));
        const uint32_t vs = j < nlay ? vVs : kBufOOB, vls = j < nlay ? vLs : kBufOOB;
        float t = pt[p], w0 = pw[p], g0 = kHasG ? pg[p] : 0.0f;
        const float Fin = pf[p];
        if constexpr (kInc) {
          inc_2str(t, w0, g0, qt[p], qw[p], qg[p]);
          WT.st(t, vls, row * l);
          WW.st(w0, vls, row * l);
          WG.st(g0, vls, row * l);
        }
        load2(p, lay_of_up(min(j + kPF, nlay - 1)));
        float alb = alb_b, src = src_b, Sdn = 0.0f;
        if (j < nlay) {
          SwCoef cf = sw_two_stream<!kHasG && !kInc>(t, w0, g0, mu0, mu0_inv, Fin, etab);
          const float denom = rcp_rn_normal(1.0f - cf.Rdif * alb_b);
          alb = cf.Rdif + cf.Tdif * cf.Tdif * alb_b * denom;
          src = cf.Sup + cf.Tdif * denom * (src_b + alb_b * cf.Sdn);
          Sdn = cf.Sdn;
        }
        const uint32_t sa = row * lev_above(l);
        WB.st(alb, vs, sa);
        WS.st(src, vs, sa);
        WD.st(Sdn, vs, row * l);
        alb_b = alb;
        src_b = src;
      }
    }
  }
  // ---- pass 3: top -> bottom fluxes + ordered broadband sums ----
  // lev: the level's array index (the g-point outputs)
  auto put = [&](float up, float dif, float dir, int r, int lev) {
    if (on) {
      const float dn = kGpt ? dif + dir : dif;  // kGpt: the total, summed as such (dn_mode off below)
      ring[(size_t)r * ngpt + g] = up;
      ring[((size_t)kRingSw + r) * ngpt + g] = dn;
      ring[((size_t)2 * kRingSw + r) * ngpt + g] = dir;
      if constexpr (kGpt) {
        const size_t o = (size_t)g + (size_t)ngpt * ((size_t)lev + (size_t)nlev * icol);
        gpt_up[o] = up;
        gpt_dn[o] = dn;
        gpt_dir[o] = dir;
      }
    }
  };
  auto flush = [&](int n, int lev0, int dl) { ring_flush<kRingSw>(ring, part, 3, n, lev0, dl, ngpt, nlev, !kGpt); };
  const int dl_dn = top_at_1 ? 1 : -1;
  float Fdn = (on && inc_dif) ? inc_dif[gcol] : 0.0f;
  put(Fdn * alb_b + src_b, Fdn, Ftop, 0, top);  // Eq 12 at the top; alb_b/src_b hold the top level's values
  flush(1, top, 1);
  {
    float pt[kPF], pw[kPF], pg[kPF], pd[kPF], pa[kPF], ps[kPF], pf[kPF];
    auto load = [&](int p, int l) {
      const uint32_t s = row * l, sb = row * lev_below(l);
      if constexpr (kInc) {
        pt[p] = WT.ld(vL, s); pw[p] = WW.ld(vL, s); pg[p] = WG.ld(vL, s);
      } else {
        pt[p] = Ttau.ld(vL, s); pw[p] = Tssa.ld(vL, s); pg[p] = ld_g(s);
      }
      pd[p] = WD.ld(vV, s);
      pa[p] = WB.ld(vV, sb); ps[p] = WS.ld(vV, sb); pf[p] = WA.ld(vV, sb);
    };
#pragma unroll
    for (int p = 0; p < kPF; p++) load(p, lay_of_down(min(p, nlay - 1)));
    for (int j0 = 0; j0 < nlay; j0 += kRingSw) {
#pragma unroll
      for (int r = 0; r < kRingSw; r++) {
        const int j = j0 + r, p = r % kPF;
        const float t = pt[p], w0 = pw[p], g0 = kHasG || kInc ? pg[p] : 0.0f;
        const float Sdn = pd[p], alb = pa[p], src = ps[p], Fdir = pf[p];
        load(p, lay_of_down(min(j + kPF, nlay - 1)));
        if (j < nlay) {
          // R_dif, T_dif exactly as pass 2 computed them (same inputs, same expressions -> same bits)
          const SwDif d = sw_dif(t, w0, (kHasG || kInc) ? g0 : 0.0f, etab);
          const float denom = rcp_rn_normal(1.0f - d.Rdif * alb);
          Fdn = (d.Tdif * Fdn + d.Rdif * src + Sdn) * denom;  // Eq 13 (adding :1583-1591)
          const float up = Fdn * alb + src;                    // Eq 12
          put(up, Fdn, Fdir, r, top + dl_dn * (j + 1));
        }
      }
      flush(min(kRingSw, nlay - j0), top + dl_dn * (j0 + 1), dl_dn);
    }
  }
  for (int l = g; l < nlev; l += blockDim.x) {
    flux_up[l + (size_t)nlev * icol] = combine4(part + 4 * l);
    flux_dn[l + (size_t)nlev * icol] = combine4(part + (size_t)nlev * 4 + 4 * l);
    flux_dir[l + (size_t)nlev * icol] = combine4(part + (size_t)2 * nlev * 4 + 4 * l);
  }
}

template <bool kHasG, bool kInc, bool kGpt = false>
static void sw_launch(rrtmgpnn_context *ctx, size_t lds, int threads, int ngpt, int nlay, int ncol,
                      int top_at_1, const float *inc_flux, const float *inc_flux_dif, const float *tau,
                      const float *ssa, const float *g, const float *mu0, const float *alb_dir, const float *alb_dif,
                      const BandArgs &bands, const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, void *ws,
                      float *flux_up, float *flux_dn, float *flux_dir)
{
  const auto &ex = ctx->extras;
  hipLaunchKernelGGL((sw_2stream_kernel<kHasG, kInc, kSwPf, kGpt>), dim3(ncol), dim3(threads), lds,
                     ctx->stream, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g, mu0, alb_dir,
                     alb_dif, bands, tau_bnd, ssa_bnd, g_bnd, (float *)ws, flux_up, flux_dn, flux_dir, ex.gpt_up,
                     ex.gpt_dn, ex.gpt_dir);
}

int launch_sw_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                      const float *inc_flux_dif, const float *tau, const float *ssa, const float *g, const float *mu0,
                      const float *alb_dir, const float *alb_dif, const BandArgs *bands, const float *tau_bnd,
                      const float *ssa_bnd, const float *g_bnd, float *flux_up, float *flux_dn, float *flux_dir,
                      const SwBc *bc)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (ngpt > kSwMaxG) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: too many g-points");
  const bool inc = bands != nullptr;
  // Even ngpt: two g-points per lane.  By default the checkpointed kernel (kernels_sw_ck.hip: 0.67 instead of 1.07 GB
  // per launch at C3, whole step C3 -3 %, C4 -1 % against kernels_sw_x2.hip, tools/gpu_ab.sh); mode 2 forces the
  // workspace-plane kernel, mode 1 one g-point per lane (also the odd-ngpt kernel).
  const int mode = ctx->sw_kernel >= 0 ? ctx->sw_kernel : g_sw_kernel_default;
  // g-point outputs (the *_gpt entries) are written by the checkpointed kernel for even ngpt, whatever the mode, and
  // by the one-per-lane kernel for odd ngpt
  const bool gpt = ctx->extras.gpt_up || ctx->extras.gpt_dn || ctx->extras.gpt_dir;
  if (gpt && (!ctx->extras.gpt_up || !ctx->extras.gpt_dn || !ctx->extras.gpt_dir))
    return fail(RRTMGPNN_ERR_ARGUMENT, "sw solver: g-point outputs need gpt_flux_up, gpt_flux_dn and gpt_flux_dn_dir");
  if (gpt && inc) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: g-point outputs with a fused increment");
  const bool ck = (ngpt % 2) == 0 && (mode == 3 || mode == 0 || gpt);
  const bool x2 = !ck && (ngpt % 2) == 0 && mode != 1;
  // the RFMIP boundary conditions (rrtmgpnn_sw_solver_2stream_rfmip): formed in the checkpointed kernel's prologue;
  // the other kernels read them from memory, formed there first by sw_boundary_kernel
  SwBcDev bcd{};
  if (bc && ck) {
    bcd = sw_boundary_device(bc);
  } else if (bc) {
    if (int rc = launch_sw_boundary(ctx, ngpt, ncol, bc->solar_source, bc->tsi, bc->sfc_alb, bc->sza, bc->toa, bc->alb,
                                    bc->mu0))
      return rc;
    inc_flux = bc->toa;
    alb_dir = alb_dif = bc->alb;
    mu0 = bc->mu0;
  }
  void *ws = nullptr;
  const size_t nlp = x2 ? sw_2stream_x2_layer_planes(inc) : (inc ? 3 : 0);
  const bool small = ck && sw_ck_small(ctx, ngpt, ncol, g != nullptr, inc, gpt), nn = !g && !inc && !gpt;
  const size_t nws = ck ? sw_2stream_ck_ws_floats(ngpt, nlay, ncol, small, inc, nn)
                        : 4 * (size_t)ngpt * (nlay + 1) * ncol + nlp * (size_t)ngpt * nlay * ncol;
  // RRTMGPNN_SW_NO_PLANES=1 (read once per process): take the fallback below from the start (tests/test_gpu_sw_planes.py)
  static const bool no_planes = [] {
    const char *e = std::getenv("RRTMGPNN_SW_NO_PLANES");
    return e && e[0] == '1';
  }();
  const size_t nws0 = ck && !small ? sw_2stream_ck_ws_floats(ngpt, nlay, ncol, false, inc, nn, false) : nws;
  int rc = no_planes && nws0 < nws ? RRTMGPNN_ERR_DEVICE : ctx->workspace(sizeof(float) * nws, &ws);
  bool planes = true;
  if (rc == RRTMGPNN_ERR_DEVICE && nws0 < nws && !ctx->ws_pinned) {
    // the large-grid instances' workspace planes (up to 3x the checkpoints) did not fit: the instances without them
    // give the same bits in the workspace a call needed before round 5
    (void)hipGetLastError();
    planes = false;
    rc = ctx->workspace(sizeof(float) * nws0, &ws);
  }
  if (rc) return rc;
  if (ck)
    return launch_sw_2stream_ck(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g, mu0, alb_dir,
                                alb_dif, bands, tau_bnd, ssa_bnd, g_bnd, ws, flux_up, flux_dn, flux_dir, planes,
                                bc ? &bcd : nullptr);
  if (x2)
    return launch_sw_2stream_x2(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g, mu0, alb_dir,
                                alb_dif, bands, tau_bnd, ssa_bnd, g_bnd, ws, flux_up, flux_dn, flux_dir);
  const int threads = (ngpt + 63) / 64 * 64;
  const size_t lds = sizeof(float) * (kExpTabFloats + (size_t)3 * kRingSw * ngpt + (size_t)3 * (nlay + 1) * 4);
  if (lds > 64 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: too many layers for LDS partials");
  const BandArgs nob{};
  const BandArgs &b = inc ? *bands : nob;
  if (gpt && g)
    sw_launch<true, false, true>(ctx, lds, threads, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g,
                                 mu0, alb_dir, alb_dif, b, nullptr, nullptr, nullptr, ws, flux_up, flux_dn, flux_dir);
  else if (gpt)
    sw_launch<false, false, true>(ctx, lds, threads, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g,
                                  mu0, alb_dir, alb_dif, b, nullptr, nullptr, nullptr, ws, flux_up, flux_dn, flux_dir);
  else if (inc && g)
    sw_launch<true, true>(ctx, lds, threads, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g,
                          mu0, alb_dir, alb_dif, b, tau_bnd, ssa_bnd, g_bnd, ws, flux_up, flux_dn, flux_dir);
  else if (inc)
    sw_launch<false, true>(ctx, lds, threads, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g,
                           mu0, alb_dir, alb_dif, b, tau_bnd, ssa_bnd, g_bnd, ws, flux_up, flux_dn, flux_dir);
  else if (g)
    sw_launch<true, false>(ctx, lds, threads, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g,
                           mu0, alb_dir, alb_dif, b, nullptr, nullptr, nullptr, ws, flux_up, flux_dn, flux_dir);
  else
    sw_launch<false, false>(ctx, lds, threads, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g,
                            mu0, alb_dir, alb_dif, b, nullptr, nullptr, nullptr, ws, flux_up, flux_dn, flux_dir);
  RRTMGPNN_LAUNCH_CHECK("sw_2stream_kernel");
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// rte_sw on 1scl (absorption-only) properties, rte/mo_rte_sw.F90:213-222: apply_BC_factor
// (flux_dir(:, top) = inc_flux * mu0, mo_rte_solver_kernels.F90:1685-1704) and sw_solver_noscat (:496-532): the
// direct beam walked down, flux_dir(l+1) = flux_dir(l) * exp(-tau(l) / mu0), and its broadband sum per level
// (sum_broadband_nocol: one sequential sum over g).  One block per column, lane = g-point; levels are staged in an
// LDS ring and each flush sums one level per thread in g order.  The broadband sum is each column's own (the
// reference sums column 1's spectral fluxes for every column, quirk B-11).
// ------------------------------------------------------------------------------------------
constexpr int kNsRing = 8;

__global__ void __launch_bounds__(1024) sw_noscat_kernel(int ngpt, int nlay, int top_at_1,
                                                         const float *__restrict__ inc_flux,
                                                         const float *__restrict__ tau, const float *__restrict__ mu0p,
                                                         float *__restrict__ flux_dir, float *__restrict__ gpt_dir)
{
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  float *ring = smem + kExpTabFloats;  // [kNsRing][ngpt]
  load_exp_table(etab);
  __syncthreads();
  const int icol = blockIdx.x, g = threadIdx.x, nlev = nlay + 1;
  const bool on = g < ngpt;
  const int gc = on ? g : ngpt - 1;
  const float mu0 = mu0p[icol], mu0_inv = 1.0f / mu0;
  const float *t = tau + (size_t)ngpt * nlay * icol;
  float *out = flux_dir + (size_t)nlev * icol;
  const int top = top_at_1 ? 0 : nlay, dl = top_at_1 ? 1 : -1;
  auto flush = [&](int n, int lev0) {
    __syncthreads();
    if ((int)threadIdx.x < n) {
      const float *r = ring + (size_t)threadIdx.x * ngpt;
      float s = 0.0f;
      for (int i = 0; i < ngpt; i++) s = s + r[i];
      out[lev0 + (int)threadIdx.x * dl] = s;
    }
    __syncthreads();
  };
  // g-point direct flux (ty_fluxes_flexible gpt_flux_dn_dir, (ngpt, nlev, ncol)) when asked for
  float *gcol = gpt_dir ? gpt_dir + (size_t)ngpt * nlev * icol : nullptr;
  float F = inc_flux[gc + (size_t)ngpt * icol] * mu0;
  if (on) ring[g] = F;
  if (on && gcol) gcol[(size_t)ngpt * top + g] = F;
  flush(1, top);
  for (int j0 = 0; j0 < nlay; j0 += kNsRing) {
    const int n = min(kNsRing, nlay - j0);
    float tv[kNsRing];
#pragma unroll
    for (int r = 0; r < kNsRing; r++) {
      const int j = min(j0 + r, nlay - 1);
      tv[r] = t[gc + (size_t)ngpt * (top_at_1 ? j : nlay - 1 - j)];
    }
#pragma unroll
    for (int r = 0; r < kNsRing; r++) {
      if (r < n) {
        F = F * solver_exp_beam(-tv[r] * mu0_inv, etab);
        if (on) ring[(size_t)r * ngpt + g] = F;
        if (on && gcol) gcol[(size_t)ngpt * (top + dl * (j0 + r + 1)) + g] = F;
      }
    }
    flush(n, top + dl * (j0 + 1));
  }
}

int launch_sw_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                     const float *tau, const float *mu0, float *flux_dir)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (ngpt > 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw_solver_noscat: more than 1024 g-points");
  const int threads = (ngpt + 63) / 64 * 64;
  const size_t lds = sizeof(float) * (kExpTabFloats + (size_t)kNsRing * ngpt);
  hipLaunchKernelGGL(sw_noscat_kernel, dim3(ncol), dim3(threads), lds, ctx->stream, ngpt, nlay, top_at_1, inc_flux,
                     tau, mu0, flux_dir, ctx->extras.gpt_dir);
  RRTMGPNN_LAUNCH_CHECK("sw_noscat_kernel");
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
