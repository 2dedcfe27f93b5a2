// kernels_lw_scat.hip -- longwave solvers with scattering for gfx950.
//
//  * lw_rescl_kernel   : lw_solver_noscat[_GaussQuad] with do_rescaling -- what rte_lw runs for two-stream
//                        optical properties unless use_2stream is set (rte/mo_rte_lw.F90:372-387): scattering
//                        folded into a scaled optical depth (rte/kernels/mo_rte_solver_kernels.F90:209-233),
//                        a no-scattering pass down, then lw_transport_1rescl (:1729-1795): up and down again
//                        with the adjustment terms
//  * lw_2stream_kernel : lw_solver_2stream (:426-486) with lw_two_stream (:1018-1069, Fu et al. coefficients),
//                        lw_source_2str (:1112-1162) and adding (:1526-1637); sum_broadband_nocol sums
//
// Same layout and launch shape as the no-scattering solver: one block per column, one lane per g-point,
// the vertical recurrences in registers, level values that a later pass needs parked in a per-column
// workspace, broadband sums in the reference's order (rte_device.hpp).  Every layer quantity is recomputed
// from the inputs in each pass with the same expressions, so it has the same bits each time.
#include "rte_device.hpp"

namespace rrtmgpnn {

constexpr int kScatRing = 8;  // levels staged per ordered flush

// rescaled layer optics (:209-233) and lw_source_noscat (:742-776; lev_source(l) / lev_source(l+1) in array
// order for every orientation, quirk B-1)
struct RsLayer {
  float trans, An, Cn, sdn, sup;
};

__device__ __forceinline__ RsLayer rs_layer(float tau, float ssal, float g, float D, float lay, float lev_l,
                                            float lev_lp1, const uint64_t *etab)
{
  const float tau_thresh = sqrtf(FLT_EPSILON);
  RsLayer r;
  const float wb = ssal * (1.0f - g) * 0.5f;
  const float scaleTau = (1.0f - ssal + wb);
  r.Cn = 0.4f * wb / scaleTau;
  const float t = tau * D * scaleTau;
  r.trans = solver_exp_neg(-t, etab);
  r.An = (1.0f - r.trans * r.trans);
  const float T = r.trans;
  const float fact = (t > tau_thresh) ? (1.0f - T) / t - T : t * (0.5f - 1.0f / 3.0f * t);
  r.sdn = (1.0f - T) * lev_lp1 + 2.0f * fact * (lay - lev_lp1);
  r.sup = (1.0f - T) * lev_l + 2.0f * fact * (lay - lev_l);
  return r;
}

__global__ void __launch_bounds__(256) lw_rescl_kernel(int ngpt, int nlay, int ncol, int top_at_1, LwAngles ang,
                                                       const float *__restrict__ inc_flux,
                                                       const float *__restrict__ tau, const float *__restrict__ ssa,
                                                       const float *__restrict__ gg, const float *__restrict__ lay,
                                                       const float *__restrict__ lev, const float *__restrict__ emis,
                                                       const float *__restrict__ sfc, float *__restrict__ ws,
                                                       float *__restrict__ flux_up, float *__restrict__ flux_dn,
                                                       float *__restrict__ gpt_up, float *__restrict__ gpt_dn)
{
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int icol = blockIdx.x, g = threadIdx.x;
  const bool on = g < ngpt;
  const int gc = on ? g : ngpt - 1;
  const int nlev = nlay + 1;
  // ty_fluxes_flexible g-point outputs (ngpt, nlev, ncol): with one angle the radiances (quirk B-5), with several they
  // are the angle accumulators
  const bool gpt = gpt_up != nullptr;
  float *gdn = gpt ? gpt_dn + (size_t)ngpt * nlev * icol : nullptr, *gup = gpt ? gpt_up + (size_t)ngpt * nlev * icol : nullptr;
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  float *ring = smem + kExpTabFloats;                 // [kScatRing][ngpt]
  float *part = ring + (size_t)kScatRing * ngpt;      // [2][nlev][4]: 0 = dn, 1 = up
  load_exp_table(etab);
  __syncthreads();
  const bool multi = ang.nmus > 1;
  // workspace per column: first-pass radn_dn and the radn_up of the up pass (nlev each), and with nmus > 1
  // the per-g flux accumulators (dn, up)
  float *wcol = ws + (size_t)(multi ? 4 : 2) * nlev * ngpt * icol;
  float *WD = wcol, *WU = wcol + (size_t)nlev * ngpt, *acc_base = wcol + (size_t)2 * nlev * ngpt;
  const size_t cl = (size_t)ngpt * nlay * icol, cv = (size_t)ngpt * nlev * icol;
  auto X = [&](int l) { return (size_t)gc + (size_t)ngpt * l; };
  const float *tc = tau + cl, *wc = ssa + cl, *gcol = gg + cl, *yc = lay + cl, *vc = lev + cv;
  const float e = emis[gc + (size_t)ngpt * icol], ss = sfc[gc + (size_t)ngpt * icol];
  const float inc = inc_flux ? inc_flux[gc + (size_t)ngpt * icol] : 0.0f;
  auto layer = [&](int l, float D) {
    return rs_layer(tc[X(l)], wc[X(l)], gcol[X(l)], D, yc[X(l)], vc[X(l)], vc[X(l + 1)], etab);
  };
  const int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0, dl_dn = top_at_1 ? 1 : -1;
  float *pdn = part, *pup = part + (size_t)nlev * 4;

  for (int imu = 0; imu < ang.nmus; imu++) {
    const float D = ang.D[imu];
    const float fac = (multi || (ngpt & 3) == 0) ? 2.0f * kPi * ang.w[imu] : 1.0f;  // quirk B-5 as noscat
    const bool acc = imu > 0;
    // v = fac * radiance; rad = the radiance
    auto put = [&](float v, float rad, int r, int q, int level) {
      if (!on) return;
      if (multi) {
        float *w = (gpt ? (q == 0 ? gdn : gup) + (size_t)level * ngpt : acc_base + ((size_t)q * nlev + level) * ngpt) + g;
        *w = acc ? *w + v : v;
      } else {
        ring[(size_t)r * ngpt + g] = v;
        if (gpt) (q == 0 ? gdn : gup)[(size_t)level * ngpt + g] = rad;
      }
    };
    auto flush = [&](float *pq, int n, int lev0, int dl) {
      if (!multi) ring_flush<kScatRing>(ring, pq, 1, n, lev0, dl, ngpt, nlev, false);
    };
    // 1: no-scattering transport down with the rescaled optics (lw_transport_noscat_dn)
    const float I0 = inc / (2.0f * kPi * ang.w[imu]);
    float I = I0;
    if (on) WD[X(top)] = I;
    for (int j = 0; j < nlay; j++) {
      const int l = top_at_1 ? j : nlay - 1 - j;
      const RsLayer r = layer(l, D);
      I = r.trans * I + r.sdn;
      if (on) WD[X(top_at_1 ? l + 1 : l)] = I;
    }
    // surface reflection and emission
    float U = I * (1.0f - e) + e * ss;
    if (on) WU[X(sfcl)] = U;
    put(fac * U, U, 0, 1, sfcl);
    flush(pup, 1, sfcl, 1);
    // 2: up with the adjustment from the first-pass radiance at the layer top (lw_transport_1rescl)
    for (int j0 = 0; j0 < nlay; j0 += kScatRing) {
      for (int s = 0; s < kScatRing; s++) {
        const int j = j0 + s;
        if (j < nlay) {
          const int l = top_at_1 ? nlay - 1 - j : j;
          const int ltop = top_at_1 ? l : l + 1;
          const RsLayer r = layer(l, D);
          const float adj = r.Cn * (r.An * WD[X(ltop)] - r.trans * r.sdn - r.sup);
          U = r.trans * U + r.sup + adj;
          if (on) WU[X(ltop)] = U;
          put(fac * U, U, s, 1, ltop);
        }
      }
      flush(pup, min(kScatRing, nlay - j0), sfcl - dl_dn * (j0 + 1), -dl_dn);
    }
    // 3: down again with the adjustment from radn_up(l) in array order: the layer top when top_at_1, the
    //    layer bottom otherwise (:1761-1767 vs :1783-1789, reproduced)
    I = I0;
    put(fac * I, I, 0, 0, top);
    flush(pdn, 1, top, 1);
    for (int j0 = 0; j0 < nlay; j0 += kScatRing) {
      for (int s = 0; s < kScatRing; s++) {
        const int j = j0 + s;
        if (j < nlay) {
          const int l = top_at_1 ? j : nlay - 1 - j;
          const RsLayer r = layer(l, D);
          const float adj = r.Cn * (r.An * WU[X(l)] - r.trans * r.sup - r.sdn);
          I = r.trans * I + r.sdn + adj;
          put(fac * I, I, s, 0, top_at_1 ? l + 1 : l);
        }
      }
      flush(pdn, min(kScatRing, nlay - j0), top + dl_dn * (j0 + 1), dl_dn);
    }
  }
  if (multi) {
    __syncthreads();
    for (int t = g; t < 2 * nlev; t += blockDim.x) {
      const float *w = gpt ? (t < nlev ? gdn : gup) + (size_t)(t % nlev) * ngpt : acc_base + (size_t)t * ngpt;
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

// lw_two_stream (:1018-1069) and lw_source_2str (:1112-1162) for one layer
struct L2Layer {
  float Rdif, Tdif, sdn, sup;
};

__device__ __forceinline__ L2Layer l2_layer(float tau, float w0, float g, float lev_top, float lev_bot,
                                            const uint64_t *etab)
{
  const float k_min = 1.e-4f, LW_diff_sec = 1.66f;
  L2Layer r;
  const float gamma1 = LW_diff_sec * (1.0f - 0.5f * w0 * (1.0f + g));
  const float gamma2 = LW_diff_sec * 0.5f * w0 * (1.0f - g);
  const float k = sqrtf(fmaxf((gamma1 - gamma2) * (gamma1 + gamma2), k_min));
  const float emk = solver_exp_neg(-tau * k, etab);
  const float em2k = emk * emk;
  const float RT = 1.0f / (k * (1.0f + em2k) + gamma1 * (1.0f - em2k));
  r.Rdif = RT * gamma2 * (1.0f - em2k);
  r.Tdif = RT * 2.0f * k * emk;
  if (tau > 1.0e-8f) {
    const float Z = (lev_bot - lev_top) / (tau * (gamma1 + gamma2));
    const float Zup_top = Z + lev_top, Zup_bottom = Z + lev_bot;
    const float Zdn_top = -Z + lev_top, Zdn_bottom = -Z + lev_bot;
    r.sup = kPi * (Zup_top - r.Rdif * Zdn_top - r.Tdif * Zup_bottom);
    r.sdn = kPi * (Zdn_bottom - r.Rdif * Zup_bottom - r.Tdif * Zdn_top);
  } else {
    r.sup = 0.0f;
    r.sdn = 0.0f;
  }
  return r;
}

__global__ void __launch_bounds__(256) lw_2stream_kernel(int ngpt, int nlay, int ncol, int top_at_1,
                                                         const float *__restrict__ inc_flux,
                                                         const float *__restrict__ tau, const float *__restrict__ ssa,
                                                         const float *__restrict__ gg, const float *__restrict__ lev,
                                                         const float *__restrict__ emis,
                                                         const float *__restrict__ sfc, float *__restrict__ ws,
                                                         float *__restrict__ flux_up, float *__restrict__ flux_dn,
                                                         float *__restrict__ gpt_up, float *__restrict__ gpt_dn)
{
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int icol = blockIdx.x, g = threadIdx.x;
  const bool on = g < ngpt;
  const int gc = on ? g : ngpt - 1;
  const int nlev = nlay + 1;
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  float *ring = smem + kExpTabFloats;                 // [2][kScatRing][ngpt]: up, dn
  float *part = ring + (size_t)2 * kScatRing * ngpt;  // [2][nlev][4]
  load_exp_table(etab);
  __syncthreads();
  // workspace per column: albedo and source of upward radiation at each level (adding, Eqs 9 and 11)
  float *WA = ws + (size_t)2 * nlev * ngpt * icol, *WS = WA + (size_t)nlev * ngpt;
  const size_t cl = (size_t)ngpt * nlay * icol, cv = (size_t)ngpt * nlev * icol;
  auto X = [&](int l) { return (size_t)gc + (size_t)ngpt * l; };
  const float *tc = tau + cl, *wc = ssa + cl, *gcol = gg + cl, *vc = lev + cv;
  auto layer = [&](int l) {
    const int lt = top_at_1 ? l : l + 1, lb = top_at_1 ? l + 1 : l;
    return l2_layer(tc[X(l)], wc[X(l)], gcol[X(l)], vc[X(lt)], vc[X(lb)], etab);
  };
  const float e = emis[gc + (size_t)ngpt * icol], ss = sfc[gc + (size_t)ngpt * icol];
  const int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0, dl_dn = top_at_1 ? 1 : -1;
  // bottom to top: albedo and source (adding :1555-1574 / :1595-1614)
  float alb_b = 1.0f - e, src_b = kPi * e * ss;
  if (on) {
    WA[X(sfcl)] = alb_b;
    WS[X(sfcl)] = src_b;
  }
  for (int j = 0; j < nlay; j++) {
    const int l = top_at_1 ? nlay - 1 - j : j;
    const L2Layer r = layer(l);
    const float denom = 1.0f / (1.0f - r.Rdif * alb_b);
    const float alb = r.Rdif + r.Tdif * r.Tdif * alb_b * denom;
    const float src = r.sup + r.Tdif * denom * (src_b + alb_b * r.sdn);
    if (on) {
      WA[X(top_at_1 ? l : l + 1)] = alb;
      WS[X(top_at_1 ? l : l + 1)] = src;
    }
    alb_b = alb;
    src_b = src;
  }
  // top to bottom: fluxes (Eqs 12-13), sum_broadband_nocol = sum(flux, 1): sequential over g
  // level `lev` of the g-point outputs (flux_up_gpt / flux_dn_gpt, :481-483), when asked for
  float *gu = gpt_up ? gpt_up + (size_t)ngpt * nlev * icol : nullptr, *gd = gpt_dn ? gpt_dn + (size_t)ngpt * nlev * icol : nullptr;
  auto put = [&](float up, float dn, int s, int lev) {
    if (on) {
      ring[(size_t)s * ngpt + g] = up;
      ring[((size_t)kScatRing + s) * ngpt + g] = dn;
      if (gu) {
        gu[(size_t)lev * ngpt + g] = up;
        gd[(size_t)lev * ngpt + g] = dn;
      }
    }
  };
  auto flush = [&](int n, int lev0, int dl) {
    ring_flush<kScatRing>(ring, part, 2, n, lev0, dl, ngpt, nlev, false, true);
  };
  float Fdn = (on && inc_flux) ? inc_flux[g + (size_t)ngpt * icol] : 0.0f;
  put(Fdn * alb_b + src_b, Fdn, 0, top);
  flush(1, top, 1);
  for (int j0 = 0; j0 < nlay; j0 += kScatRing) {
    for (int s = 0; s < kScatRing; s++) {
      const int j = j0 + s;
      if (j < nlay) {
        const int l = top_at_1 ? j : nlay - 1 - j, lbelow = top_at_1 ? l + 1 : l;
        const L2Layer r = layer(l);
        const float alb = WA[X(lbelow)], src = WS[X(lbelow)];
        const float denom = 1.0f / (1.0f - r.Rdif * alb);
        Fdn = (r.Tdif * Fdn + r.Rdif * src + r.sdn) * denom;
        put(Fdn * alb + src, Fdn, s, lbelow);
      }
    }
    flush(min(kScatRing, nlay - j0), top + dl_dn * (j0 + 1), dl_dn);
  }
  for (int l = g; l < nlev; l += blockDim.x) {
    flux_up[l + (size_t)nlev * icol] = combine4(part + 4 * l);
    flux_dn[l + (size_t)nlev * icol] = combine4(part + (size_t)nlev * 4 + 4 * l);
  }
}

int launch_lw_rescl(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus, const float *Ds,
                    const float *wts, const float *inc_flux, const float *tau, const float *ssa, const float *g,
                    const float *lay_source, const float *lev_source, const float *sfc_emis, const float *sfc_source,
                    float *flux_up, float *flux_dn)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (nmus < 1 || nmus > 4) return fail(RRTMGPNN_ERR_ARGUMENT, "lw solver: nmus must be 1..4");
  if (ngpt > 256) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw rescaled solver: more than 256 g-points");
  LwAngles a{};
  a.nmus = nmus;
  for (int i = 0; i < nmus; i++) { a.D[i] = Ds[i]; a.w[i] = wts[i]; }
  const int threads = (ngpt + 63) / 64 * 64;
  const size_t lds = sizeof(float) * (kExpTabFloats + (size_t)kScatRing * ngpt + (size_t)2 * (nlay + 1) * 4);
  if (lds > 64 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw rescaled solver: too many layers for LDS partials");
  void *ws = nullptr;
  if (int rc = ctx->workspace(sizeof(float) * (nmus > 1 ? 4 : 2) * (size_t)ngpt * (nlay + 1) * ncol, &ws)) return rc;
  const auto &ex = ctx->extras;
  if ((ex.gpt_up == nullptr) != (ex.gpt_dn == nullptr))
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw solver: g-point outputs need both gpt_flux_up and gpt_flux_dn");
  hipLaunchKernelGGL(lw_rescl_kernel, dim3(ncol), dim3(threads), lds, ctx->stream, ngpt, nlay, ncol, top_at_1, a,
                     inc_flux, tau, ssa, g, lay_source, lev_source, sfc_emis, sfc_source, (float *)ws, flux_up,
                     flux_dn, ex.gpt_up, ex.gpt_dn);
  RRTMGPNN_LAUNCH_CHECK("lw_rescl_kernel");
  return RRTMGPNN_OK;
}

int launch_lw_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                      const float *tau, const float *ssa, const float *g, const float *lev_source,
                      const float *sfc_emis, const float *sfc_source, float *flux_up, float *flux_dn)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (ngpt > 256) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw two-stream solver: more than 256 g-points");
  const int threads = (ngpt + 63) / 64 * 64;
  const size_t lds = sizeof(float) * (kExpTabFloats + (size_t)2 * kScatRing * ngpt + (size_t)2 * (nlay + 1) * 4);
  if (lds > 64 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "lw two-stream solver: too many layers for LDS partials");
  void *ws = nullptr;
  if (int rc = ctx->workspace(sizeof(float) * 2 * (size_t)ngpt * (nlay + 1) * ncol, &ws)) return rc;
  const auto &ex = ctx->extras;
  if ((ex.gpt_up == nullptr) != (ex.gpt_dn == nullptr))
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw solver: g-point outputs need both gpt_flux_up and gpt_flux_dn");
  hipLaunchKernelGGL(lw_2stream_kernel, dim3(ncol), dim3(threads), lds, ctx->stream, ngpt, nlay, ncol, top_at_1,
                     inc_flux, tau, ssa, g, lev_source, sfc_emis, sfc_source, (float *)ws, flux_up, flux_dn, ex.gpt_up,
                     ex.gpt_dn);
  RRTMGPNN_LAUNCH_CHECK("lw_2stream_kernel");
  return RRTMGPNN_OK;
}

}  // namespace rrtmgpnn
