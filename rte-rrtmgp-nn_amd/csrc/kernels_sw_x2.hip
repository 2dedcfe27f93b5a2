// kernels_sw_x2.hip -- the SW two-stream solver with two g-points per lane (packed fp32).
//
// Same algorithm, passes, workspace and ordered reductions as sw_2stream_kernel (kernels_rte.hip), but each
// lane carries g-points 2i and 2i+1 as a two-wide vector: the per-layer arithmetic -- products, sums and the
// fma chains of the correctly rounded reciprocal and square root -- issues as v_pk_mul_f32 / v_pk_add_f32 /
// v_pk_fma_f32 (two IEEE operations each, so the same bits as the scalar kernel), loads and stores move 8
// bytes per lane, and half as many lanes walk the column.  The glibc-exact exps (double precision), the IEEE
// divisions and the selects stay per element.  Used when ngpt is even.
#include "x2_device.hpp"

namespace rrtmgpnn {
using namespace x2;

namespace {

struct SwDif2 {
  f2 gamma1, gamma2, k, emk, em2k, RT, Rdif, Tdif;
};

__device__ __forceinline__ SwDif2 sw_dif2(f2 tau, f2 w0, f2 g, const uint64_t *etab)
{
  const float k_min = 1.e-4f;
  SwDif2 d;
  d.gamma1 = (8.0f - w0 * (5.0f + 3.0f * g)) * .25f;
  d.gamma2 = 3.0f * (w0 * (1.0f - g)) * .25f;
  d.k = sqrt2(vmax((d.gamma1 - d.gamma2) * (d.gamma1 + d.gamma2), splat(k_min)));
  d.emk = exp2v(-tau * d.k, etab);
  d.em2k = d.emk * d.emk;
  d.RT = rcp2(d.k * (1.0f + d.em2k) + d.gamma1 * (1.0f - d.em2k));
  d.Rdif = d.RT * d.gamma2 * (1.0f - d.em2k);
  d.Tdif = d.RT * 2.0f * d.k * d.emk;
  return d;
}

struct SwCoef2 {
  f2 Rdif, Tdif, Sup, Sdn, Tnoscat;
};

// sw_two_stream of kernels_rte.hip, term by term
template <bool kG0 = false>
__device__ __forceinline__ SwCoef2 sw_two_stream2(f2 tau, f2 w0, f2 g, float mu0, float mu0_inv, f2 dir_inc,
                                                 const uint64_t *etab)
{
  const float eps = FLT_EPSILON;
  SwCoef2 c;
  const SwDif2 d = sw_dif2(tau, w0, g, etab);
  const f2 gamma1 = d.gamma1, gamma2 = d.gamma2, k = d.k, emk = d.emk, em2k = d.em2k;
  const f2 Tnoscat = exp2v_beam(-tau * mu0_inv, etab);
  const f2 gamma3 = kG0 ? splat(0.5f) : (2.0f - 3.0f * mu0 * g) * .25f;  // g == 0: exactly 0.5
  const f2 gamma4 = 1.0f - gamma3;
  const f2 alpha1 = gamma1 * gamma4 + gamma2 * gamma3;
  const f2 alpha2 = gamma1 * gamma3 + gamma2 * gamma4;
  const f2 k2e = 2.0f * k * emk;
  c.Rdif = d.Rdif;
  c.Tdif = d.Tdif;
  const f2 k_mu = k * mu0, k_mu2 = k_mu * k_mu, k_g3 = k * gamma3, k_g4 = k * gamma4;
  const f2 omk = 1.0f - k_mu2;
  f2 dd;
  dd.x = (fabsf(omk.x) >= eps) ? omk.x : eps;
  dd.y = (fabsf(omk.y) >= eps) ? omk.y : eps;
  const f2 RT = div2(w0 * d.RT, dd);
  f2 Rdir = RT * ((1.0f - k_mu) * (alpha2 + k_g3) - (1.0f + k_mu) * (alpha2 - k_g3) * em2k -
                  k2e * (gamma3 - alpha2 * mu0) * Tnoscat);
  f2 Tdir = RT * (k2e * (gamma4 + alpha1 * mu0) -
                  Tnoscat * ((1.0f + k_mu) * (alpha1 + k_g4) - (1.0f - k_mu) * (alpha1 - k_g4) * em2k));
  Rdir = vmax(splat(0.0f), vmin(Rdir, (1.0f - Tnoscat)));
  Tdir = vmax(splat(0.0f), vmin(Tdir, (1.0f - Tnoscat - Rdir)));
  c.Sup = Rdir * dir_inc;
  c.Sdn = Tdir * dir_inc;
  c.Tnoscat = Tnoscat;
  return c;
}

// inc_2str of kernels_rte.hip for a pair
__device__ __forceinline__ void inc_2str2(f2 &t1, f2 &w1, f2 &g1, f2 t2, f2 w2, f2 g2)
{
  const float eps = 3.0f * FLT_MIN;
  const f2 tau12 = t1 + t2;
  const f2 tauscat12 = t1 * w1 + t2 * w2;
  g1 = (t1 * w1 * g1 + t2 * w2 * g2) / vmax(splat(eps), tauscat12);
  w1 = tauscat12 / vmax(splat(eps), tau12);
  t1 = tau12;
}

}  // namespace

// layers of inputs in flight per lane: 3 for the NN path's g = NULL kernel (C3 -1.5 %, C4 -2 %, no spill), 2 for the
// kernels that also read g (3 spilled there) and for the fused cloud increment
constexpr int kSw2Pf = 2, kSw2PfNoG = 3, kSw2PfInc = 2;
constexpr int kSw2Waves = 4;  // __launch_bounds__ minimum waves per SIMD
// Pass 3 of the clear-sky kernels recomputes the direct beam and the layer's full two-stream coefficients (S_dn
// included) instead of reading them back (3 fewer plane transfers per launch: the S_dn store + load, the beam's second
// read, for the ~250 VALU of a second sw_two_stream per g-point and layer); with the fused cloud increment pass 2
// stores S_dn and pass 3 reads it and the beam back, evaluating only R_dif / T_dif.  Chosen per instantiation by
// whole-step A/B (tools/ab_trees.sh, alternating runs of two trees on one box): the clear-sky NN path recomputes
// (storing was 1 % slower at C3); with the increment storing is 4.5 % faster alone and the C4 step 4 % faster.
// Storing more (R_dif / T_dif, the beam transmittance) was 5-10 % slower: more planes cost more than the VALU they
// save; a branch-free layer step was 2 % slower with the increment and within noise without (rounds 1-2).
constexpr bool kSw2Recomp = true, kSw2RecompInc = false;
constexpr int kSw2Ring = 6;  // levels staged per ordered flush (2, 4, 8 were 2-25 % slower)
// With the fused cloud increment, pass 3 forms the incremented (tau, ssa, g) again from the gas arrays and the
// band-resolved cloud arrays (same expressions, same bits) instead of reading three g-resolved planes pass 2 would park
// in workspace: 3 plane stores and 1 plane load fewer per launch (the band arrays are 16x smaller and stay in cache).

template <bool kHasG, bool kInc, int kPF>
__global__ void __launch_bounds__(512, kSw2Waves)
    sw_2stream_x2_kernel(int ngpt, int nlay, int ncol, int top_at_1, int ncb, const float *__restrict__ inc_flux,
                         const float *__restrict__ inc_dif, const float *__restrict__ tau,
                         const float *__restrict__ ssa, const float *__restrict__ gg, const float *__restrict__ mu0p,
                         const float *__restrict__ alb_dir, const float *__restrict__ alb_dif, BandArgs bands,
                         const float *__restrict__ tau_bnd, const float *__restrict__ ssa_bnd,
                         const float *__restrict__ g_bnd, float *__restrict__ ws, float *__restrict__ flux_up,
                         float *__restrict__ flux_dn, float *__restrict__ flux_dir)
{
  static_assert(kSw2Ring % kPF == 0, "prefetch depth must divide the ring");
  constexpr bool kRc = kInc ? kSw2RecompInc : kSw2Recomp;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // `ncb` columns per block (as sw_2stream_kernel): lane t works on column c = t / (ngpt/2), g-points g, g + 1
  const int nlev = nlay + 1, lanes = ngpt / 2;
  const int icol0 = blockIdx.x * ncb, nc = min(ncb, ncol - icol0);
  const int craw = (int)threadIdx.x / lanes;
  const bool on = craw < nc;
  const int c = on ? craw : nc - 1;
  const int g = 2 * ((int)threadIdx.x - craw * lanes);
  const int gc = on ? g : ngpt - 2;
  const int icol = icol0 + c;
  float *ring = smem + kExpTabFloats + (size_t)c * 3 * kSw2Ring * ngpt;  // this column's [3][kSw2Ring][ngpt]
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  load_exp_table(etab);
  __syncthreads();
  const uint32_t row = 4u * (uint32_t)ngpt;
  const uint32_t vL = 4u * (uint32_t)gc + (uint32_t)c * row * nlay, vV = 4u * (uint32_t)gc + (uint32_t)c * row * nlev;
  const size_t cl = (size_t)ngpt * nlay * icol0, cv = (size_t)ngpt * nlev * icol0, plane = (size_t)ngpt * nlev * ncol;
  const uint32_t bL = (uint32_t)nc * row * nlay, bV = (uint32_t)nc * row * nlev;
  const ColArr2 Ttau(tau, cl, bL), Tssa(ssa, cl, bL), Tg(kHasG ? gg : tau, cl, bL);
  const ColArr2 WA(ws, cv, bV), WB(ws + plane, cv, bV), WS(ws + 2 * plane, cv, bV), WD(ws + 3 * plane, cv, bV);
  // band-resolved increments: one band offset per g-point of the pair
  const size_t cb = (size_t)bands.nbnd * nlay * icol0;
  const uint32_t brow = 4u * (uint32_t)bands.nbnd, vbc = (uint32_t)c * brow * nlay;
  const uint32_t vb0 = kInc ? 4u * (uint32_t)band_of(bands, gc) + vbc : 0u,
                 vb1 = kInc ? 4u * (uint32_t)band_of(bands, gc + 1) + vbc : 0u;
  const uint32_t bB = kInc ? (uint32_t)nc * brow * nlay : 0u;
  const ColArr2 Bt(kInc ? tau_bnd : tau, kInc ? cb : 0, bB), Bw(kInc ? ssa_bnd : tau, kInc ? cb : 0, bB),
      Bg(kInc ? g_bnd : tau, kInc ? cb : 0, bB);
  auto ld_bnd = [&](const ColArr2 &a, int l) {
    return kInc ? (f2){a.ld1(vb0, brow * (uint32_t)l), a.ld1(vb1, brow * (uint32_t)l)} : splat(0.0f);
  };
  const float mu0 = mu0p[icol], mu0_inv = 1.0f / mu0;
  auto lev_above = [&](int l) { return top_at_1 ? l : l + 1; };
  auto lev_below = [&](int l) { return top_at_1 ? l + 1 : l; };
  auto lay_of_down = [&](int j) { return top_at_1 ? j : nlay - 1 - j; };
  auto lay_of_up = [&](int j) { return top_at_1 ? nlay - 1 - j : j; };
  auto ld_g = [&](uint32_t soff) { return kHasG ? Tg.ld(vL, soff) : splat(0.0f); };
  auto ld_col = [&](const float *p) { return on ? *(const f2 *)(p + gc + (size_t)ngpt * icol) : splat(0.0f); };
  const int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0;
  const f2 Ftop = ld_col(inc_flux) * mu0;

  // ---- pass 1: direct beam ----
  // Straight-line layer steps as in sw_2stream_kernel: memory operations on every step (idle lanes and steps past
  // nlay store at kBufOOB), arithmetic alone under the uniform `j < nlay` branch.
  const uint32_t vVs = on ? vV : kBufOOB;
  f2 Fd = Ftop;
  WA.st(Fd, vVs, row * top);
  {
    f2 pt[kPF], pi[kPF];
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
        const f2 t = kInc ? pt[p] + pi[p] : pt[p];
        {
          const int ln = lay_of_down(min(j + kPF, nlay - 1));
          pt[p] = Ttau.ld(vL, row * ln);
          pi[p] = ld_bnd(Bt, ln);
        }
        if (j < nlay) Fd = exp2v_beam(-t * mu0_inv, etab) * Fd;
        WA.st(Fd, j < nlay ? vVs : kBufOOB, row * lev_below(l));
      }
    }
  }
  // ---- pass 2: bottom -> top adding ----
  f2 alb_b = ld_col(alb_dif);
  f2 src_b = Fd * ld_col(alb_dir);
  WB.st(alb_b, vVs, row * sfcl);
  WS.st(src_b, vVs, row * sfcl);
  {
    f2 pt[kPF], pw[kPF], pg[kPF], pf[kPF], qt[kPF], qw[kPF], qg[kPF];
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
        const uint32_t vs = j < nlay ? vVs : kBufOOB;
        f2 t = pt[p], w0 = pw[p], g0 = kHasG ? pg[p] : splat(0.0f);
        const f2 Fin = pf[p];
        if constexpr (kInc) inc_2str2(t, w0, g0, qt[p], qw[p], qg[p]);
        load2(p, lay_of_up(min(j + kPF, nlay - 1)));
        f2 alb = alb_b, src = src_b, Sdn = splat(0.0f);
        if (j < nlay) {
          const SwCoef2 cf = sw_two_stream2<!kHasG && !kInc>(t, w0, g0, mu0, mu0_inv, Fin, etab);
          const f2 denom = rcp2(1.0f - cf.Rdif * alb_b);
          alb = cf.Rdif + cf.Tdif * cf.Tdif * alb_b * denom;
          src = cf.Sup + cf.Tdif * denom * (src_b + alb_b * cf.Sdn);
          Sdn = cf.Sdn;
        }
        const uint32_t sa = row * lev_above(l);
        WB.st(alb, vs, sa);
        WS.st(src, vs, sa);
        if constexpr (!kRc) WD.st(Sdn, vs, row * l);
        alb_b = alb;
        src_b = src;
      }
    }
  }
  // ---- pass 3: top -> bottom fluxes + ordered broadband sums ----
  auto put = [&](f2 up, f2 dif, f2 dir, int r) {
    if (on) {
      *(f2 *)&ring[(size_t)r * ngpt + g] = up;
      *(f2 *)&ring[((size_t)kSw2Ring + r) * ngpt + g] = dif;
      *(f2 *)&ring[((size_t)2 * kSw2Ring + r) * ngpt + g] = dir;
    }
  };
  auto flush = [&](int n, int lev0, int dl) {
    ring_flush_sw<kSw2Ring>(smem + kExpTabFloats, ncb, n, lev0, dl, ngpt, nlev, icol0, ncol, flux_up, flux_dn,
                            flux_dir);
  };
  const int dl_dn = top_at_1 ? 1 : -1;
  f2 Fdn = inc_dif ? ld_col(inc_dif) : splat(0.0f);
  put(Fdn * alb_b + src_b, Fdn, Ftop, 0);
  flush(1, top, 1);
  {
    f2 pt[kPF], pw[kPF], pg[kPF], pd[kPF], pa[kPF], ps[kPF], pf[kPF], qt[kPF], qw[kPF], qg[kPF];
    auto load = [&](int p, int l) {
      const uint32_t s = row * l, sb = row * lev_below(l);
      pt[p] = Ttau.ld(vL, s); pw[p] = Tssa.ld(vL, s); pg[p] = ld_g(s);
      if constexpr (kInc) {
        qt[p] = ld_bnd(Bt, l); qw[p] = ld_bnd(Bw, l); qg[p] = ld_bnd(Bg, l);
      }
      pa[p] = WB.ld(vV, sb); ps[p] = WS.ld(vV, sb);
      if constexpr (!kRc) {
        pd[p] = WD.ld(vV, s);
        pf[p] = WA.ld(vV, sb);
      }
    };
    f2 Fd3 = Ftop;  // kRc: the direct beam again, top down, exactly as pass 1 formed it
#pragma unroll
    for (int p = 0; p < kPF; p++) load(p, lay_of_down(min(p, nlay - 1)));
    for (int j0 = 0; j0 < nlay; j0 += kSw2Ring) {
#pragma unroll
      for (int r = 0; r < kSw2Ring; r++) {
        const int j = j0 + r, p = r % kPF;
        f2 t = pt[p], w0 = pw[p], g0 = kHasG ? pg[p] : splat(0.0f);
        if constexpr (kInc) inc_2str2(t, w0, g0, qt[p], qw[p], qg[p]);
        const f2 alb = pa[p], src = ps[p];
        f2 Rdif, Tdif, Sdn = kRc ? splat(0.0f) : pd[p], Fdir = kRc ? splat(0.0f) : pf[p];
        load(p, lay_of_down(min(j + kPF, nlay - 1)));
        if (j < nlay) {
          if constexpr (kRc) {
            // pass 2's coefficients from the same inputs (same bits), the beam from pass 1's recurrence
            const SwCoef2 cf = sw_two_stream2<!kHasG && !kInc>(t, w0, g0, mu0, mu0_inv, Fd3, etab);
            Rdif = cf.Rdif;
            Tdif = cf.Tdif;
            Sdn = cf.Sdn;
            Fd3 = cf.Tnoscat * Fd3;
            Fdir = Fd3;
          } else {
            const SwDif2 d = sw_dif2(t, w0, g0, etab);
            Rdif = d.Rdif;
            Tdif = d.Tdif;
          }
          const f2 denom = rcp2(1.0f - Rdif * alb);
          Fdn = (Tdif * Fdn + Rdif * src + Sdn) * denom;
          const f2 up = Fdn * alb + src;
          put(up, Fdn, Fdir, r);
        }
      }
      flush(min(kSw2Ring, nlay - j0), top + dl_dn * (j0 + 1), dl_dn);
    }
  }
}

// layer planes (ngpt x nlay x ncol floats) the x2 kernel needs after its 4 level planes: none
size_t sw_2stream_x2_layer_planes(bool) { return 0; }

// ngpt even and <= 256; workspace: 4 level planes + sw_2stream_x2_layer_planes(inc) layer planes
int launch_sw_2stream_x2(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                         const float *inc_flux_dif, const float *tau, const float *ssa, const float *g,
                         const float *mu0, const float *alb_dir, const float *alb_dif, const BandArgs *bands,
                         const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, void *ws, float *flux_up,
                         float *flux_dn, float *flux_dir)
{
  // Columns per block: 2 (224 g-points: 224 lanes in 4 waves, 32 idle, a 32 KB ring).  Four columns fill 7 waves
  // exactly and were 5 % faster alone at C4, but in the overlapped step the smaller blocks share the CUs better with
  // the LW chain: whole step C3 -1.7 %, C4 -3.5 % (tools/ab_env.sh RRTMGPNN_LIB).
  const int ncb = 2 * (ngpt / 2) <= 512 ? 2 : columns_per_block(ngpt / 2);
  const int threads = (ncb * (ngpt / 2) + 63) / 64 * 64;
  const size_t lds = sizeof(float) * (kExpTabFloats + (size_t)ncb * 3 * kSw2Ring * ngpt);
  if (lds > 160 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: LDS ring exceeds 160 KiB");
  const BandArgs nob{};
  const BandArgs &b = bands ? *bands : nob;
  const dim3 grid((ncol + ncb - 1) / ncb), block(threads);
  constexpr int PF = kSw2Pf, PFN = kSw2PfNoG, PFI = kSw2PfInc;
  auto go = [&](auto kern, const float *tb, const float *sb, const float *gb) -> int {
    // rings past 64 KiB (4 columns of 224 g-points: 64.5 KiB) need the dynamic-LDS limit raised (per device)
    if (lds > 64 * 1024)
      if (int rc = raise_lds_limit((const void *)kern)) return rc;
    hipLaunchKernelGGL(kern, grid, block, lds, ctx->stream, ngpt, nlay, ncol, top_at_1, ncb, inc_flux, inc_flux_dif,
                       tau, ssa, g, mu0, alb_dir, alb_dif, b, tb, sb, gb, (float *)ws, flux_up, flux_dn, flux_dir);
    RRTMGPNN_LAUNCH_CHECK("sw_2stream_x2_kernel");
    return RRTMGPNN_OK;
  };
  if (bands && g) return go(sw_2stream_x2_kernel<true, true, PF>, tau_bnd, ssa_bnd, g_bnd);
  if (bands) return go(sw_2stream_x2_kernel<false, true, PFI>, tau_bnd, ssa_bnd, g_bnd);
  if (g) return go(sw_2stream_x2_kernel<true, false, PF>, nullptr, nullptr, nullptr);
  return go(sw_2stream_x2_kernel<false, false, PFN>, nullptr, nullptr, nullptr);
}

}  // namespace rrtmgpnn
