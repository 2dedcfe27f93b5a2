// kernels_sw_ck.hip -- the SW two-stream solver with checkpointed passes (two g-points per lane, packed fp32).
//
// Same arithmetic as sw_2stream_x2_kernel (kernels_sw_x2.hip) and so the same bits as the reference's
// sw_solver_2stream + sw_two_stream_source + adding (rte/kernels/mo_rte_solver_kernels.F90:541-692, 1366-1480,
// 1526-1637), but the three per-level workspace planes (direct beam, adding albedo, adding source: 3 x 98 MB written
// and read back at C3) are replaced by checkpoints every K levels:
//
//   pass 1 (top -> bottom) : direct beam; stores the beam at the top of every chunk of K layers (1/K of a plane).
//   pass 2 (bottom -> top) : per chunk, from the chunk's beam checkpoint: the beam forward through the chunk (its
//                            transmittances exp(-tau/mu0) are the ones sw_two_stream needs anyway, passed in), then the
//                            adding albedo / source backward through it; stores them at the top of every chunk.
//   pass 3 (top -> bottom) : per chunk: sw_two_stream of its K layers (the beam carried from the top as in pass 1),
//                            albedo / source walked up from the checkpoint at the chunk's bottom (pass 2's recurrence,
//                            same expressions, same bits), then the fluxes walked down (Eqs 12-13), into the ordered
//                            broadband reduction's LDS ring.
//
// Per launch this reads tau three times and ssa twice (as before) but moves 3/K planes of checkpoints instead of 6
// planes of workspace.  The VALU work per element is pass 2's and 3's sw_two_stream plus one more adding step in pass
// 3; the K layers of a chunk are independent until the recurrences, which gives the scheduler K-wide ILP.
// Workspace: (ngpt, nck, ncol) beam checkpoints, then (ngpt, nck+1, ncol) albedo and source checkpoints, nck =
// ceil(nlay / K); index c holds level c*K counted from the top, index nck the surface.
#include "x2_device.hpp"

#include <algorithm>

namespace rrtmgpnn {
using namespace x2;

namespace {

struct Dif2 {
  f2 Rdif, Tdif, RT, k, emk, em2k, gamma1, gamma2;
};

__device__ __forceinline__ Dif2 ck_dif(f2 tau, f2 w0, f2 g, const uint64_t *etab)
{
  const float k_min = 1.e-4f;
  Dif2 d;
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

struct Coef2 {
  f2 Rdif, Tdif, Sup, Sdn;
};

// sw_two_stream (kernels_rte.hip) term by term, with the direct-beam transmittance Tnoscat = exp(-tau/mu0) given
template <bool kG0>
__device__ __forceinline__ Coef2 ck_two_stream(f2 tau, f2 w0, f2 g, float mu0, f2 Tnoscat, f2 dir_inc,
                                               const uint64_t *etab)
{
  const float eps = FLT_EPSILON;
  Coef2 c;
  const Dif2 d = ck_dif(tau, w0, g, etab);
  const f2 gamma1 = d.gamma1, gamma2 = d.gamma2, k = d.k, emk = d.emk, em2k = d.em2k;
  const f2 gamma3 = (kG0 && RRTMGPNN_FASTOPS) ? splat(0.5f) : (2.0f - 3.0f * mu0 * g) * .25f;
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
  return c;
}

// inc_2stream_by_2stream_bybnd (rte/kernels/mo_optical_props_kernels.F90:430-463) for a pair, as inc_2str2
__device__ __forceinline__ void ck_inc(f2 &t1, f2 &w1, f2 &g1, f2 t2, f2 w2, f2 g2)
{
  const float eps = 3.0f * FLT_MIN;
  const f2 tau12 = t1 + t2;
  const f2 tauscat12 = t1 * w1 + t2 * w2;
  g1 = (t1 * w1 * g1 + t2 * w2 * g2) / vmax(splat(eps), tauscat12);
  w1 = tauscat12 / vmax(splat(eps), tau12);
  t1 = tau12;
}

}  // namespace

// K: layers per chunk (checkpoint spacing); RING: levels staged for the ordered broadband sums (a multiple of K)
#ifndef RRTMGPNN_SWCK_K
#define RRTMGPNN_SWCK_K 3
#endif
#ifndef RRTMGPNN_SWCK_RING
#define RRTMGPNN_SWCK_RING 6
#endif
// K = 3 layers per chunk under a 3-waves-per-SIMD register budget (132 VGPRs, no spill; at 4 waves K = 3 spilled and
// K = 2 fit): C3 step -3 %, C4 -1 % against K = 2 or the two-per-lane workspace kernel; K = 4 (148 VGPRs) was best
// alone at C3 but 13 % slower at C4, K = 6 spilled (tools/gpu_ab.sh, round 2)
#ifndef RRTMGPNN_SWCK_WAVES
#define RRTMGPNN_SWCK_WAVES 3
#endif
// KEEPD = 1: the walk up keeps each layer's adding denominator for the walk down (K more register pairs); 0: the walk
// down forms it again (one more reciprocal per element, fewer registers)
#ifndef RRTMGPNN_SWCK_KEEPD
#define RRTMGPNN_SWCK_KEEPD 1
#endif
constexpr bool kCkKeepD = RRTMGPNN_SWCK_KEEPD != 0;
constexpr int kCkK = RRTMGPNN_SWCK_K, kCkRing = RRTMGPNN_SWCK_RING;

// Waves per SIMD of the clear-sky NN instance (g = NULL, no increment), which needs fewer registers: at 4 (128 VGPRs,
// 2 spilled) the C3 grid (900 blocks of 4 waves) is resident at once instead of 768 + a second round of 132; SW solver
// -2.5 % at C3, step -0.7 %, C5 shard equal (tools/gpu_ab.sh, round 2)
#ifndef RRTMGPNN_SWCK_WAVES_NN
#define RRTMGPNN_SWCK_WAVES_NN 4
#endif

// kGpt: also store the g-point fluxes (ty_fluxes_flexible: up, total down, direct; (ngpt, nlay+1, ncol)) and sum the
// broadband down flux from the total as sw_solver_2stream does when it saves them (:572-588, :660-684)
// Small grids (the clear-sky instance when the grid fits in one round of resident waves, e.g. C3): K = 4 layers per
// chunk at 2 waves per SIMD (more independent layers per wave where there are too few waves to hide the exps'
// latency), ring of 8 levels.  Whole-step A/B at C3 (one box, alternating): +1.3 %, SW solver -2.4 %; a ring of 4 was
// 3 % slower, K = 2 at 4 waves +0.5 %.  With many columns (C4, C5) K = 3 at 3-4 waves stays (K = 4 was 13 % slower).
#ifndef RRTMGPNN_SWCK_SMALL
#define RRTMGPNN_SWCK_SMALL 1
#endif
#ifndef RRTMGPNN_SWCK_K_SMALL
#define RRTMGPNN_SWCK_K_SMALL 4
#endif
#ifndef RRTMGPNN_SWCK_RING_SMALL
#define RRTMGPNN_SWCK_RING_SMALL 8
#endif
#ifndef RRTMGPNN_SWCK_WAVES_SMALL
#define RRTMGPNN_SWCK_WAVES_SMALL 2
#endif
constexpr int kCkKSmall = RRTMGPNN_SWCK_K_SMALL, kCkRingSmall = RRTMGPNN_SWCK_RING_SMALL,
              kCkWavesSmall = RRTMGPNN_SWCK_WAVES_SMALL;
// the small-grid instance keeps pass 1's beam transmittances exp(-tau/mu0) in a workspace plane and passes 2 and 3 read
// them (one more plane written and two read) instead of evaluating the exp again
#ifndef RRTMGPNN_SWCK_TN_SMALL
#define RRTMGPNN_SWCK_TN_SMALL 1
#endif
constexpr bool kCkTnSmall = RRTMGPNN_SWCK_TN_SMALL != 0;
// the same for the all-sky instances (fused cloud increment), whatever the grid
#ifndef RRTMGPNN_SWCK_TN_INC
#define RRTMGPNN_SWCK_TN_INC 0
#endif
constexpr bool kCkTnInc = RRTMGPNN_SWCK_TN_INC != 0;

template <bool kHasG, bool kInc, int K, bool kGpt = false, int R = kCkRing,
          int WAVES = (!kHasG && !kInc && !kGpt) ? RRTMGPNN_SWCK_WAVES_NN : RRTMGPNN_SWCK_WAVES, bool kTn = false>
__global__ void __launch_bounds__(512, WAVES)
    sw_2stream_ck_kernel(int ngpt, int nlay, int ncol, int top_at_1, int ncb, const float *__restrict__ inc_flux,
                         const float *__restrict__ inc_dif, const float *__restrict__ tau,
                         const float *__restrict__ ssa, const float *__restrict__ gg, const float *__restrict__ mu0p,
                         const float *__restrict__ alb_dir, const float *__restrict__ alb_dif, BandArgs bands,
                         const float *__restrict__ tau_bnd, const float *__restrict__ ssa_bnd,
                         const float *__restrict__ g_bnd, float *__restrict__ ws, float *__restrict__ flux_up,
                         float *__restrict__ flux_dn, float *__restrict__ flux_dir, float *__restrict__ gpt_up,
                         float *__restrict__ gpt_dn, float *__restrict__ gpt_dir)
{
  static_assert(R % K == 0, "the flux ring must hold whole chunks");
  constexpr bool kG0 = !kHasG && !kInc;  // g is the literal 0 (the NN path)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // `ncb` columns per block: lane t works on column c = t / (ngpt/2), g-points g, g + 1
  const int nlev = nlay + 1, lanes = ngpt / 2, nck = (nlay + K - 1) / K;
  const int icol0 = blockIdx.x * ncb, nc = min(ncb, ncol - icol0);
  const int craw = (int)threadIdx.x / lanes;
  const bool on = craw < nc;
  const int c = on ? craw : nc - 1;
  const int g = 2 * ((int)threadIdx.x - craw * lanes);
  const int gc = on ? g : ngpt - 2;
  const int icol = icol0 + c;
  float *ring = smem + kExpTabFloats + (size_t)c * 3 * R * ngpt;  // this column's [3][R][ngpt]
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  load_exp_table(etab);
  __syncthreads();
  const uint32_t row = 4u * (uint32_t)ngpt;
  const uint32_t vL = 4u * (uint32_t)gc + (uint32_t)c * row * nlay;
  const size_t cl = (size_t)ngpt * nlay * icol0;
  const uint32_t bL = (uint32_t)nc * row * nlay;
  const ColArr2 Ttau(tau, cl, bL), Tssa(ssa, cl, bL), Tg(kHasG ? gg : tau, cl, bL);
  // checkpoints: beam (ngpt, nck, ncol), albedo and source (ngpt, nck+1, ncol)
  const size_t pB = (size_t)ngpt * nck * ncol, pA = (size_t)ngpt * (nck + 1) * ncol;
  const uint32_t vB = 4u * (uint32_t)gc + (uint32_t)c * row * nck, vA = 4u * (uint32_t)gc + (uint32_t)c * row * (nck + 1);
  const ColArr2 CB(ws, (size_t)ngpt * nck * icol0, (uint32_t)nc * row * nck);
  const ColArr2 CA(ws + pB, (size_t)ngpt * (nck + 1) * icol0, (uint32_t)nc * row * (nck + 1));
  const ColArr2 CS(ws + pB + pA, (size_t)ngpt * (nck + 1) * icol0, (uint32_t)nc * row * (nck + 1));
  // kTn: the beam transmittances (ngpt, nlay, ncol), addressed as tau
  const ColArr2 CT(kTn ? ws + pB + 2 * pA : ws, kTn ? cl : 0, kTn ? bL : 0u);
  const uint32_t vBs = on ? vB : kBufOOB, vAs = on ? vA : kBufOOB;
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
  // j counts layers from the top (clamped to the last layer); the result is the array layer
  auto lay = [&](int j) { return top_at_1 ? min(j, nlay - 1) : nlay - 1 - min(j, nlay - 1); };
  auto ld_col = [&](const float *p) { return on ? *(const f2 *)(p + gc + (size_t)ngpt * icol) : splat(0.0f); };
  const int top = top_at_1 ? 0 : nlay;
  const f2 Ftop = ld_col(inc_flux) * mu0;

  // one chunk's optical properties (the band increment is formed as they are used, as inc_2str2 does)
  struct Chunk {
    f2 t[K], w[K], g[K], qt[K], qw[K], qg[K], tn[K];
  };
  auto load_chunk = [&](Chunk &ch, int ck, bool with_ssa) {
#pragma unroll
    for (int p = 0; p < K; p++) {
      const int l = lay(ck * K + p);
      const uint32_t s = row * (uint32_t)l;
      ch.t[p] = Ttau.ld(vL, s);
      ch.tn[p] = kTn && with_ssa ? CT.ld(vL, s) : splat(0.0f);
      ch.w[p] = with_ssa ? Tssa.ld(vL, s) : splat(0.0f);
      ch.g[p] = kHasG && with_ssa ? Tg.ld(vL, s) : splat(0.0f);
      if constexpr (kInc) {
        ch.qt[p] = ld_bnd(Bt, l);
        ch.qw[p] = with_ssa ? ld_bnd(Bw, l) : splat(0.0f);
        ch.qg[p] = with_ssa ? ld_bnd(Bg, l) : splat(0.0f);
      } else {
        ch.qt[p] = ch.qw[p] = ch.qg[p] = splat(0.0f);
      }
    }
  };
  // the (incremented) properties of layer p of a chunk
  auto props = [&](const Chunk &ch, int p, f2 &t, f2 &w, f2 &g0) {
    t = ch.t[p];
    w = ch.w[p];
    g0 = kHasG ? ch.g[p] : splat(0.0f);
    if constexpr (kInc) ck_inc(t, w, g0, ch.qt[p], ch.qw[p], ch.qg[p]);
  };

  // ---- pass 1: direct beam, checkpoint at every chunk top ----
  f2 Fd = Ftop;
  {
    Chunk cur, nxt;
    load_chunk(cur, 0, false);
    for (int ck = 0; ck < nck; ck++) {
      CB.st(Fd, vBs, row * (uint32_t)ck);
      load_chunk(nxt, min(ck + 1, nck - 1), false);
      const int n = min(K, nlay - ck * K);
      f2 Tn[K];
#pragma unroll
      for (int p = 0; p < K; p++) Tn[p] = exp2v_beam(-(kInc ? cur.t[p] + cur.qt[p] : cur.t[p]) * mu0_inv, etab);
      if constexpr (kTn) {
#pragma unroll
        for (int p = 0; p < K; p++) CT.st(Tn[p], (on && p < n) ? vL : kBufOOB, row * (uint32_t)lay(ck * K + p));
      }
#pragma unroll
      for (int p = 0; p < K; p++)
        if (p < n) Fd = Tn[p] * Fd;
      cur = nxt;
    }
  }
  // ---- pass 2: bottom -> top adding; albedo / source checkpoint at every chunk top and at the surface ----
  f2 alb_b = ld_col(alb_dif);
  f2 src_b = Fd * ld_col(alb_dir);
  CA.st(alb_b, vAs, row * (uint32_t)nck);
  CS.st(src_b, vAs, row * (uint32_t)nck);
  {
    Chunk cur, nxt;
    load_chunk(cur, nck - 1, true);
    f2 Fb = CB.ld(vB, row * (uint32_t)(nck - 1));
    for (int ck = nck - 1; ck >= 0; ck--) {
      const int n = min(K, nlay - ck * K);
      load_chunk(nxt, max(ck - 1, 0), true);
      const f2 Fbn = CB.ld(vB, row * (uint32_t)max(ck - 1, 0));
      f2 t[K], w[K], g0[K], Tn[K], Fin[K];
#pragma unroll
      for (int p = 0; p < K; p++) {
        props(cur, p, t[p], w[p], g0[p]);
        Tn[p] = kTn ? cur.tn[p] : exp2v_beam(-t[p] * mu0_inv, etab);  // pass 1's transmittance, same bits
        Fin[p] = Fb;                           // the beam at the layer's top
        Fb = Tn[p] * Fb;
      }
#pragma unroll
      for (int p = K - 1; p >= 0; p--) {
        if (p < n) {
          const Coef2 cf = ck_two_stream<kG0>(t[p], w[p], g0[p], mu0, Tn[p], Fin[p], etab);
          const f2 denom = rcp2(1.0f - cf.Rdif * alb_b);
          const f2 alb = cf.Rdif + cf.Tdif * cf.Tdif * alb_b * denom;
          const f2 src = cf.Sup + cf.Tdif * denom * (src_b + alb_b * cf.Sdn);
          alb_b = alb;
          src_b = src;
        }
      }
      CA.st(alb_b, ck > 0 ? vAs : kBufOOB, row * (uint32_t)ck);
      CS.st(src_b, ck > 0 ? vAs : kBufOOB, row * (uint32_t)ck);
      cur = nxt;
      Fb = Fbn;
    }
  }
  // ---- pass 3: top -> bottom fluxes + ordered broadband sums ----
  // level `lev` (array index) of the g-point outputs
  auto put = [&](f2 up, f2 dif, f2 dir, int r, int lev) {
    if (on) {
      const f2 dn = kGpt ? dif + dir : dif;  // kGpt: the total, rounded once ("flux_dn is total", :665-666)
      *(f2 *)&ring[(size_t)r * ngpt + g] = up;
      *(f2 *)&ring[((size_t)R + r) * ngpt + g] = dn;
      *(f2 *)&ring[((size_t)2 * R + r) * ngpt + g] = dir;
      if constexpr (kGpt) {
        const size_t o = (size_t)g + (size_t)ngpt * ((size_t)lev + (size_t)nlev * icol);
        *(f2 *)&gpt_up[o] = up;
        *(f2 *)&gpt_dn[o] = dn;
        *(f2 *)&gpt_dir[o] = dir;
      }
    }
  };
  auto flush = [&](int n, int lev0, int dl) {
    ring_flush_sw<R, kGpt>(smem + kExpTabFloats, ncb, n, lev0, dl, ngpt, nlev, icol0, ncol, flux_up, flux_dn,
                           flux_dir);
  };
  const int dl_dn = top_at_1 ? 1 : -1;
  f2 Fdn = inc_dif ? ld_col(inc_dif) : splat(0.0f);
  put(Fdn * alb_b + src_b, Fdn, Ftop, 0, top);
  flush(1, top, 1);
  {
    Chunk cur, nxt;
    load_chunk(cur, 0, true);
    f2 albE = CA.ld(vA, row * 1u), srcE = CS.ld(vA, row * 1u);  // level min(K, nlay): the chunk's bottom
    f2 Fd3 = Ftop;
    for (int ck = 0; ck < nck; ck++) {
      const int n = min(K, nlay - ck * K);
      load_chunk(nxt, min(ck + 1, nck - 1), true);
      const uint32_t sE = row * (uint32_t)min(ck + 2, nck);
      const f2 albN = CA.ld(vA, sE), srcN = CS.ld(vA, sE);
      // the chunk's coefficients, top down, the beam carried as pass 1 carries it
      f2 Rd[K], Td[K], Su[K], Sd[K], Fdir[K];
#pragma unroll
      for (int p = 0; p < K; p++) {
        f2 t, w, g0;
        props(cur, p, t, w, g0);
        const f2 Tn = kTn ? cur.tn[p] : exp2v_beam(-t * mu0_inv, etab);
        const Coef2 cf = ck_two_stream<kG0>(t, w, g0, mu0, Tn, Fd3, etab);
        Rd[p] = cf.Rdif;
        Td[p] = cf.Tdif;
        Su[p] = cf.Sup;
        Sd[p] = cf.Sdn;
        if (p < n) Fd3 = Tn * Fd3;
        Fdir[p] = Fd3;  // the beam at the layer's bottom
      }
      // albedo / source at levels ck*K + p + 1 (A[p], S[p]), walked up from the checkpoint with pass 2's expressions;
      // D[p] = 1 / (1 - R_dif(p) * A[p]) is the adding denominator both walks use
      f2 A[K], S[K], D[K];
      {
        f2 a = albE, s = srcE;
#pragma unroll
        for (int p = K - 1; p >= 0; p--) {
          A[p] = a;
          S[p] = s;
          if (kCkKeepD) D[p] = splat(0.0f);
          if (p < n) {
            const f2 denom = rcp2(1.0f - Rd[p] * a);
            if (kCkKeepD) D[p] = denom;
            if (p > 0) {
              const f2 an = Rd[p] + Td[p] * Td[p] * a * denom;
              const f2 sn = Su[p] + Td[p] * denom * (s + a * Sd[p]);
              a = an;
              s = sn;
            }
          }
        }
      }
      // fluxes down the chunk (adding :1583-1591, Eqs 12-13)
      const int rbase = (ck * K) % R;
#pragma unroll
      for (int p = 0; p < K; p++) {
        if (p < n) {
          const f2 denom = kCkKeepD ? D[p] : rcp2(1.0f - Rd[p] * A[p]);
          Fdn = (Td[p] * Fdn + Rd[p] * S[p] + Sd[p]) * denom;
          const f2 up = Fdn * A[p] + S[p];
          put(up, Fdn, Fdir[p], rbase + p, top + dl_dn * (ck * K + p + 1));
        }
      }
      if (rbase + K == R || ck == nck - 1) {
        const int j0 = ck * K - rbase;  // first layer of this ring's levels
        flush(min(R, nlay - j0), top + dl_dn * (j0 + 1), dl_dn);
      }
      cur = nxt;
      albE = albN;
      srcE = srcN;
    }
  }
}

bool sw_ck_small(const rrtmgpnn_context *ctx, int ngpt, int ncol, bool has_g, bool inc, bool gpt)
{
  // 2 g-points per lane; one round of 16 waves of 64 lanes per CU
  return RRTMGPNN_SWCK_SMALL && !has_g && !inc && !gpt && (long long)ncol * (ngpt / 2) <= 64LL * 16 * ctx->num_cus;
}

// workspace floats of the checkpointed kernel (sized for the smaller of the chunk lengths, so it holds either
// instance; small: plus the small-grid instance's plane of beam transmittances)
size_t sw_2stream_ck_ws_floats(int ngpt, int nlay, int ncol, bool small, bool inc)
{
  const size_t tn = (small && kCkTnSmall) || (inc && kCkTnInc) ? (size_t)ngpt * nlay * ncol : 0;
  const int k = std::min(kCkK, kCkKSmall);
  const size_t nck = (size_t)(nlay + k - 1) / k;
  return (size_t)ngpt * ncol * (nck + 2 * (nck + 1)) + tn;
}

// ngpt even and <= 256
int launch_sw_2stream_ck(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                         const float *inc_flux_dif, const float *tau, const float *ssa, const float *g,
                         const float *mu0, const float *alb_dir, const float *alb_dif, const BandArgs *bands,
                         const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, void *ws, float *flux_up,
                         float *flux_dn, float *flux_dir)
{
#ifndef RRTMGPNN_SWCK_NCB
#define RRTMGPNN_SWCK_NCB 2
#endif
  const int ncb = RRTMGPNN_SWCK_NCB * (ngpt / 2) <= 512 ? RRTMGPNN_SWCK_NCB : 1;
  const int threads = (ncb * (ngpt / 2) + 63) / 64 * 64;
  const BandArgs nob{};
  const BandArgs &b = bands ? *bands : nob;
  const dim3 grid((ncol + ncb - 1) / ncb), block(threads);
  const auto &ex = ctx->extras;
  size_t lds = 0;
  auto lds_for = [&](int ring) { return sizeof(float) * (kExpTabFloats + (size_t)ncb * 3 * ring * ngpt); };
  auto go = [&](auto kern, const float *tb, const float *sb, const float *gb, int ring = kCkRing) -> int {
    lds = lds_for(ring);
    if (lds > 160 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: LDS ring exceeds 160 KiB");
    if (lds > 64 * 1024)
      if (int rc = raise_lds_limit((const void *)kern)) return rc;
    hipLaunchKernelGGL(kern, grid, block, lds, ctx->stream, ngpt, nlay, ncol, top_at_1, ncb, inc_flux, inc_flux_dif,
                       tau, ssa, g, mu0, alb_dir, alb_dif, b, tb, sb, gb, (float *)ws, flux_up, flux_dn, flux_dir,
                       ex.gpt_up, ex.gpt_dn, ex.gpt_dir);
    RRTMGPNN_LAUNCH_CHECK("sw_2stream_ck_kernel");
    return RRTMGPNN_OK;
  };
  if (ex.gpt_up || ex.gpt_dn || ex.gpt_dir) {  // ty_fluxes_flexible g-point outputs
    if (!ex.gpt_up || !ex.gpt_dn || !ex.gpt_dir)
      return fail(RRTMGPNN_ERR_ARGUMENT, "sw solver: g-point outputs need gpt_flux_up, gpt_flux_dn and gpt_flux_dn_dir");
    if (bands) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: g-point outputs with a fused increment");
    if (g) return go(sw_2stream_ck_kernel<true, false, kCkK, true>, nullptr, nullptr, nullptr);
    return go(sw_2stream_ck_kernel<false, false, kCkK, true>, nullptr, nullptr, nullptr);
  }
  constexpr int kW = RRTMGPNN_SWCK_WAVES;
  if (bands && g) return go(sw_2stream_ck_kernel<true, true, kCkK, false, kCkRing, kW, kCkTnInc>, tau_bnd, ssa_bnd, g_bnd);
  if (bands) return go(sw_2stream_ck_kernel<false, true, kCkK, false, kCkRing, kW, kCkTnInc>, tau_bnd, ssa_bnd, g_bnd);
  if (g) return go(sw_2stream_ck_kernel<true, false, kCkK>, nullptr, nullptr, nullptr);
  // the small-grid instance when the clear-sky grid fits in one round of resident waves (2 g-points per lane, 16
  // waves per CU)
  if (sw_ck_small(ctx, ngpt, ncol, false, false, false))
    return go(sw_2stream_ck_kernel<false, false, kCkKSmall, false, kCkRingSmall, kCkWavesSmall, kCkTnSmall>, nullptr,
              nullptr, nullptr, kCkRingSmall);
  return go(sw_2stream_ck_kernel<false, false, kCkK>, nullptr, nullptr, nullptr);
}

}  // namespace rrtmgpnn
