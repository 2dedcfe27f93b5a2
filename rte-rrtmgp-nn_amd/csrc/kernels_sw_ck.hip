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
// Workspace: (ngpt, 3 nck + 2, ncol) checkpoints, per column nck beam rows, then nck+1 albedo and nck+1 source rows,
// nck = ceil(nlay / K); row c of each holds level c*K counted from the top, albedo / source row nck the surface.
#include "x2_device.hpp"

#include <algorithm>
#include <type_traits>

namespace rrtmgpnn {
using namespace x2;

namespace {

// V: one lane's g-points, f2 (two per lane, packed fp32) or float (one per lane)
template <class V>
struct Coef2 {
  V Rdif, Tdif, Sup, Sdn;
};

// max-by-magnitude guard of sw_two_stream's 1 - (k mu0)^2 denominator, element by element
__device__ __forceinline__ float ck_eps_guard(float v, float eps) { return (fabsf(v) >= eps) ? v : eps; }
__device__ __forceinline__ f2 ck_eps_guard(f2 v, float eps) { return (f2){ck_eps_guard(v.x, eps), ck_eps_guard(v.y, eps)}; }

// sw_two_stream (kernels_rte.hip) term by term for the K layers of a chunk, with the direct-beam transmittances
// Tnoscat = exp(-tau/mu0) given, stage by stage so that the K layers' exps share one batch of table reads
// kEmk: 0 forms exp(-tau k); 1 forms it and hands it out in emk_io; 2 takes it from emk_io (the value mode 1 handed
// out for the same layer, same bits)
template <bool kG0, int K, class V, int kEmk = 0>
__device__ __forceinline__ void ck_two_stream_k(const V (&tau)[K], const V (&w0)[K], const V (&g)[K], float mu0,
                                                const V (&Tnoscat)[K], const V (&dir_inc)[K], Coef2<V> (&c)[K],
                                                const uint64_t *etab, V (&emk_io)[K])
{
  const float eps = FLT_EPSILON, k_min = 1.e-4f;
  V gamma1[K], gamma2[K], k[K], arg[K], emk[K];
#pragma unroll
  for (int p = 0; p < K; p++) {
    if constexpr (kG0) {
      // g = 0: one rounding of the value the reference rounds at 4x and scales back exactly -- the same bits for
      // every |ssa| < 6.8e37 (tools/check_sw_identities.py walks all of those floats), two operations fewer
      gamma1[p] = 2.0f - w0[p] * 1.25f;
      gamma2[p] = w0[p] * .75f;
    } else {
      gamma1[p] = (8.0f - w0[p] * (5.0f + 3.0f * g[p])) * .25f;
      gamma2[p] = 3.0f * (w0[p] * (1.0f - g[p])) * .25f;
    }
    k[p] = sqrt2(vmax((gamma1[p] - gamma2[p]) * (gamma1[p] + gamma2[p]), (V)k_min));
    arg[p] = -tau[p] * k[p];
  }
  if constexpr (kEmk == 2) {
#pragma unroll
    for (int p = 0; p < K; p++) emk[p] = emk_io[p];
  } else {
    exp_neg_batch(arg, emk, etab);
    if constexpr (kEmk == 1) {
#pragma unroll
      for (int p = 0; p < K; p++) emk_io[p] = emk[p];
    }
  }
#pragma unroll
  for (int p = 0; p < K; p++) {
    const V em2k = emk[p] * emk[p];
    const V RTd = rcp2(k[p] * (1.0f + em2k) + gamma1[p] * (1.0f - em2k));
    c[p].Rdif = RTd * gamma2[p] * (1.0f - em2k);
    c[p].Tdif = RTd * 2.0f * k[p] * emk[p];
    const V gamma3 = kG0 ? (V)0.5f : (2.0f - 3.0f * mu0 * g[p]) * .25f;
    const V gamma4 = 1.0f - gamma3;
    // g = 0 (gamma3 = gamma4 = 1/2): alpha1 = alpha2 = (gamma1 + gamma2) / 2, the sum k's radicand already formed
    // (same bits, tools/check_sw_identities.py)
    const V alpha1 = kG0 ? (gamma1[p] + gamma2[p]) * .5f : gamma1[p] * gamma4 + gamma2[p] * gamma3;
    const V alpha2 = kG0 ? alpha1 : gamma1[p] * gamma3 + gamma2[p] * gamma4;
    const V k2e = 2.0f * k[p] * emk[p];
    const V k_mu = k[p] * mu0, k_mu2 = k_mu * k_mu, k_g3 = k[p] * gamma3, k_g4 = k[p] * gamma4;
    const V dd = ck_eps_guard(1.0f - k_mu2, eps);
    const V RT = div2(w0[p] * RTd, dd);
    const V Tn = Tnoscat[p];
    V Rdir = RT * ((1.0f - k_mu) * (alpha2 + k_g3) - (1.0f + k_mu) * (alpha2 - k_g3) * em2k -
                   k2e * (gamma3 - alpha2 * mu0) * Tn);
    V Tdir = RT * (k2e * (gamma4 + alpha1 * mu0) -
                   Tn * ((1.0f + k_mu) * (alpha1 + k_g4) - (1.0f - k_mu) * (alpha1 - k_g4) * em2k));
    Rdir = vmax((V)0.0f, vmin(Rdir, (1.0f - Tn)));
    Tdir = vmax((V)0.0f, vmin(Tdir, (1.0f - Tn - Rdir)));
    c[p].Sup = Rdir * dir_inc[p];
    c[p].Sdn = Tdir * dir_inc[p];
  }
}

// inc_2stream_by_2stream_bybnd (rte/kernels/mo_optical_props_kernels.F90:430-463) for a lane's g-points, as inc_2str2
template <class V>
__device__ __forceinline__ void ck_inc(V &t1, V &w1, V &g1, V t2, V w2, V g2)
{
  const float eps = 3.0f * FLT_MIN;
  const V tau12 = t1 + t2;
  const V tauscat12 = t1 * w1 + t2 * w2;
  g1 = (t1 * w1 * g1 + t2 * w2 * g2) / vmax((V)eps, tauscat12);
  w1 = tauscat12 / vmax((V)eps, tau12);
  t1 = tau12;
}

// the flush walks the ordered sums one lane per partial (ring_flush_sw_lanes) when the block has the lanes for it
// (C3 flush 18 us from 31 us with one lane per column); flux-ring rows are padded by 4 floats, so the lanes of one
// partial read different banks
constexpr bool kCkFlushLanes = true;
__host__ __device__ constexpr int ck_ring_stride(int ngpt) { return ngpt + 4; }

}  // namespace

// K: layers per chunk (checkpoint spacing); kCkRing: levels staged for the ordered broadband sums (a multiple of K).
// K = 3 layers per chunk under a 3-waves-per-SIMD register budget (132 VGPRs, no spill; at 4 waves K = 3 spilled and
// K = 2 fit): C3 step -3 %, C4 -1 % against K = 2 or the two-per-lane workspace kernel; K = 4 (148 VGPRs) was best
// alone at C3 but 13 % slower at C4, K = 6 spilled (tools/gpu_ab.sh, round 2).  Round 4 (the SW solver alone,
// alternating, bitwise; tools/kernel_ab.py): a ring of 9 levels (7 flushes per 60-layer column instead of 10) C4 -2.7 %;
// a 2-wave floor (no VGPR spill) +7 % with K = 3, +5 % with K = 4 / ring 8.
constexpr int kCkK = 3, kCkRing = 9, kCkWaves = 3;
// pass 1 loads kCkP1 chunks of optical depths per step (and the next step's while it computes)
constexpr int kCkP1 = 2;
// Waves per SIMD of the large-grid clear-sky NN instance (g = NULL, no increment; C5).  Round 2 chose 4 (128 VGPRs)
// when it also ran C3; since the small-grid instance took C3 over, the register floor spilled 19-21 VGPRs for no
// residency gain: at 3 (no spill) the C5 shard's SW solver runs 10 % faster alone, 12 % with the ring of 9 (round 4).
constexpr int kCkWavesNN = 3;
// Workspace planes of the large-grid instances (as the small-grid instance's kCkTnSmall / kCkEmkSmall): the clear-sky
// NN instance (C5) and the all-sky ones (C4).  Round 5 (tools/kernel_ab.py alone, tools/gpu_ab.sh whole steps;
// bitwise): the C5 shard's SW solver 32.68 -> 31.64 ms with both planes (the transmittances alone 32.24, exp(-k tau)
// alone 33.23: with both, pass 3 reads no tau), whole steps 66.63 -> 64.77 ms (2 alternating pairs); the large grid is
// then at HBM (199 GB per launch at 6.3 TB/s) where it was at its VALU floor (valu_busy 0.99, 3.35 TB/s).  C4 all sky:
// the transmittance plane 1.480 -> 1.458 ms alone (1.50 -> 1.435 in steps), steps within noise (-0.5 %); exp(-k tau)
// +1.3 %.  A/B knobs: tools/ablations.py swck_nnplanes / swck_incplanes.  The planes cost workspace (C5 shard: 15.7 ->
// 46.4 GB): when that allocation fails, launch_sw_2stream retries without them and these instances run without planes
// (the round-4 forms; same bits).
constexpr bool kCkTnNN = true, kCkEmkNN = true;
constexpr bool kCkTnInc = true, kCkEmkInc = false;

// kGpt: also store the g-point fluxes (ty_fluxes_flexible: up, total down, direct; (ngpt, nlay+1, ncol)) and sum the
// broadband down flux from the total as sw_solver_2stream does when it saves them (:572-588, :660-684)
// Small grids (the clear-sky instance when the grid fits in one round of resident waves, e.g. C3): 2 waves per SIMD
// as the register floor (more independent layers per wave where there are too few waves to hide the exps' latency);
// chunk length and ring below.  Whole-step A/B at C3 (one box, alternating): +1.3 %, SW solver -2.4 %; a ring of 4 was
// 3 % slower, K = 2 at 4 waves +0.5 %.  With many columns (C4, C5) K = 3 at 3-4 waves stays (K = 4 was 13 % slower).
// The small-grid instance also keeps pass 1's beam transmittances exp(-tau/mu0) in a workspace plane that passes 2 and
// 3 read instead of evaluating the exp again, and pass 2's exp(-tau k) in a second plane that pass 3 reads (C3: SW
// solver -3.7 %, step -3.7 %, alternating A/B on one box).  One g-point per lane (twice the waves to hide latency with;
// packed fp32 issues at the same cost per element as scalar fp32 on gfx950, tools/valu_rates.hip) measured slower than
// two.  (The transmittance plane in the all-sky instances measured slower in round 3; on the round-4 kernels it was
// faster at C4 and is on there since round 5: kCkTnInc above.)
// Round 4 (alone, alternating, bitwise; with the fence-free walk): K = 3 with a ring of 9 levels (three chunks per
// flush, 7 flushes per column instead of 8) -2.3 % against K = 4 / ring 8; K = 3 / ring 6 +3 %, K = 2 / ring 6 +5 %,
// K = 5 / ring 10 equal; a 3-wave floor equal.  A ring of 12 levels would not leave room for three blocks per CU.
constexpr int kCkKSmall = 3, kCkRingSmall = 9, kCkWavesSmall = 2;
constexpr bool kCkTnSmall = true, kCkEmkSmall = true;
using VSmall = f2;
// pass-1 chunks per load step of the small-grid instance (its pass 1 is latency-bound at C3: 10 dependent load steps
// of 6 layers per 60-layer column with the default)
constexpr int kCkP1Small = 2;
// passes 2 and 3 of the small-grid instance prefetch this many chunks ahead (three register buffers for 2): at C3
// each pass streams at 4.8-5.2 TB/s where the same 8-byte loads reach 6.3 TB/s at 3 waves per SIMD with 4 per lane in
// flight (tools/bw_width.hip), i.e. a chunk's loads are not always back when its body starts
constexpr int kCkAheadSmall = 1;

// V: f2 (two g-points per lane) or float (one per lane).  kBandPair (fused increment, two g-points per lane): every
// band starts at an even g-point, so both g-points of a lane lie in one band and its band values are one load each
// (the RRTMGP g-point sets: 16 per band).  Round 4, C4: SW solver -1.7 % alone, steps -0.8 % (3 alternating pairs)
template <bool kHasG, bool kInc, int K, bool kGpt = false, int R = kCkRing,
          int WAVES = (!kHasG && !kInc && !kGpt) ? kCkWavesNN : kCkWaves, bool kTn = false,
          class V = f2, bool kEmk = false, bool kBandPair = false, int P1C = kCkP1, int AHEAD = 1>
__global__ void __launch_bounds__(512, WAVES)
    sw_2stream_ck_kernel(int ngpt, int nlay, int ncol, int top_at_1, int ncb, const float *__restrict__ inc_flux,
                         const float *__restrict__ inc_dif, const float *__restrict__ tau,
                         const float *__restrict__ ssa, const float *__restrict__ gg, const float *__restrict__ mu0p,
                         const float *__restrict__ alb_dir, const float *__restrict__ alb_dif, BandArgs bands,
                         const float *__restrict__ tau_bnd, const float *__restrict__ ssa_bnd,
                         const float *__restrict__ g_bnd, float *__restrict__ ws, float *__restrict__ flux_up,
                         float *__restrict__ flux_dn, float *__restrict__ flux_dir, float *__restrict__ gpt_up,
                         float *__restrict__ gpt_dn, float *__restrict__ gpt_dir, SwBcDev bc)
{
  static_assert(R % K == 0, "the flux ring must hold whole chunks");
  constexpr bool kG0 = !kHasG && !kInc;  // g is the literal 0 (the NN path)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // `ncb` columns per block: lane t works on column c = t / (ngpt/NPL), g-points g .. g + NPL - 1
  constexpr int NPL = sizeof(V) / sizeof(float);
  using CA_ = ColArrV<V>;
  const int nlev = nlay + 1, lanes = ngpt / NPL, nck = (nlay + K - 1) / K;
  const int icol0 = blockIdx.x * ncb, nc = min(ncb, ncol - icol0);
  const int craw = (int)threadIdx.x / lanes;
  const bool on = craw < nc;
  const int c = on ? craw : nc - 1;
  const int g = NPL * ((int)threadIdx.x - craw * lanes);
  const int gc = on ? g : ngpt - NPL;
  const int icol = icol0 + c;
  // this column's ring [3][R][rs]: rows padded by 4 floats, so the flush threads' rows start in different LDS banks
  const int rs = ck_ring_stride(ngpt);
  float *ring = smem + kExpTabFloats + (size_t)c * 3 * R * rs;
  uint64_t *etab = (uint64_t *)(smem + kExpTabOff);
  load_exp_table(etab);
  // bc.tsi != NULL: the RFMIP driver's boundary conditions formed here (sw_boundary_kernel's expressions, same bits):
  // the solar source is staged in the ring's LDS, which pass 3 first writes after a barrier below
  const bool bcf = bc.tsi != nullptr;
  float *const bsrc = smem + kExpTabFloats;
  if (bcf)
    for (int i = threadIdx.x; i < ngpt; i += blockDim.x) bsrc[i] = bc.solar_source[i];
  // small-grid instance: the barrier comes after pass 1's first loads (kEarly below)
  constexpr bool kEarly = !kInc && WAVES == kCkWavesSmall;
  if constexpr (!kEarly) __syncthreads();
  const int dl_dn = top_at_1 ? 1 : -1;
  const uint32_t row = 4u * (uint32_t)ngpt;
  const uint32_t vL = 4u * (uint32_t)gc + (uint32_t)c * row * nlay;
  const size_t cl = (size_t)ngpt * nlay * icol0;
  const uint32_t bL = (uint32_t)nc * row * nlay;
  const CA_ Ttau(tau, cl, bL), Tssa(ssa, cl, bL), Tg(kHasG ? gg : tau, cl, bL);
  // checkpoints, column by column: (ngpt, 3 nck + 2, ncol) -- rows [0, nck) the beam, [nck, 2 nck + 1) the albedo,
  // [2 nck + 1, 3 nck + 2) the source; one buffer descriptor for the three (the layer offset in the SGPR offset)
  const int nrw = 3 * nck + 2;
  const size_t pW = (size_t)ngpt * nrw * ncol;
  const uint32_t vW = 4u * (uint32_t)gc + (uint32_t)c * row * nrw;
  const CA_ CW(ws, (size_t)ngpt * nrw * icol0, (uint32_t)nc * row * nrw);
  const uint32_t sA0 = row * (uint32_t)nck, sS0 = row * (uint32_t)(2 * nck + 1);
  // kTn: the beam transmittances (ngpt, nlay, ncol), addressed as tau.  kEmk: pass 2's exp(-tau k) in the plane after
  // it, which pass 3 reads instead of evaluating the exp again.  (Keeping all four coefficients R_dif, T_dif, S_up, S_dn
  // instead, so that pass 3 forms none, was 23 % slower at C3: four planes written and read cost more than they save.)
  const size_t plane = (size_t)ngpt * nlay * ncol;
  const CA_ CT(kTn ? ws + pW : ws, kTn ? cl : 0, kTn ? bL : 0u);
  const CA_ CE(kEmk ? ws + pW + (kTn ? plane : 0) : ws, kEmk ? cl : 0, kEmk ? bL : 0u);
  const uint32_t vWs = on ? vW : kBufOOB;
  // band-resolved increments: one band offset per g-point of the lane
  const size_t cb = (size_t)bands.nbnd * nlay * icol0;
  const uint32_t brow = 4u * (uint32_t)bands.nbnd, vbc = (uint32_t)c * brow * nlay;
  const uint32_t vb0 = kInc ? 4u * (uint32_t)band_of(bands, gc) + vbc : 0u,
                 vb1 = kInc ? 4u * (uint32_t)band_of(bands, gc + NPL - 1) + vbc : 0u;
  const uint32_t bB = kInc ? (uint32_t)nc * brow * nlay : 0u;
  const CA_ Bt(kInc ? tau_bnd : tau, kInc ? cb : 0, bB), Bw(kInc ? ssa_bnd : tau, kInc ? cb : 0, bB),
      Bg(kInc ? g_bnd : tau, kInc ? cb : 0, bB);
  auto ld_bnd = [&](const CA_ &a, int l) -> V {
    if constexpr (!kInc) return (V)0.0f;
    else if constexpr (NPL == 2 && kBandPair) {
      const float v = a.ld1(vb0, brow * (uint32_t)l);
      return (f2){v, v};
    } else if constexpr (NPL == 2) return (f2){a.ld1(vb0, brow * (uint32_t)l), a.ld1(vb1, brow * (uint32_t)l)};
    else return a.ld1(vb0, brow * (uint32_t)l);
  };
  // mu0 = merge(cos(sza * deg_to_rad), 1, usecol) (rrtmgp_rfmip_sw.F90:236-238, 421-427) or the caller's
  const float sza = bcf ? bc.sza[icol] : 0.0f;
  const float mu0 = bcf ? (sza < bc.sza_max ? ref_cosf(sza * bc.deg_to_rad) : 1.0f) : mu0p[icol];
  const float mu0_inv = 1.0f / mu0;
  // j counts layers from the top (clamped to the last layer); the result is the array layer
  auto lay = [&](int j) { return top_at_1 ? min(j, nlay - 1) : nlay - 1 - min(j, nlay - 1); };
  auto ld_col = [&](const float *p) -> V { return on ? *(const V *)(p + gc + (size_t)ngpt * icol) : (V)0.0f; };
  const int top = top_at_1 ? 0 : nlay;
  // the surface albedo, spectrally constant (rrtmgp_rfmip_sw.F90:428-433), or the caller's per g-point
  const V alb_bc = on && bcf ? (V)bc.sfc_alb[icol] : (V)0.0f;
  // Pass 1 reads P1 = kCkP1 * K layers per step (little arithmetic per layer: it needs many loads in flight).  In the
  // small-grid instance (one round of blocks: every block's prologue is on the kernel's path) its first step's loads go
  // out here, ahead of the prologue's barrier, which would hold them back until the exp table and the solar source are
  // in LDS.  Round 6, C3: the solver alone -1.3 %; in the large clear-sky instance C5 steps +0.3 % (2 pairs), so not
  // there (profiles/r06/swearly_*.txt)
  constexpr int P1 = P1C * K;
  struct Buf1 {
    V t[P1];
  } A1, B1;
  auto load1 = [&](Buf1 &b, int c1) {
#pragma unroll
    for (int p = 0; p < P1; p++) {
      const int l = lay(c1 * P1 + p);
      b.t[p] = Ttau.ldv(vL, row * (uint32_t)l);
      if constexpr (kInc) b.t[p] += ld_bnd(Bt, l);
    }
  };
  if constexpr (kEarly) {
    load1(A1, 0);
    __syncthreads();
  }
  // the incident flux toa = toa_src * tsi / def_tsi (rrtmgp_rfmip_sw.F90:403-418), def_tsi the source summed in g order
  // by every lane (broadcast LDS reads; no barrier); or the caller's
  auto bc_toa = [&]() -> V {
    float s = 0.0f;
    int i = 0;
    for (; i + 8 <= ngpt; i += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = bsrc[i + j];
#pragma unroll
      for (int j = 0; j < 8; j++) s = s + v[j];
    }
    for (; i < ngpt; i++) s = s + bsrc[i];
    const float t = bc.tsi[icol];
    if constexpr (NPL == 2) return on ? (V){bsrc[gc] * t / s, bsrc[gc + 1] * t / s} : (V)0.0f;
    else return on ? (V)(bsrc[gc] * t / s) : (V)0.0f;
  };
  const V Ftop = (bcf ? bc_toa() : ld_col(inc_flux)) * mu0;

  // one chunk's optical properties (the band increment is formed as they are used, as inc_2str2 does), with the
  // checkpoints the pass reads for it: fb the beam at the chunk's top (pass 2), ae / se the albedo and source at its
  // bottom (pass 3)
  struct Chunk {
    V t[K], w[K], g[K], qt[K], qw[K], qg[K], tn[K], em[K], fb, ae, se;
  };
  // pass: 2 or 3
  auto load_chunk = [&](Chunk &ch, int ck, int pass) {
#pragma unroll
    for (int p = 0; p < K; p++) {
      const int l = lay(ck * K + p);
      const uint32_t s = row * (uint32_t)l;
      ch.t[p] = Ttau.ldv(vL, s);
      ch.tn[p] = kTn ? CT.ldv(vL, s) : (V)0.0f;
      ch.em[p] = (kEmk && pass == 3) ? CE.ldv(vL, s) : (V)0.0f;
      ch.w[p] = Tssa.ldv(vL, s);
      ch.g[p] = kHasG ? Tg.ldv(vL, s) : (V)0.0f;
      if constexpr (kInc) {
        ch.qt[p] = ld_bnd(Bt, l);
        ch.qw[p] = ld_bnd(Bw, l);
        ch.qg[p] = ld_bnd(Bg, l);
      } else {
        ch.qt[p] = ch.qw[p] = ch.qg[p] = (V)0.0f;
      }
    }
    if (pass == 2) {
      ch.fb = CW.ldv(vW, row * (uint32_t)ck);
    } else {
      const uint32_t sE = row * (uint32_t)min(ck + 1, nck);
      ch.ae = CW.ldv(vW, sA0 + sE);
      ch.se = CW.ldv(vW, sS0 + sE);
    }
  };
  // the (incremented) properties of layer p of a chunk
  auto props = [&](const Chunk &ch, int p, V &t, V &w, V &g0) {
    t = ch.t[p];
    w = ch.w[p];
    g0 = kHasG ? ch.g[p] : (V)0.0f;
    if constexpr (kInc) ck_inc(t, w, g0, ch.qt[p], ch.qw[p], ch.qg[p]);
  };
  // Each pass walks its chunks two at a time through two register buffers: the loads of the next chunk go to the other
  // buffer while this one is computed, so no copy waits for them at the end of the step.  body(buf, ck, valid)
  // computes chunk ck; idx(i) is the pass's i-th chunk.  With an odd count the last step's second body runs on the
  // last chunk again with valid = false (no state change, no stores), so that no branch separates a prefetch from its
  // use (the compiler sinks loads past such a branch).  No scheduling fences between the loads and the bodies: the
  // scheduler may then start a chunk's independent coefficient algebra under the previous chunk's recurrence (round
  // 4: C3 SW solver -0.6 to -2.5 %, C4 -1.1 %, tools/kernel_ab.py).
  auto walk = [&](auto &&load, auto &&body, int count, auto &&idx, auto &A, auto &B, bool preloaded = false) {
    if (!preloaded) load(A, idx(0));
    for (int i = 0; i < count; i += 2) {
      load(B, idx(min(i + 1, count - 1)));
      body(A, idx(i), true);
      load(A, idx(min(i + 2, count - 1)));
      body(B, idx(min(i + 1, count - 1)), i + 1 < count);
    }
  };
  // the same walk two chunks ahead through three buffers (same bodies in the same order: same bits)
  auto walk3 = [&](auto &&load, auto &&body, int count, auto &&idx, auto &A, auto &B, auto &C) {
    load(A, idx(0));
    load(B, idx(min(1, count - 1)));
    for (int i = 0; i < count; i += 3) {
      load(C, idx(min(i + 2, count - 1)));
      body(A, idx(i), true);
      load(A, idx(min(i + 3, count - 1)));
      body(B, idx(min(i + 1, count - 1)), i + 1 < count);
      load(B, idx(min(i + 4, count - 1)));
      body(C, idx(min(i + 2, count - 1)), i + 2 < count);
    }
  };

  // ---- pass 1: direct beam, checkpoint at every chunk top (steps of P1 layers, A1 / B1 / load1 above) ----
  V Fd = Ftop;
  {
    const int np1 = (nlay + P1 - 1) / P1;
    auto body1 = [&](Buf1 &b, int c1, bool valid) {
      const int n = valid ? min(P1, nlay - c1 * P1) : 0;
      V arg[P1], Tn[P1];
#pragma unroll
      for (int p = 0; p < P1; p++) arg[p] = -b.t[p] * mu0_inv;
      exp_beam_batch(arg, Tn, etab);
      if constexpr (kTn) {
#pragma unroll
        for (int p = 0; p < P1; p++) CT.stv(Tn[p], (on && p < n) ? vL : kBufOOB, row * (uint32_t)lay(c1 * P1 + p));
      }
#pragma unroll
      for (int p = 0; p < P1; p++) {
        if (p % K == 0) CW.stv(Fd, (p < n) ? vWs : kBufOOB, row * (uint32_t)(c1 * P1C + p / K));
        Fd = (p < n) ? Tn[p] * Fd : Fd;
      }
    };
    walk(load1, body1, np1, [](int i) { return i; }, A1, B1, kEarly);
  }
  // ---- pass 2: bottom -> top adding; albedo / source checkpoint at every chunk top and at the surface ----
  V alb_b = bcf ? alb_bc : ld_col(alb_dif);
  V src_b = Fd * (bcf ? alb_bc : ld_col(alb_dir));
  CW.stv(alb_b, vWs, sA0 + row * (uint32_t)nck);
  CW.stv(src_b, vWs, sS0 + row * (uint32_t)nck);
  {
    Chunk A, B;
    auto load2 = [&](Chunk &ch, int ck) { load_chunk(ch, ck, 2); };
    auto body2 = [&](Chunk &cur, int ck, bool valid) {
      const int n = valid ? min(K, nlay - ck * K) : 0;
      V t[K], w[K], g0[K], Tn[K], Fin[K];
      V Fb = cur.fb;
#pragma unroll
      for (int p = 0; p < K; p++) props(cur, p, t[p], w[p], g0[p]);
      if constexpr (kTn) {
#pragma unroll
        for (int p = 0; p < K; p++) Tn[p] = cur.tn[p];  // pass 1's transmittances
      } else {
        V arg[K];
#pragma unroll
        for (int p = 0; p < K; p++) arg[p] = -t[p] * mu0_inv;
        exp_beam_batch(arg, Tn, etab);  // pass 1's expressions, same bits
      }
#pragma unroll
      for (int p = 0; p < K; p++) {
        Fin[p] = Fb;  // the beam at the layer's top
        Fb = Tn[p] * Fb;
      }
      // the chunk's coefficients (layers past nlay in the last chunk see the clamped last layer and are not used),
      // then the adding recurrence
      Coef2<V> cf[K];
      V em[K];
      ck_two_stream_k<kG0, K, V, kEmk ? 1 : 0>(t, w, g0, mu0, Tn, Fin, cf, etab, em);
      if constexpr (kEmk) {
#pragma unroll
        for (int p = 0; p < K; p++) CE.stv(em[p], (on && p < n) ? vL : kBufOOB, row * (uint32_t)lay(ck * K + p));
      }
#pragma unroll
      for (int p = K - 1; p >= 0; p--) {
        const V denom = rcp2(1.0f - cf[p].Rdif * alb_b);
        const V alb = cf[p].Rdif + cf[p].Tdif * cf[p].Tdif * alb_b * denom;
        const V src = cf[p].Sup + cf[p].Tdif * denom * (src_b + alb_b * cf[p].Sdn);
        alb_b = (p < n) ? alb : alb_b;
        src_b = (p < n) ? src : src_b;
      }
      CW.stv(alb_b, valid && ck > 0 ? vWs : kBufOOB, sA0 + row * (uint32_t)ck);
      CW.stv(src_b, valid && ck > 0 ? vWs : kBufOOB, sS0 + row * (uint32_t)ck);
    };
    if constexpr (AHEAD == 2) {
      Chunk C;
      walk3(load2, body2, nck, [&](int i) { return nck - 1 - i; }, A, B, C);
    } else {
      walk(load2, body2, nck, [&](int i) { return nck - 1 - i; }, A, B);
    }
  }
  // ---- pass 3: top -> bottom fluxes + ordered broadband sums ----
  // idle lanes (past the block's columns) store their ring values to one spare slot instead of branching around the
  // stores; slots past the last level (the last chunk's padding layers) are written and never read
  float *const spare = smem + kExpTabFloats + (size_t)ncb * 3 * R * rs;
  // level `lev` (array index) of the g-point outputs
  auto put = [&](V up, V dif, V dir, int r, int lev, bool valid) {
    const V dn = kGpt ? dif + dir : dif;  // kGpt: the total, rounded once ("flux_dn is total", :665-666)
    *(V *)(on ? &ring[(size_t)r * rs + g] : spare) = up;
    *(V *)(on ? &ring[((size_t)R + r) * rs + g] : spare) = dn;
    *(V *)(on ? &ring[((size_t)2 * R + r) * rs + g] : spare) = dir;
    if constexpr (kGpt) {
      if (on && valid) {
        const size_t o = (size_t)g + (size_t)ngpt * ((size_t)lev + (size_t)nlev * icol);
        *(V *)&gpt_up[o] = up;
        *(V *)&gpt_dn[o] = dn;
        *(V *)&gpt_dir[o] = dir;
      }
    }
  };
  auto flush = [&](int n, int lev0, int dl, int slot0 = 0) {
    if (kCkFlushLanes && (ngpt & 3) == 0 && 3 * ncb * n * 4 <= (int)blockDim.x)
      ring_flush_sw_lanes<R, kGpt>(smem + kExpTabFloats, ncb, n, lev0, dl, ngpt, nlev, icol0, ncol, flux_up, flux_dn,
                                   flux_dir, rs, slot0);
    else
      ring_flush_sw<R, kGpt>(smem + kExpTabFloats, ncb, n, lev0, dl, ngpt, nlev, icol0, ncol, flux_up, flux_dn,
                             flux_dir, rs, slot0);
  };
  // the ring holds M = R / K chunks; the block flushes it when it is full (a barrier, the ordered sums, a barrier).
  // (Staggering the blocks' flush phases, so that blocks sharing a CU flush at different chunks, measured equal, round
  // 4: the flush's cost is its own latency inside each block, not the whole chip flushing at once.)
  constexpr int M = R / K;
  V Fdn = inc_dif ? ld_col(inc_dif) : (V)0.0f;
  if (bcf) __syncthreads();  // every lane has read the staged solar source before the ring is written
  put(Fdn * alb_b + src_b, Fdn, Ftop, 0, top, true);
  flush(1, top, 1);
  {
    Chunk A, B;
    V Fd3 = Ftop;
    auto load3 = [&](Chunk &ch, int ck) { load_chunk(ch, ck, 3); };
    auto body3 = [&](Chunk &cur, int ck, bool valid) {
      const int n = valid ? min(K, nlay - ck * K) : 0;
      // the chunk's coefficients, top down, the beam carried as pass 1 carries it
      V t[K], w[K], g0[K], Tn[K], Fin[K], Fdir[K];
#pragma unroll
      for (int p = 0; p < K; p++) props(cur, p, t[p], w[p], g0[p]);
      if constexpr (kTn) {
#pragma unroll
        for (int p = 0; p < K; p++) Tn[p] = cur.tn[p];
      } else {
        V arg[K];
#pragma unroll
        for (int p = 0; p < K; p++) arg[p] = -t[p] * mu0_inv;
        exp_beam_batch(arg, Tn, etab);
      }
#pragma unroll
      for (int p = 0; p < K; p++) {
        Fin[p] = Fd3;
        Fd3 = (p < n) ? Tn[p] * Fd3 : Fd3;
        Fdir[p] = Fd3;  // the beam at the layer's bottom
      }
      Coef2<V> cf[K];
      ck_two_stream_k<kG0, K, V, kEmk ? 2 : 0>(t, w, g0, mu0, Tn, Fin, cf, etab, cur.em);
      // albedo / source at levels ck*K + p + 1 (A[p], S[p]), walked up from the checkpoint with pass 2's expressions;
      // D[p] = 1 / (1 - R_dif(p) * A[p]) is the adding denominator both walks use
      V Al[K], S[K], D[K];
      {
        V a = cur.ae, s = cur.se;
#pragma unroll
        for (int p = K - 1; p >= 0; p--) {
          Al[p] = a;
          S[p] = s;
          const V denom = rcp2(1.0f - cf[p].Rdif * a);
          D[p] = denom;
          if (p > 0) {
            const V an = cf[p].Rdif + cf[p].Tdif * cf[p].Tdif * a * denom;
            const V sn = cf[p].Sup + cf[p].Tdif * denom * (s + a * cf[p].Sdn);
            a = (p < n) ? an : a;
            s = (p < n) ? sn : s;
          }
        }
      }
      // fluxes down the chunk (adding :1583-1591, Eqs 12-13)
      const int rbase = (ck % M) * K;
#pragma unroll
      for (int p = 0; p < K; p++) {
        const V fdn = (cf[p].Tdif * Fdn + cf[p].Rdif * S[p] + cf[p].Sdn) * D[p];
        Fdn = (p < n) ? fdn : Fdn;
        put(fdn * Al[p] + S[p], fdn, Fdir[p], rbase + p, top + dl_dn * (ck * K + p + 1), p < n);
      }
      if (valid && (rbase + K == R || ck == nck - 1)) {
        const int j0 = ck * K - rbase;  // first layer of this ring's levels
        flush(min(R, nlay - j0), top + dl_dn * (j0 + 1), dl_dn);
      }
    };
    if constexpr (AHEAD == 2) {
      Chunk C;
      walk3(load3, body3, nck, [](int i) { return i; }, A, B, C);
    } else {
      walk(load3, body3, nck, [](int i) { return i; }, A, B);
    }
  }
}

bool sw_ck_small(const rrtmgpnn_context *ctx, int ngpt, int ncol, bool has_g, bool inc, bool gpt)
{
  // 2 g-points per lane; one round of 16 waves of 64 lanes per CU
  return !has_g && !inc && !gpt && (long long)ncol * (ngpt / 2) <= 64LL * 16 * ctx->num_cus;
}

// workspace floats of the checkpointed kernel (sized for the smaller of the chunk lengths, so it holds either
// instance) plus the planes of the instance that runs: small-grid clear sky, large-grid clear sky (NN: g = NULL, no
// increment, no g-point outputs) or all sky (inc)
size_t sw_2stream_ck_ws_floats(int ngpt, int nlay, int ncol, bool small, bool inc, bool nn, bool planes)
{
  const int np = small  ? (int)kCkTnSmall + (int)kCkEmkSmall
                 : !planes ? 0
                 : nn     ? (int)kCkTnNN + (int)kCkEmkNN
                 : inc    ? (int)kCkTnInc + (int)kCkEmkInc
                          : 0;
  const size_t tn = (size_t)np * ngpt * nlay * ncol;
  const int k = std::min(kCkK, kCkKSmall);
  const size_t nck = (size_t)(nlay + k - 1) / k;
  return (size_t)ngpt * ncol * (nck + 2 * (nck + 1)) + tn;
}

// ngpt even and <= 256
int launch_sw_2stream_ck(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                         const float *inc_flux_dif, const float *tau, const float *ssa, const float *g,
                         const float *mu0, const float *alb_dir, const float *alb_dif, const BandArgs *bands,
                         const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, void *ws, float *flux_up,
                         float *flux_dn, float *flux_dir, bool planes, const SwBcDev *bc)
{
  const int ncb2 = 2 * (ngpt / 2) <= 512 ? 2 : 1;  // two columns per block where 512 lanes hold them
  const BandArgs nob{};
  const BandArgs &b = bands ? *bands : nob;
  const SwBcDev nobc{};  // tsi == NULL: the caller's inc_flux, mu0 and albedos
  const SwBcDev &bcd = bc ? *bc : nobc;
  const auto &ex = ctx->extras;
  // npl g-points per lane, ncb columns per block
  auto go = [&](auto kern, const float *tb, const float *sb, const float *gb, int ring = kCkRing, int npl = 2) -> int {
    const int ncb = npl == 2 ? ncb2 : columns_per_block(ngpt);
    if (ncb > kFlushLanesMaxCols)  // the flush's lane -> column map (ring_flush_sw_lanes) covers at most 4 columns
      return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: more columns per block than the ordered flush maps");
    const int threads = (ncb * (ngpt / npl) + 63) / 64 * 64;
    const dim3 grid((ncol + ncb - 1) / ncb), block(threads);
    const size_t lds = sizeof(float) * (kExpTabFloats + (size_t)ncb * 3 * ring * ck_ring_stride(ngpt) + 4);  // + spare
    if (lds > 160 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw solver: LDS ring exceeds 160 KiB");
    if (lds > 64 * 1024)
      if (int rc = raise_lds_limit((const void *)kern)) return rc;
    hipLaunchKernelGGL(kern, grid, block, lds, ctx->stream, ngpt, nlay, ncol, top_at_1, ncb, inc_flux, inc_flux_dif,
                       tau, ssa, g, mu0, alb_dir, alb_dif, b, tb, sb, gb, (float *)ws, flux_up, flux_dn, flux_dir,
                       ex.gpt_up, ex.gpt_dn, ex.gpt_dir, bcd);
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
  if (bands) {
    bool pair = true;  // every band starts at an even (0-based) g-point
    for (int i = 0; i < b.nbnd; i++) pair = pair && ((b.lims[2 * i] - 1) % 2 == 0);
    constexpr int W = kCkWaves;
    constexpr bool T = kCkTnInc, E = kCkEmkInc;
    if (!planes) {  // the workspace planes did not fit (launch_sw_2stream's fallback): the same bits, recomputed
      if (pair && g)
        return go(sw_2stream_ck_kernel<true, true, kCkK, false, kCkRing, W, false, f2, false, true>, tau_bnd, ssa_bnd,
                  g_bnd);
      if (pair)
        return go(sw_2stream_ck_kernel<false, true, kCkK, false, kCkRing, W, false, f2, false, true>, tau_bnd, ssa_bnd,
                  g_bnd);
      if (g) return go(sw_2stream_ck_kernel<true, true, kCkK, false, kCkRing, W>, tau_bnd, ssa_bnd, g_bnd);
      return go(sw_2stream_ck_kernel<false, true, kCkK, false, kCkRing, W>, tau_bnd, ssa_bnd, g_bnd);
    }
    if (pair && g)
      return go(sw_2stream_ck_kernel<true, true, kCkK, false, kCkRing, W, T, f2, E, true>, tau_bnd, ssa_bnd, g_bnd);
    if (pair)
      return go(sw_2stream_ck_kernel<false, true, kCkK, false, kCkRing, W, T, f2, E, true>, tau_bnd, ssa_bnd, g_bnd);
    if (g) return go(sw_2stream_ck_kernel<true, true, kCkK, false, kCkRing, W, T, f2, E>, tau_bnd, ssa_bnd, g_bnd);
    return go(sw_2stream_ck_kernel<false, true, kCkK, false, kCkRing, W, T, f2, E>, tau_bnd, ssa_bnd, g_bnd);
  }
  if (g) return go(sw_2stream_ck_kernel<true, false, kCkK>, nullptr, nullptr, nullptr);
  // the small-grid instance when the clear-sky grid fits in one round of resident waves (2 g-points per lane, 16
  // waves per CU)
  if (sw_ck_small(ctx, ngpt, ncol, false, false, false))
    return go(sw_2stream_ck_kernel<false, false, kCkKSmall, false, kCkRingSmall, kCkWavesSmall, kCkTnSmall, VSmall,
                                   kCkEmkSmall, false, kCkP1Small, kCkAheadSmall>,
              nullptr, nullptr, nullptr, kCkRingSmall, (int)(sizeof(VSmall) / sizeof(float)));
  if (!planes) return go(sw_2stream_ck_kernel<false, false, kCkK, false, kCkRing, kCkWavesNN>, nullptr, nullptr, nullptr);
  return go(sw_2stream_ck_kernel<false, false, kCkK, false, kCkRing, kCkWavesNN, kCkTnNN, f2, kCkEmkNN>, nullptr,
            nullptr, nullptr);
}

}  // namespace rrtmgpnn
