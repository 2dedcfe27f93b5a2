// kernels_nn.hip -- NN gas-optics kernels for gfx950 (MI355X).
//
//  * nn_inputs_kernel : compute_nn_inputs (rrtmgp/mo_gas_optics_rrtmgp.F90:618-798)
//  * col_dry_kernel   : get_col_dry       (rrtmgp/mo_gas_optics_rrtmgp.F90:1662-1707)
//  * tlev_kernel      : level temperatures (rrtmgp/mo_gas_optics_rrtmgp.F90:317-337)
//  * mlp_pair_kernel  : the whole 3-layer MLP (softsign, softsign, linear) of ONE OR TWO networks
//    that share the same inputs, fused with their post-processing:
//       LW pair : tau = (std*(y+b)+mean)^8 * col_dry  and  pfrac = (y+b)^2
//                 (neural/mod_network_rrtmgp.F90:125-317, predict_nn_lw_blas_sp
//                  rrtmgp/kernels/mo_gas_optics_kernels.F90:690-774)
//       SW pair : tau_abs, tau_ray -> tau = tau_abs + tau_ray, ssa = tau_ray/tau, g = 0
//                 (:869-953 with INLINE_COMBINE, mod_network_rrtmgp.F90:224-229,
//                  mo_gas_optics_rrtmgp.F90:560-567)
//       LW both : one model with 2*ngpt outputs (output_sgemm_lw + :744-772)
//    The reference runs this as three SGEMMs per model with activations materialised in
//    (neurons x nlay*ncol) HBM arrays; here each wave keeps its 16 samples' activations in
//    MFMA accumulators and chains layers register-to-register.
//
// MFMA mapping (v_mfma_f32_16x16x4_f32, exact f32, fmaf-chain numerics):
//   lane l: j = l & 15, q = l >> 4.  A operand A[i=j][k=q], B operand B[k=q][n=j],
//   accumulator register r holds D[row = 4q + r][col = j].
//   Hidden layers compute H^T (units x samples):  A = packed W^T, B = activations.
//   The output layer computes Y (samples x g-points): A = H2 taken straight from the hidden
//   accumulators (sample on the lane, units in registers), B = packed W3.
//   Hidden units are stored PERMUTED in the accumulators: physical row R = 4q + r of tile m
//   holds logical unit u = 16m + 4r + q.  With that permutation, K-step (m, t) of the next
//   layer feeds unit 16m + 4t + q from lane group q, i.e. every dot product is accumulated in
//   ascending k order -- bit-identical to a sequential fmaf chain (the oracle's order).
#include "nn_device.hpp"

#include <algorithm>
#include <cmath>

namespace rrtmgpnn {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// compute_nn_inputs + col_dry are elementwise over (lay, col).
// ------------------------------------------------------------------------------------------
// One thread per (lay, col) sample.  The gas loop is unrolled over kMaxInputs so every gas pointer and
// scaling constant stays a kernel-argument SGPR (a runtime index would put them in scratch), and the
// block's (nx x 256) outputs are staged in LDS so the store to `out` is one contiguous stream.
constexpr int kInThreads = 256;

__global__ void __launch_bounds__(kInThreads) nn_inputs_kernel(int ncol, int nlay, int nx,
                                                               const float *__restrict__ play,
                                                               const float *__restrict__ tlay, GasArgs gas,
                                                               NnInArgs sc, float *__restrict__ out)
{
  __shared__ float st[kInThreads * kMaxInputs];
  const long long N = (long long)ncol * nlay;
  const long long s0 = (long long)blockIdx.x * kInThreads;
  const long long s = s0 + threadIdx.x;
  const int ns = (int)min((long long)kInThreads, N - s0);
  if (s < N) {
    const int ilay = (int)(s % nlay);
    float *o = st + nx * threadIdx.x;
    o[0] = (tlay[s] - sc.mn[0]) / (sc.mx[0] - sc.mn[0]);
    o[1] = (ref_logf(play[s]) - sc.mn[1]) / (sc.mx[1] - sc.mn[1]);
    o[2] = (sqrtf(sqrtf(gas.p[2][s])) - sc.mn[2]) / (sc.mx[2] - sc.mn[2]);
    o[3] = (sqrtf(sqrtf(gas.p[3][s])) - sc.mn[3]) / (sc.mx[3] - sc.mn[3]);
#pragma unroll
    for (int k = 4; k < kMaxInputs; k++) {
      if (k < nx) {
        float c;
        const float *p = gas.p[k];
        if (!p) c = 0.0f;
        else if (gas.nd[k] == 0) c = p[0];
        else if (gas.nd[k] == 1) c = p[ilay];
        else c = p[s];
        o[k] = (c - sc.mn[k]) / (sc.mx[k] - sc.mn[k]);
      }
    }
  }
  __syncthreads();
  float *dst = out + (size_t)nx * s0;
  for (int i = threadIdx.x; i < nx * ns; i += kInThreads) dst[i] = st[i];
}

__global__ void col_dry_kernel(int ncol, int nlay, const float *__restrict__ h2o, const float *__restrict__ plev,
                               float *__restrict__ col_dry)
{
  long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (long long)ncol * nlay) return;
  int icol = (int)(s / nlay), ilev = (int)(s % nlay);
  const float *pl = plev + (size_t)(nlay + 1) * icol;
  col_dry[s] = col_dry_of(h2o[s], pl[ilev], pl[ilev + 1]);
}

__global__ void tlev_kernel(int ncol, int nlay, const float *__restrict__ play, const float *__restrict__ plev,
                            const float *__restrict__ tlay, float *__restrict__ tlev)
{
  long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (long long)ncol * (nlay + 1)) return;
  int icol = (int)(s / (nlay + 1)), ilev = (int)(s % (nlay + 1));
  const float *pa = play + (size_t)nlay * icol, *pv = plev + (size_t)(nlay + 1) * icol;
  const float *ta = tlay + (size_t)nlay * icol;
  float r;
  if (ilev == 0)
    r = ta[0] + (pv[0] - pa[0]) * (ta[1] - ta[0]) / (pa[1] - pa[0]);
  else if (ilev == nlay)
    r = ta[nlay - 1] + (pv[nlay] - pa[nlay - 1]) * (ta[nlay - 1] - ta[nlay - 2]) / (pa[nlay - 1] - pa[nlay - 2]);
  else
    r = (pa[ilev - 1] * ta[ilev - 1] * (pv[ilev] - pa[ilev]) + pa[ilev] * ta[ilev] * (pa[ilev - 1] - pv[ilev])) /
        (pv[ilev] * (pa[ilev - 1] - pa[ilev]));
  tlev[s] = r;
}

int launch_nn_inputs(rrtmgpnn_context *ctx, int ncol, int nlay, int nx, const float *play, const float *tlay,
                     const GasArgs &gas, const float *in_min_max, float *out)
{
  NnInArgs sc;
  for (int k = 0; k < nx; k++) { sc.mn[k] = in_min_max[k]; sc.mx[k] = in_min_max[nx + k]; }
  long long N = (long long)ncol * nlay;
  if (N == 0) return RRTMGPNN_OK;
  if (nx < 4 || nx > kMaxInputs) return fail(RRTMGPNN_ERR_ARGUMENT, "nn_inputs: need 4..32 inputs");
  hipLaunchKernelGGL(nn_inputs_kernel, dim3((unsigned)((N + kInThreads - 1) / kInThreads)), dim3(kInThreads), 0,
                     ctx->stream, ncol, nlay, nx, play, tlay, gas, sc, out);
  RRTMGPNN_LAUNCH_CHECK("nn_inputs_kernel");
  return RRTMGPNN_OK;
}

int launch_col_dry(rrtmgpnn_context *ctx, int ncol, int nlay, const float *h2o, const float *plev, float *col_dry)
{
  long long N = (long long)ncol * nlay;
  if (N == 0) return RRTMGPNN_OK;
  hipLaunchKernelGGL(col_dry_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, ctx->stream, ncol, nlay, h2o,
                     plev, col_dry);
  RRTMGPNN_LAUNCH_CHECK("col_dry_kernel");
  return RRTMGPNN_OK;
}

int launch_tlev(rrtmgpnn_context *ctx, int ncol, int nlay, const float *play, const float *plev, const float *tlay,
                float *tlev)
{
  long long N = (long long)ncol * (nlay + 1);
  if (N == 0) return RRTMGPNN_OK;
  hipLaunchKernelGGL(tlev_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, ctx->stream, ncol, nlay, play,
                     plev, tlay, tlev);
  RRTMGPNN_LAUNCH_CHECK("tlev_kernel");
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// Activations: neural/mod_activation.F90 (bias added before, as bias_and_activation does).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float activate(int act, float x)
{
  switch (act) {
  case RRTMGPNN_ACT_SOFTSIGN: return x / (fabsf(x) + 1.0f);
  case RRTMGPNN_ACT_RELU: return fmaxf(0.0f, x);
  case RRTMGPNN_ACT_SIGMOID: return 1.0f / (1.0f + ref_expf(-x));
  case RRTMGPNN_ACT_HARD_SIGMOID: return fmaxf(0.0f, fminf(1.0f, 0.2f * x + 0.5f));
  case 5: return tanhf(x);
  case 6: return ref_expf(-x * x);
  default: return x;
  }
}

// Compile-time activation sets of the fused kernel: ACTS == 1 is the shipped models' softsign,
// softsign, linear (Appendix A of SURVEY.md), inlined straight-line; ACTS == 0 dispatches on the
// runtime codes (any other combination).
template <int ACTS>
__device__ __forceinline__ float act_hidden(int act, float x)
{
  if constexpr (ACTS == 1) return softsign(x);  // nn_device.hpp (mod_activation.F90:107-128)
  else return activate(act, x);
}
template <int ACTS>
__device__ __forceinline__ float act_out(int act, float x)
{
  if constexpr (ACTS == 1) return x;  // linear
  else return activate(act, x);
}

// ------------------------------------------------------------------------------------------
// Packed image layout (floats) of a 3-layer network [nx, h1, h2, ny]:
//   K1S = ceil(nx/4), H1T = ceil(h1/16), H2T = ceil(h2/16), NGT = ceil(ny/16)
//   L1 [H1T][K1S][64]        lane(i,q): W1[k=4t+q][u(i)]         u(i) = 16mo + 4(i&3) + (i>>2)
//   L2 [H2T][4*H1T][64]      lane(i,q): W2[k=16m+4t+q][u(i)]
//   L3 [NGT][4*H2T][64]      lane(i,q): W3[k=16m+4t+q][g=16go+i]   (the A operand: rows are g-points)
//   B1 [H1T*16], B2 [H2T*16] bias by PHYSICAL row R: b[16m + 4(R&3) + (R>>2)]
//   B3, STD, MEAN [NGT*16]   by g
// ------------------------------------------------------------------------------------------
struct ImgLayout {
  int l1, l2, l3, b1, b2, b3, sd, mn, total;
};
__host__ __device__ inline ImgLayout img_layout(int K1S, int H1T, int H2T, int NGT)
{
  ImgLayout L;
  L.l1 = 0;
  L.l2 = L.l1 + H1T * K1S * 64;
  L.l3 = L.l2 + H2T * H1T * 4 * 64;
  L.b1 = L.l3 + NGT * H2T * 4 * 64;
  L.b2 = L.b1 + H1T * 16;
  L.b3 = L.b2 + H2T * 16;
  L.sd = L.b3 + NGT * 16;
  L.mn = L.sd + NGT * 16;
  L.total = L.mn + NGT * 16;
  return L;
}

int pack_network(rrtmgpnn_network *net)
{
  if (net->nlayers != 3) return RRTMGPNN_OK;  // generic path only
  const int nx = net->dims[0], h1 = net->dims[1], h2 = net->dims[2], ny = net->dims[3];
  if (nx > kMaxInputs || h1 > 128 || h2 > 128) return RRTMGPNN_OK;
  const int K1S = (nx + 3) / 4, H1T = (h1 + 15) / 16, H2T = (h2 + 15) / 16, NGT = (ny + 15) / 16;
  ImgLayout L = img_layout(K1S, H1T, H2T, NGT);
  std::vector<float> img(L.total, 0.0f);
  const std::vector<float> &W1 = net->w[0], &W2 = net->w[1], &W3 = net->w[2];
  auto unit = [](int m, int i) { return 16 * m + 4 * (i & 3) + (i >> 2); };
  for (int mo = 0; mo < H1T; mo++)
    for (int t = 0; t < K1S; t++)
      for (int l = 0; l < 64; l++) {
        int i = l & 15, q = l >> 4, k = 4 * t + q, u = unit(mo, i);
        img[L.l1 + (mo * K1S + t) * 64 + l] = (k < nx && u < h1) ? W1[(size_t)k * h1 + u] : 0.0f;
      }
  for (int mo = 0; mo < H2T; mo++)
    for (int s = 0; s < 4 * H1T; s++)
      for (int l = 0; l < 64; l++) {
        int i = l & 15, q = l >> 4, m = s >> 2, t = s & 3, k = 16 * m + 4 * t + q, u = unit(mo, i);
        img[L.l2 + (mo * 4 * H1T + s) * 64 + l] = (k < h1 && u < h2) ? W2[(size_t)k * h2 + u] : 0.0f;
      }
  for (int go = 0; go < NGT; go++)
    for (int s = 0; s < 4 * H2T; s++)
      for (int l = 0; l < 64; l++) {
        int j = l & 15, q = l >> 4, m = s >> 2, t = s & 3, k = 16 * m + 4 * t + q, g = 16 * go + j;
        img[L.l3 + (go * 4 * H2T + s) * 64 + l] = (k < h2 && g < ny) ? W3[(size_t)k * ny + g] : 0.0f;
      }
  for (int m = 0; m < H1T; m++)
    for (int R = 0; R < 16; R++) {
      int u = unit(m, R);
      img[L.b1 + 16 * m + R] = u < h1 ? net->b[0][u] : 0.0f;
    }
  for (int m = 0; m < H2T; m++)
    for (int R = 0; R < 16; R++) {
      int u = unit(m, R);
      img[L.b2 + 16 * m + R] = u < h2 ? net->b[1][u] : 0.0f;
    }
  for (int g = 0; g < NGT * 16; g++) {
    img[L.b3 + g] = g < ny ? net->b[2][g] : 0.0f;
    img[L.sd + g] = (g < ny && net->has_out_scaling()) ? net->out_std[g] : 0.0f;
    img[L.mn + g] = (g < ny && net->has_out_scaling()) ? net->out_mean[g] : 0.0f;
  }
  float *d = nullptr;
  RRTMGPNN_HIP(hipMalloc(&d, sizeof(float) * img.size()));
  RRTMGPNN_HIP(hipMemcpy(d, img.data(), sizeof(float) * img.size(), hipMemcpyHostToDevice));
  net->d_packed = d;
  net->packed_floats = L.total;
  net->k1s = K1S; net->h1t = H1T; net->h2t = H2T; net->ngt = NGT;
  net->off_l1 = L.l1; net->off_l2 = L.l2; net->off_l3 = L.l3; net->off_b1 = L.b1; net->off_b2 = L.b2;
  net->off_b3 = L.b3; net->off_std = L.sd; net->off_mean = L.mn;
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// Fused MLP kernel.
// ------------------------------------------------------------------------------------------
struct MlpArgs {
  const float *x;        // (nx, nbatch)
  const float *col_dry;  // (nbatch)
  float *out0, *out1, *out2;
  const float *imgA, *imgB;
  int nx;
  int ngpt;    // g-points of the physical outputs
  int ngt;     // output g-tiles per network (NGT)
  int imgA_floats, imgB_floats;
  int vec4;    // outputs may be stored 16 bytes at a time (ngpt % 4 == 0, 16-byte aligned arrays)
  int actA[3], actB[3];
  long long nbatch;
  // in-kernel inputs (MlpInputs, the fused gas-optics entries): x and col_dry formed per sample from the state
  const float *play, *tlay, *plev, *h2o;
  int nlay;
  GasArgs gas;
  NnInArgs sc;
};

// Hidden layers of one network for a 16-sample tile: returns H2 accumulators.
template <int K1S, int H1T, int H2T, int ACTS>
__device__ __forceinline__ void mlp_hidden(const float *__restrict__ img, int NGT, const float (&xv)[K1S], int lane,
                                           int act1, int act2, floatx4 (&h2)[H2T])
{
  const ImgLayout L = img_layout(K1S, H1T, H2T, NGT);
  const int q = lane >> 4;
  floatx4 h1[H1T];
#pragma unroll
  for (int mo = 0; mo < H1T; mo++) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < K1S; t++)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(img[L.l1 + (mo * K1S + t) * 64 + lane], xv[t], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; r++) acc[r] = act_hidden<ACTS>(act1, acc[r] + img[L.b1 + 16 * mo + 4 * q + r]);
    h1[mo] = acc;
  }
#pragma unroll
  for (int mo = 0; mo < H2T; mo++) {
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int m = 0; m < H1T; m++)
#pragma unroll
      for (int t = 0; t < 4; t++)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(img[L.l2 + (mo * 4 * H1T + 4 * m + t) * 64 + lane], h1[m][t], acc,
                                                   0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; r++) acc[r] = act_hidden<ACTS>(act2, acc[r] + img[L.b2 + 16 * mo + 4 * q + r]);
    h2[mo] = acc;
  }
}

template <int H2T>
__device__ __forceinline__ floatx4 mlp_out_tile(const float *__restrict__ img, int l3, int go, const floatx4 (&h2)[H2T],
                                                int lane)
{
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < H2T; m++)
#pragma unroll
    for (int t = 0; t < 4; t++)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(img[l3 + (go * 4 * H2T + 4 * m + t) * 64 + lane], h2[m][t], acc, 0, 0,
                                                 0);
  return acc;
}

// Threads per MLP block: the weight images live once per block in LDS, so a wider block raises the waves per SIMD
// that share one copy of them (a 1024-thread LW instance was 13 % faster alone at C3 but took every register of every
// SIMD, and the overlapped C3 step got 18 % slower).  The shipped pairs' output g-tile counts are compiled in (LW 16,
// SW 14): the output loop then unrolls (LW 4 tiles per trip: -5 % C3 / -7 % C4 against the runtime loop, full
// unrolling spills; SW 2: -9 % at C4), and the next tile's inputs are loaded before this tile's stores, so the wait
// for them (vmcnt counts loads and stores together, in order) no longer drains the stores.
constexpr int kMlpThreads = 512, kGoUnroll = 1;

// XIN: the inputs are formed in-kernel (compute_nn_inputs + get_col_dry per sample, the expressions of
// nn_inputs_kernel and col_dry_kernel) instead of read from nn_inputs / col_dry arrays.  Lane (j, q) needs inputs
// k = 4t + q of sample s0 + j: the raw state values are loaded a tile ahead (with the next tile's prefetch) and
// turned into inputs at the tile's start.
template <int AK, int AH1, int AH2, int BK, int BH1, int BH2, int MODE, int ACTS, int NGTC = 0, bool XIN = false,
          int NT = kMlpThreads>
__global__ __launch_bounds__(NT) void mlp_pair_kernel(MlpArgs a)
{
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // Stage both weight images in LDS (read by every tile of every wave of this block).
  {
    const int nA = a.imgA_floats, nB = (MODE == MLP_LW_PAIR || MODE == MLP_SW_PAIR) ? a.imgB_floats : 0;
    for (int i = threadIdx.x; i < nA; i += blockDim.x) lds[i] = a.imgA[i];
    for (int i = threadIdx.x; i < nB; i += blockDim.x) lds[nA + i] = a.imgB[i];
  }
  __syncthreads();
  const float *imgA = lds;
  const float *imgB = lds + a.imgA_floats;
  const int lane = threadIdx.x & 63, j = lane & 15, q = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nwaves = blockDim.x >> 6;
  const int NGT = NGTC > 0 ? NGTC : a.ngt, nx = a.nx, ngpt = a.ngpt;
  const ImgLayout LA = img_layout(AK, AH1, AH2, NGT);
  const ImgLayout LB = img_layout(BK, BH1, BH2, NGT);
  const long long ntiles = (a.nbatch + 15) / 16;

  const long long tstride = (long long)gridDim.x * nwaves;
  // Layer-1 B operand: x[sample s0+j][k = 4t+q].  XIN: raw[t] holds the state value input k is formed from
  // (t = 0: tlay, play, h2o or o3 by q; t > 0: gas 4t+q), raw[AK..AK+2] = h2o, p(lev ilay), p(lev ilay+1) for col_dry.
  constexpr int NR = XIN ? AK + 3 : AK;
  auto load_x = [&](long long tl, float (&xv)[NR]) {
    const long long s = tl * 16 + j;
    if constexpr (XIN) {
      const bool ok = s < a.nbatch;
      const long long sc = ok ? s : 0;
      const int ilay = (int)(sc % a.nlay);
      const long long icol = sc / a.nlay;
      // inputs 3, 4 (h2o, o3) are 2-D; constant indices keep the pointers in SGPRs (a lane index would spill them)
      const float *p0 = q == 0 ? a.tlay : (q == 1 ? a.play : (q == 2 ? a.gas.p[2] : a.gas.p[3]));
      xv[0] = (ok && q < nx) ? p0[sc] : 0.0f;
#pragma unroll
      for (int t = 1; t < AK; t++) {
        const int k = 4 * t + q;
        const float *pk = a.gas.p[4 * t];
        int nd = a.gas.nd[4 * t];
#pragma unroll
        for (int r = 1; r < 4; r++)
          if (q == r) { pk = a.gas.p[4 * t + r]; nd = a.gas.nd[4 * t + r]; }
        const long long idx = nd == 0 ? 0 : (nd == 1 ? (long long)ilay : sc);
        xv[t] = (ok && k < nx && pk) ? pk[idx] : 0.0f;
      }
      const float *pl = a.plev + (size_t)(a.nlay + 1) * icol;
      xv[AK] = ok ? a.h2o[sc] : 0.0f;
      xv[AK + 1] = ok ? pl[ilay] : 0.0f;
      xv[AK + 2] = ok ? pl[ilay + 1] : 1.0f;
    } else {
#pragma unroll
      for (int t = 0; t < AK; t++) {
        int k = 4 * t + q;
        xv[t] = (s < a.nbatch && k < nx) ? a.x[(size_t)s * nx + k] : 0.0f;
      }
    }
  };
  // XIN: compute_nn_inputs (nn_inputs_kernel's expressions) from the raw values, in place; returns col_dry
  auto form_x = [&](float (&xv)[NR]) -> float {
    if constexpr (XIN) {
      const float r0 = xv[0];
      const float v0 = q == 1 ? ref_logf(r0) : (q >= 2 ? sqrtf(sqrtf(r0)) : r0);
      float mn = a.sc.mn[0], mx = a.sc.mx[0];
#pragma unroll
      for (int r = 1; r < 4; r++)
        if (q == r) { mn = a.sc.mn[r]; mx = a.sc.mx[r]; }
      xv[0] = q < nx ? (v0 - mn) / (mx - mn) : 0.0f;
#pragma unroll
      for (int t = 1; t < AK; t++) {
        const int k = 4 * t + q;
        float mnk = a.sc.mn[4 * t], mxk = a.sc.mx[4 * t];
#pragma unroll
        for (int r = 1; r < 4; r++)
          if (q == r && 4 * t + r < kMaxInputs) { mnk = a.sc.mn[4 * t + r]; mxk = a.sc.mx[4 * t + r]; }
        xv[t] = k < nx ? (xv[t] - mnk) / (mxk - mnk) : 0.0f;
      }
      return col_dry_of(xv[AK], xv[AK + 1], xv[AK + 2]);
    } else {
      return 0.0f;
    }
  };
  float xn[NR];  // NGTC: the next tile's inputs, loaded before this tile's stores
  if constexpr (NGTC > 0) load_x((long long)blockIdx.x * nwaves + wave, xn);
  for (long long tile = (long long)blockIdx.x * nwaves + wave; tile < ntiles; tile += tstride) {
    const long long s0 = tile * 16;
    float xv[NR];
    if constexpr (NGTC > 0) {
#pragma unroll
      for (int t = 0; t < NR; t++) xv[t] = xn[t];
      load_x(tile + tstride, xn);
    } else {
      load_x(tile, xv);
    }
    const float cd_in = form_x(xv);
    float x1[AK];
#pragma unroll
    for (int t = 0; t < AK; t++) x1[t] = xv[t];
    floatx4 hA[AH2];
    mlp_hidden<AK, AH1, AH2, ACTS>(imgA, NGT, x1, lane, a.actA[0], a.actA[1], hA);
    floatx4 hB[BH2];
    if constexpr (MODE == MLP_LW_PAIR || MODE == MLP_SW_PAIR) {
      static_assert(BK == AK, "paired networks share their inputs");
      mlp_hidden<BK, BH1, BH2, ACTS>(imgB, NGT, x1, lane, a.actB[0], a.actB[1], hB);
    }
    // Layer 3 runs with the weights as the A operand (rows = g-points) and the hidden activations as B
    // (columns = samples): lane (j, q) holds g = 16go + 4q + r, r = 0..3, of sample s0 + j, so each lane
    // stores 16 contiguous bytes per output array.  Same k-ordered chains as the oracle, same bits.
    const long long s = s0 + j;
    const bool sok = s < a.nbatch;
    float cd = 0.0f;
    if constexpr (XIN) cd = sok ? cd_in : 0.0f;
    else if constexpr (MODE != MLP_PLAIN) cd = sok ? a.col_dry[s] : 0.0f;
    // 4 consecutive g of one sample: one 16-byte store when the row allows it, else element by element
    auto put4 = [&](float *out, int row, int gc, const floatx4 &v) {
      if (!sok) return;
      float *p = out + (size_t)s * row + gc;
      if (a.vec4 && gc + 3 < row) {
        *(floatx4 *)p = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++)
          if (gc + r < row) p[r] = v[r];
      }
    };
    auto out_tile = [&](int go) {
      const int g0 = 16 * go + 4 * q;
      const floatx4 yA = mlp_out_tile<AH2>(imgA, LA.l3, go, hA, lane);
      const floatx4 bA = *(const floatx4 *)&imgA[LA.b3 + g0];
      if constexpr (MODE == MLP_PLAIN) {
        floatx4 o;
#pragma unroll
        for (int r = 0; r < 4; r++) o[r] = act_out<ACTS>(a.actA[2], yA[r] + bA[r]);
        put4(a.out0, ngpt, g0, o);
      } else if constexpr (MODE == MLP_LW_BOTH) {
        // single model, outputs [0,ngpt) -> tau, [ngpt, 2 ngpt) -> pfrac (mo_gas_optics_kernels.F90:754-766)
        const floatx4 sd = *(const floatx4 *)&imgA[LA.sd + g0], mn = *(const floatx4 *)&imgA[LA.mn + g0];
        floatx4 tau, pf;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const float y = yA[r] + bA[r];
          float t = sd[r] * y;
          t = t + mn[r];
          tau[r] = pow8(t) * cd;
          pf[r] = y * y;
        }
        if (a.vec4 && g0 + 3 < ngpt) {
          put4(a.out0, ngpt, g0, tau);
        } else if (a.vec4 && g0 >= ngpt) {
          put4(a.out1, ngpt, g0 - ngpt, pf);
        } else if (sok) {  // a 4-group straddling the tau / pfrac boundary or the end
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int g = g0 + r;
            if (g < ngpt) a.out0[(size_t)s * ngpt + g] = tau[r];
            else if (g < 2 * ngpt) a.out1[(size_t)s * ngpt + (g - ngpt)] = pf[r];
          }
        }
      } else {
        const floatx4 sdA = *(const floatx4 *)&imgA[LA.sd + g0], mnA = *(const floatx4 *)&imgA[LA.mn + g0];
        if constexpr (MODE == MLP_SW_ABS) {
          floatx4 tau;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            float t = sdA[r] * (yA[r] + bA[r]);
            t = t + mnA[r];
            tau[r] = pow8(t) * cd;
          }
          put4(a.out0, ngpt, g0, tau);
        } else {
          const floatx4 yB = mlp_out_tile<BH2>(imgB, LB.l3, go, hB, lane);
          const floatx4 bB = *(const floatx4 *)&imgB[LB.b3 + g0];
          if constexpr (MODE == MLP_LW_PAIR) {
            floatx4 tau, pf;
#pragma unroll
            for (int r = 0; r < 4; r++) {
              float t = sdA[r] * (yA[r] + bA[r]);
              t = t + mnA[r];
              const float p = yB[r] + bB[r];
              tau[r] = pow8(t) * cd;
              pf[r] = p * p;
            }
            {
              put4(a.out0, ngpt, g0, tau);  // tau
              put4(a.out1, ngpt, g0, pf);   // pfrac
            }
          } else {  // MLP_SW_PAIR
            const floatx4 sdB = *(const floatx4 *)&imgB[LB.sd + g0], mnB = *(const floatx4 *)&imgB[LB.mn + g0];
            floatx4 tot, ssa;
#pragma unroll
            for (int r = 0; r < 4; r++) {
              float ta = sdA[r] * (yA[r] + bA[r]);
              ta = ta + mnA[r];
              const float vabs = pow8(ta) * cd;
              float tr = sdB[r] * (yB[r] + bB[r]);
              tr = tr + mnB[r];
              const float vray = pow8(tr) * cd;
              tot[r] = vabs + vray;
              ssa[r] = vray / tot[r];
            }
            put4(a.out0, ngpt, g0, tot);  // tau = tau_abs + tau_ray
            put4(a.out1, ngpt, g0, ssa);  // ssa
            if (a.out2) put4(a.out2, ngpt, g0, floatx4{0.0f, 0.0f, 0.0f, 0.0f});  // g
          }
        }
      }
    };
    if constexpr (NGTC > 0 && MODE == MLP_LW_PAIR) {
#pragma unroll 4
      for (int go = 0; go < NGTC; go++) out_tile(go);
    } else if constexpr (NGTC > 0) {
#pragma unroll 2
      for (int go = 0; go < NGTC; go++) out_tile(go);
    } else {
#pragma unroll kGoUnroll
      for (int go = 0; go < NGT; go++) out_tile(go);
    }
  }
}

template <int AK, int AH1, int AH2, int BK, int BH1, int BH2, int MODE, int ACTS, int NGTC = 0, bool XIN = false,
          int NT = kMlpThreads>
static int launch_mlp_acts(rrtmgpnn_context *ctx, MlpArgs &a)
{
  auto kern = mlp_pair_kernel<AK, AH1, AH2, BK, BH1, BH2, MODE, ACTS, NGTC, XIN, NT>;
  size_t lds = sizeof(float) * (size_t)(a.imgA_floats + ((MODE == MLP_LW_PAIR || MODE == MLP_SW_PAIR) ? a.imgB_floats : 0));
  if (lds > 160 * 1024) return fail(RRTMGPNN_ERR_UNSUPPORTED, "mlp: weight images exceed 160 KiB of LDS");
  // the dynamic-LDS limit, raised once per (instantiation, device)
  if (lds > 64 * 1024)
    if (int rc = raise_lds_limit((const void *)kern)) return rc;
  long long ntiles = (a.nbatch + 15) / 16;
  constexpr int kThreads = NT;
  const int wpb = kThreads / 64;
  int per_cu = std::max(1, (int)((160 * 1024) / std::max<size_t>(lds, 1)));
  per_cu = std::min(per_cu, 2048 / kThreads);
  long long want = (ntiles + wpb - 1) / wpb;
  const int cus = ctx->mlp_max_cus > 0 ? std::min(ctx->mlp_max_cus, ctx->num_cus) : ctx->num_cus;
  long long grid = std::min<long long>(want, (long long)cus * per_cu);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kThreads), lds, ctx->stream, a);
  RRTMGPNN_LAUNCH_CHECK("mlp_pair_kernel");
  return RRTMGPNN_OK;
}

template <int AK, int AH1, int AH2, int BK, int BH1, int BH2, int MODE>
static int launch_mlp_t(rrtmgpnn_context *ctx, MlpArgs &a)
{
  const bool pair = MODE == MLP_LW_PAIR || MODE == MLP_SW_PAIR;
  auto std_acts = [](const int *act) {
    return act[0] == RRTMGPNN_ACT_SOFTSIGN && act[1] == RRTMGPNN_ACT_SOFTSIGN && act[2] == RRTMGPNN_ACT_LINEAR;
  };
  if (std_acts(a.actA) && (!pair || std_acts(a.actB))) {
    // the shipped pairs' output tile counts compiled in: LW g256 (16 tiles), SW g224 (14)
    constexpr bool lw = MODE == MLP_LW_PAIR && AK == 5 && AH1 == 4 && AH2 == 4 && BH1 == 1 && BH2 == 1;
    constexpr bool sw = MODE == MLP_SW_PAIR && AK == 2 && AH1 == 1 && AH2 == 1 && BH1 == 1 && BH2 == 1;
    if constexpr (lw) {
      if (a.ngt == 16 && a.play) return launch_mlp_acts<AK, AH1, AH2, BK, BH1, BH2, MODE, 1, 16, true>(ctx, a);
      if (a.ngt == 16) return launch_mlp_acts<AK, AH1, AH2, BK, BH1, BH2, MODE, 1, 16>(ctx, a);
    }
    if constexpr (sw) {
      if (a.ngt == 14 && a.play) return launch_mlp_acts<AK, AH1, AH2, BK, BH1, BH2, MODE, 1, 14, true>(ctx, a);
      if (a.ngt == 14) return launch_mlp_acts<AK, AH1, AH2, BK, BH1, BH2, MODE, 1, 14>(ctx, a);
    }
    if (a.play) return RRTMGPNN_ERR_UNSUPPORTED;  // no in-kernel-input instance: the caller runs the three kernels
    return launch_mlp_acts<AK, AH1, AH2, BK, BH1, BH2, MODE, 1>(ctx, a);
  }
  if (a.play) return RRTMGPNN_ERR_UNSUPPORTED;
  return launch_mlp_acts<AK, AH1, AH2, BK, BH1, BH2, MODE, 0>(ctx, a);
}

// Shape dispatch: the shipped models (Appendix A of SURVEY.md).
//   LW g256 pair: abs 18-58-58-256 (K1S 5, H 4,4) + pfrac 18-16-16-256 (5, 1,1)
//   SW g224 pair: 7-16-16-224 (2, 1,1) x 2
//   LW g128 both: 18-64-64-256 (5, 4,4)
#define RRTMGPNN_MLP_SHAPES(X) \
  X(5, 4, 4)                   \
  X(5, 1, 1)                   \
  X(2, 1, 1)                   \
  X(2, 2, 2)                   \
  X(5, 2, 2)                   \
  X(5, 5, 5)                   \
  X(5, 3, 3)                   \
  X(5, 8, 8)

static bool shape_is(const rrtmgpnn_network *n, int k, int h1, int h2)
{
  return n && n->d_packed && n->k1s == k && n->h1t == h1 && n->h2t == h2;
}

int launch_mlp(rrtmgpnn_context *ctx, MlpMode mode, const rrtmgpnn_network *A, const rrtmgpnn_network *B,
               long long nbatch, int ngpt, const float *x, const float *col_dry, float *out0, float *out1, float *out2,
               const MlpInputs *in)
{
  if (nbatch <= 0) return RRTMGPNN_OK;
  if (mode == MLP_LW_PAIR || mode == MLP_LW_BOTH || mode == MLP_SW_PAIR) {  // the 32x32x2 kernel first (kernels_nn32.hip)
    const int rc = launch_mlp32(ctx, mode, A, B, nbatch, ngpt, x, col_dry, out0, out1, out2, in);
    if (rc != RRTMGPNN_ERR_UNSUPPORTED) return rc;
  }
  if (!A || !A->d_packed) return fail(RRTMGPNN_ERR_UNSUPPORTED, "mlp: network has no MFMA image (needs 3 layers)");
  bool paired = (mode == MLP_LW_PAIR || mode == MLP_SW_PAIR);
  if (paired && (!B || !B->d_packed)) return fail(RRTMGPNN_ERR_UNSUPPORTED, "mlp: second network has no MFMA image");
  if (paired && (A->ngt != B->ngt || A->k1s != B->k1s || A->dims[0] != B->dims[0]))
    return fail(RRTMGPNN_ERR_ARGUMENT, "mlp: paired networks differ in inputs or outputs");
  MlpArgs a{};
  a.x = x; a.col_dry = col_dry; a.out0 = out0; a.out1 = out1; a.out2 = out2;
  a.imgA = A->d_packed; a.imgA_floats = A->packed_floats;
  a.imgB = paired ? B->d_packed : nullptr; a.imgB_floats = paired ? B->packed_floats : 0;
  a.nx = A->dims[0]; a.ngpt = ngpt; a.ngt = A->ngt; a.nbatch = nbatch;
  if (in) {  // fused gas optics: x and col_dry formed in-kernel (returns RRTMGPNN_ERR_UNSUPPORTED, no error set,
             // when no such instance exists for the shape; the caller then runs the separate kernels)
    a.play = in->play; a.tlay = in->tlay; a.plev = in->plev; a.h2o = in->h2o; a.nlay = in->nlay;
    a.gas = in->gas;
    for (int k = 0; k < kMaxInputs; k++) { a.sc.mn[k] = in->mn[k]; a.sc.mx[k] = in->mx[k]; }
  }
  auto al16 = [](const float *p) { return ((uintptr_t)p & 15) == 0; };
  a.vec4 = (ngpt % 4 == 0) && al16(out0) && (!out1 || al16(out1)) && (!out2 || al16(out2));
  for (int i = 0; i < 3; i++) { a.actA[i] = A->act[i]; a.actB[i] = paired ? B->act[i] : 0; }

#define TRY_PAIR(AK, AH1, AH2, BK, BH1, BH2, MODE) \
  if (shape_is(A, AK, AH1, AH2) && shape_is(B, BK, BH1, BH2)) return launch_mlp_t<AK, AH1, AH2, BK, BH1, BH2, MODE>(ctx, a);
#define TRY_ONE(AK, AH1, AH2, MODE) \
  if (shape_is(A, AK, AH1, AH2)) return launch_mlp_t<AK, AH1, AH2, AK, 1, 1, MODE>(ctx, a);

  switch (mode) {
  case MLP_LW_PAIR:
    TRY_PAIR(5, 4, 4, 5, 1, 1, MLP_LW_PAIR)
    TRY_PAIR(5, 5, 5, 5, 2, 2, MLP_LW_PAIR)
    TRY_PAIR(5, 4, 4, 5, 2, 2, MLP_LW_PAIR)
    break;
  case MLP_SW_PAIR:
    TRY_PAIR(2, 1, 1, 2, 1, 1, MLP_SW_PAIR)
    TRY_PAIR(2, 2, 2, 2, 1, 1, MLP_SW_PAIR)
    TRY_PAIR(2, 2, 2, 2, 2, 2, MLP_SW_PAIR)
    break;
  case MLP_SW_ABS:
#define X(K, H1, H2) TRY_ONE(K, H1, H2, MLP_SW_ABS)
    RRTMGPNN_MLP_SHAPES(X)
#undef X
    break;
  case MLP_LW_BOTH:
#define X(K, H1, H2) TRY_ONE(K, H1, H2, MLP_LW_BOTH)
    RRTMGPNN_MLP_SHAPES(X)
#undef X
    break;
  case MLP_PLAIN:
#define X(K, H1, H2) TRY_ONE(K, H1, H2, MLP_PLAIN)
    RRTMGPNN_MLP_SHAPES(X)
#undef X
    break;
  }
#undef TRY_PAIR
#undef TRY_ONE
  return fail(RRTMGPNN_ERR_UNSUPPORTED, "mlp: no compiled MFMA kernel for this network shape");
}

// ------------------------------------------------------------------------------------------
// Generic (any depth/width) forward, one thread per sample: correctness path for networks the
// fused kernel is not instantiated for.  Hidden widths <= 256.
// ------------------------------------------------------------------------------------------
struct GenArgs {
  const float *raw;
  long long w_off[kMaxLayers], b_off[kMaxLayers];
  int dims[kMaxLayers + 1];
  int act[kMaxLayers];
  int nlayers;
};

__global__ void mlp_generic_kernel(GenArgs g, long long nbatch, const float *__restrict__ x, float *__restrict__ out)
{
  long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nbatch) return;
  float a[256], b[256];
  int nin = g.dims[0];
  for (int k = 0; k < nin; k++) a[k] = x[(size_t)s * nin + k];
  for (int n = 0; n < g.nlayers; n++) {
    int nout = g.dims[n + 1];
    const float *W = g.raw + g.w_off[n];
    const float *B = g.raw + g.b_off[n];
    bool last = (n == g.nlayers - 1);
    for (int i = 0; i < nout; i++) {
      float acc = 0.0f;
      for (int k = 0; k < nin; k++) acc = fmaf(W[(size_t)k * nout + i], a[k], acc);
      float v = activate(g.act[n], acc + B[i]);
      if (last) out[(size_t)s * nout + i] = v;
      else b[i] = v;
    }
    if (!last)
      for (int i = 0; i < nout; i++) a[i] = b[i];
    nin = nout;
  }
}

int launch_mlp_generic(rrtmgpnn_context *ctx, const rrtmgpnn_network *net, long long nbatch, const float *x,
                       float *out)
{
  if (nbatch <= 0) return RRTMGPNN_OK;
  GenArgs g{};
  g.raw = net->d_raw;
  g.nlayers = net->nlayers;
  for (int n = 0; n <= net->nlayers; n++) {
    g.dims[n] = net->dims[n];
    if (n > 0 && n < net->nlayers && net->dims[n] > 256)
      return fail(RRTMGPNN_ERR_UNSUPPORTED, "generic mlp: hidden width > 256");
  }
  if (net->dims[0] > 256) return fail(RRTMGPNN_ERR_UNSUPPORTED, "generic mlp: input width > 256");
  for (int n = 0; n < net->nlayers; n++) {
    g.w_off[n] = (long long)net->raw_w_off[n];
    g.b_off[n] = (long long)net->raw_b_off[n];
    g.act[n] = net->act[n];
  }
  hipLaunchKernelGGL(mlp_generic_kernel, dim3((unsigned)((nbatch + 127) / 128)), dim3(128), 0, ctx->stream, g, nbatch,
                     x, out);
  RRTMGPNN_LAUNCH_CHECK("mlp_generic_kernel");
  return RRTMGPNN_OK;
}

}  // namespace rrtmgpnn
