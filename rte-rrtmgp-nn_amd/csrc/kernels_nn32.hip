// kernels_nn32.hip -- the LW gas-optics networks on v_mfma_f32_32x32x2_f32 (gfx950), 32 samples per wave tile.
//
// Same networks, epilogues and bits as mlp_pair_kernel's LW modes (kernels_nn.hip):
//   LW pair : tau = (std*(y+b)+mean)^8 * col_dry  and  pfrac = (y+b)^2
//             (predict_nn_lw_blas_sp, rrtmgp/kernels/mo_gas_optics_kernels.F90:690-774;
//              neural/mod_network_rrtmgp.F90:125-317)
//   LW both : one model with 2*ngpt outputs (output_sgemm_lw, mod_network_rrtmgp.F90:319-409;
//             mo_gas_optics_kernels.F90:744-772)
// optionally with the inputs formed in-kernel (compute_nn_inputs + get_col_dry, the fused gas-optics entry).
//
// Why a second tiling: the 16x16x4 f32 MFMA issues every 32 cycles but its dependent-accumulator latency is 40, and
// each instruction takes its weight operand from LDS (one ds_read per 2 048 flop).  The 32x32x2 form issues every 64
// cycles with a 64-cycle dependent latency, so a single accumulation chain runs at the issue rate, and it does
// 4 096 flop per operand; the weight images are packed so one ds_read_b128 feeds 4 MFMAs.  The shipped sizes also
// divide evenly: 18 inputs = 9 K-steps, 58 hidden units = 29 K-steps (the 16x16x4 tiling pads 18 -> 20, 58 -> 64).
//
// MFMA mapping (v_mfma_f32_32x32x2_f32: exact f32, D = (C + a0*b0) + a1*b1 as an fmaf chain):
//   lane l: j = l & 31 (sample / output row), h = l >> 5 (k within the step).
//   A[i = j][k = h], B[k = h][col = j]; accumulator register r holds D[row (r&3) + 8(r>>2) + 4h][col j].
//   Hidden layers compute H^T (units x samples): A = packed W^T, B = activations.  Physical row R of hidden tile mo
//   holds logical unit u = 32mo + 2((R&3) + 4(R>>3)) + ((R>>2)&1), so register r of lane half h holds unit
//   32mo + 2r + h: K-step S = 16mo + r of the next layer takes units 2S (h = 0) and 2S+1 (h = 1) from the lanes'
//   own registers, and every dot product accumulates in ascending k -- the oracle's fmaf order, bit for bit.
//   The output layer computes Y^T (g-points x samples) with the weights as A: lane (j, h) holds g = 32go + 8b + 4h + i
//   (b, i = 0..3) of sample j, 4 float4 stores per output array and g-tile.
#include "nn_device.hpp"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <vector>

namespace rrtmgpnn {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------------------
// Packed image (floats) of a 3-layer network [nx, h1, h2, ny]:
//   KS = ceil(nx/2), HT1 = ceil(h1/32), N2 = ceil(h1/2), HT2 = ceil(h2/32), N3 = ceil(h2/2), NGT = ceil(ny/32);
//   q(n) = ceil(n/4): operand steps are grouped by 4, [group][lane][4], one 16-byte LDS read per lane per group.
//   L1 [HT1][q(KS)][64][4]  lane (i, h), step s: W1[k = 2s+h][u(mo, i)]
//   L2 [HT2][q(N2)][64][4]  step S: W2[k = 2S+h][u(mo, i)]
//   L3 [NGT][q(N3)][64][4]  step S: W3[k = 2S+h][g = 32go + i]
//   B1 [HT1][2][16], B2 [HT2][2][16]: b[32mo + 2r + h] at [mo][h][r] (a lane's 16 biases are contiguous)
//   B3, STD, MEAN [NGT*32] by g
//   XS [2][16] input minimum, then [2][16] input range (max - min) of input k = 2t + h at [h][t] (compute_nn_inputs'
//      scaling, in the fused entry); past nx: minimum 0, range 1, so a zero raw value scales to 0
// ------------------------------------------------------------------------------------------
struct Img32 {
  int l1, l2, l3, b1, b2, b3, sd, mn, xs, total;
};
__host__ __device__ constexpr Img32 img32_layout(int KS, int HT1, int N2, int HT2, int N3, int NGT)
{
  Img32 L{};
  L.l1 = 0;
  L.l2 = L.l1 + HT1 * ((KS + 3) / 4) * 256;
  L.l3 = L.l2 + HT2 * ((N2 + 3) / 4) * 256;
  L.b1 = L.l3 + NGT * ((N3 + 3) / 4) * 256;
  L.b2 = L.b1 + HT1 * 32;
  L.b3 = L.b2 + HT2 * 32;
  L.sd = L.b3 + NGT * 32;
  L.mn = L.sd + NGT * 32;
  L.xs = L.mn + NGT * 32;
  L.total = L.xs + 64;
  return L;
}

int pack_network32(rrtmgpnn_network *net)
{
  if (net->nlayers != 3) return RRTMGPNN_OK;
  const int nx = net->dims[0], h1 = net->dims[1], h2 = net->dims[2], ny = net->dims[3];
  if (nx > kMaxInputs || h1 > 64 || h2 > 64) return RRTMGPNN_OK;  // the 16x16x4 kernel covers the rest
  const int KS = (nx + 1) / 2, HT1 = (h1 + 31) / 32, N2 = (h1 + 1) / 2, HT2 = (h2 + 31) / 32, N3 = (h2 + 1) / 2,
            NGT = (ny + 31) / 32;
  const Img32 L = img32_layout(KS, HT1, N2, HT2, N3, NGT);
  std::vector<float> img(L.total, 0.0f);
  const std::vector<float> &W1 = net->w[0], &W2 = net->w[1], &W3 = net->w[2];
  auto unit = [](int mo, int R) { return 32 * mo + 2 * ((R & 3) + 4 * (R >> 3)) + ((R >> 2) & 1); };
  // operand arrays: [tile][step group][lane][4]
  auto put = [&](int base, int nsteps, int tile, int S, int l, float v) {
    const int q = (nsteps + 3) / 4;
    img[base + ((tile * q + S / 4) * 64 + l) * 4 + (S & 3)] = v;
  };
  for (int mo = 0; mo < HT1; mo++)
    for (int s = 0; s < KS; s++)
      for (int l = 0; l < 64; l++) {
        const int i = l & 31, h = l >> 5, k = 2 * s + h, u = unit(mo, i);
        put(L.l1, KS, mo, s, l, (k < nx && u < h1) ? W1[(size_t)k * h1 + u] : 0.0f);
      }
  for (int mo = 0; mo < HT2; mo++)
    for (int S = 0; S < N2; S++)
      for (int l = 0; l < 64; l++) {
        const int i = l & 31, h = l >> 5, k = 2 * S + h, u = unit(mo, i);
        put(L.l2, N2, mo, S, l, (k < h1 && u < h2) ? W2[(size_t)k * h2 + u] : 0.0f);
      }
  for (int go = 0; go < NGT; go++)
    for (int S = 0; S < N3; S++)
      for (int l = 0; l < 64; l++) {
        const int i = l & 31, h = l >> 5, k = 2 * S + h, g = 32 * go + i;
        put(L.l3, N3, go, S, l, (k < h2 && g < ny) ? W3[(size_t)k * ny + g] : 0.0f);
      }
  for (int mo = 0; mo < HT1; mo++)
    for (int h = 0; h < 2; h++)
      for (int r = 0; r < 16; r++) {
        const int u = 32 * mo + 2 * r + h;
        img[L.b1 + (mo * 2 + h) * 16 + r] = u < h1 ? net->b[0][u] : 0.0f;
      }
  for (int mo = 0; mo < HT2; mo++)
    for (int h = 0; h < 2; h++)
      for (int r = 0; r < 16; r++) {
        const int u = 32 * mo + 2 * r + h;
        img[L.b2 + (mo * 2 + h) * 16 + r] = u < h2 ? net->b[1][u] : 0.0f;
      }
  for (int g = 0; g < NGT * 32; g++) {
    img[L.b3 + g] = g < ny ? net->b[2][g] : 0.0f;
    img[L.sd + g] = (g < ny && net->has_out_scaling()) ? net->out_std[g] : 0.0f;
    img[L.mn + g] = (g < ny && net->has_out_scaling()) ? net->out_mean[g] : 0.0f;
  }
  for (int h = 0; h < 2; h++)
    for (int t = 0; t < 16; t++) {
      const int k = 2 * t + h;
      const bool on = k < nx && k < (int)net->in_min.size() && k < (int)net->in_max.size();
      img[L.xs + h * 16 + t] = on ? net->in_min[k] : 0.0f;
      img[L.xs + 32 + h * 16 + t] = on ? net->in_max[k] - net->in_min[k] : 1.0f;
    }
  float *d = nullptr;
  RRTMGPNN_HIP(hipMalloc(&d, sizeof(float) * img.size()));
  RRTMGPNN_HIP(hipMemcpy(d, img.data(), sizeof(float) * img.size(), hipMemcpyHostToDevice));
  net->d_packed32 = d;
  net->packed32_floats = L.total;
  net->s32[0] = KS; net->s32[1] = HT1; net->s32[2] = N2; net->s32[3] = HT2; net->s32[4] = N3; net->s32[5] = NGT;
  return RRTMGPNN_OK;
}

// ------------------------------------------------------------------------------------------
// Kernel
// ------------------------------------------------------------------------------------------
// Every load and store of a tile goes through a raw buffer descriptor: a lane past the batch (or the lane half an
// input does not belong to) uses an offset past the descriptor's range, where loads return 0 and stores are dropped.
// The tile body then has no branch, so it is one basic block and the scheduler can interleave the output tiles'
// epilogues and stores with the next tiles' MFMA chains, and one network's activations with the other's MFMAs.
static constexpr uint32_t kOOB = 0x7ffff000u;  // past every descriptor's range (the host checks the sizes)
static constexpr uint32_t kMaxRecords = 0x7ff00000u;

struct Buf {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ Buf(const void *base, uint32_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)bytes, 0x00020000)) {}
  __device__ __forceinline__ float ld(uint32_t voff) const
  {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
  }
  __device__ __forceinline__ void st(float v, uint32_t voff) const
  {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, 0, 0);
  }
  __device__ __forceinline__ void st4(const floatx4 &v, uint32_t voff) const
  {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, voff, 0, 0);
  }
};

struct Mlp32Args {
  const float *x;        // (nx, nbatch)
  const float *col_dry;  // (nbatch)
  float *out0, *out1, *out2;
  const float *imgA, *imgB;
  int imgA_floats, imgB_floats;
  int nx, ngpt;
  int nbatch;
  // in-kernel inputs (the fused gas-optics entry)
  const float *play, *tlay, *plev, *h2o;
  int nlay, ncol;
  GasArgs gas;
  // per input k (host-made, so the device offsets need no branch): byte offset of sample s, layer ilay =
  // s * gsm[k] + ilay * glm[k] (2-D: 4, 0; 1-D: 0, 4; scalar: 0, 0); grec[k] = the array's bytes (0: absent or k >= nx)
  uint32_t gsm[kMaxInputs], glm[kMaxInputs], grec[kMaxInputs];
  // the same per input as a 2-bit code (0 absent, 1 scalar, 2 1-D, 3 2-D), 16 inputs per word (kMlpPackedIn)
  uint32_t gcode[(kMaxInputs + 15) / 16];
};

// In-kernel inputs of the LW pair: per-input multipliers and ranges from the packed codes (a few scalar ops per tile)
// and the gas pointers re-read per tile, instead of 3 x 18 words and 18 buffer descriptors held across the tile loop
// (163 SGPRs spilled into VGPR lanes, reloaded by 83 v_readlane per tile; now 16).  Round 5, alone, alternating,
// bitwise: C3 LW network 76.0 -> 74.8 us, C4 362.9 -> 357.3 us; serialised in-step 81.8 -> 79.4 us.  The SW pair (no
// spills) keeps the held form: the packed one made it 3 % slower.  A/B knob: tools/ablations.py mlp_packin.
constexpr bool kMlpPackedIn = true;

__device__ __forceinline__ floatx16 mfma32(float a, float b, const floatx16 &c)
{
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// D += sum over steps s < NS of W[tile][s] * v[s]  (v[s]: the lane's B operand of step s)
template <int NS>
__device__ __forceinline__ floatx16 mfma_chain(const float *__restrict__ w, int tile, const float (&v)[NS], int lane)
{
  constexpr int Q = (NS + 3) / 4;
  floatx16 acc = {};
  const floatx4 *wp = (const floatx4 *)w + (size_t)tile * Q * 64 + lane;
#pragma unroll
  for (int g4 = 0; g4 < Q; g4++) {
    const floatx4 wv = wp[g4 * 64];
#pragma unroll
    for (int e = 0; e < 4; e++)
      if (4 * g4 + e < NS) acc = mfma32(wv[e], v[4 * g4 + e], acc);
  }
  return acc;
}

// The output layer with the operands swapped: A = the layer-2 activations (lane (j, h): sample j, unit 2S+h, exactly
// the registers the B operand takes), B = the weights (lane (i, h): unit 2S+h, g-point 32go+i, exactly the image the A
// operand takes), so D = Y (samples x g-points): lane (c, h) holds g-point 32go + c of samples (r&3) + 8(r>>2) + 4h,
// and a store of one register writes two 128-byte row segments instead of 32 pieces of 32 bytes.  Same k order.
template <int NS>
__device__ __forceinline__ floatx16 mfma_chain_t(const float *__restrict__ w, int tile, const float (&v)[NS], int lane)
{
  constexpr int Q = (NS + 3) / 4;
  floatx16 acc = {};
  const floatx4 *wp = (const floatx4 *)w + (size_t)tile * Q * 64 + lane;
#pragma unroll
  for (int g4 = 0; g4 < Q; g4++) {
    const floatx4 wv = wp[g4 * 64];
#pragma unroll
    for (int e = 0; e < 4; e++)
      if (4 * g4 + e < NS) acc = mfma32(v[4 * g4 + e], wv[e], acc);
  }
  return acc;
}

// Hidden layers of one network for a 32-sample tile: returns the layer-2 activations as the output layer's B
// operands (N3 K-steps)
template <int KS, int HT1, int N2, int HT2, int N3, int NGT>
__device__ __forceinline__ void mlp32_hidden(const float *__restrict__ img, const float (&x)[KS], int lane,
                                             float (&h2)[N3])
{
  constexpr Img32 L = img32_layout(KS, HT1, N2, HT2, N3, NGT);
  const int h = lane >> 5;
  float h1[N2];
#pragma unroll
  for (int mo = 0; mo < HT1; mo++) {
    const floatx16 acc = mfma_chain<KS>(img + L.l1, mo, x, lane);
    const float *bb = img + L.b1 + (mo * 2 + h) * 16;
#pragma unroll
    for (int r = 0; r < 16; r++)
      if (16 * mo + r < N2) h1[16 * mo + r] = softsign(acc[r] + bb[r]);
  }
#pragma unroll
  for (int mo = 0; mo < HT2; mo++) {
    const floatx16 acc = mfma_chain<N2>(img + L.l2, mo, h1, lane);
    const float *bb = img + L.b2 + (mo * 2 + h) * 16;
#pragma unroll
    for (int r = 0; r < 16; r++)
      if (16 * mo + r < N3) h2[16 * mo + r] = softsign(acc[r] + bb[r]);
  }
}

// 8-wave blocks, one output g-tile per loop step.  The SW pair keeps the same block: 4- and 12-wave blocks measured
// equal or slower at C3 and C4 (SW network alone, alternating on one box, round 3: 12 waves +29 % at C3; 4 waves
// +1 %).  Round 5, the LW pair alone: 12-wave blocks (3 waves per SIMD, 168 VGPRs) +27-38 % at C3, 16-wave blocks
// +13 % at C3 and +23 % at C4 (profiles/r05/ab/lwshape_c{3,4}.txt); one g-tile per step instead of two equal alone
// and in C3 steps, C4 steps -0.6 % (3 of 3 alternating pairs; the SW network's in-step stage 62 -> 55 us, 29 -> 9 KB of
// code; profiles/r05/ab/u1_*.txt).  A/B knob: tools/ablations.py mlp_unroll.
constexpr int kMlp32Threads = 512, kSwNT = 512, kSwWPE = 1;

// A: (KS, AH1, AN2, AH2, AN3), B: (KS, BH1, BN2, BH2, BN3) -- B unused for MLP_LW_BOTH.  The host guarantees that the
// g-tiles are full: ngpt = 32 NGT (LW pair) or 2 ngpt = 32 NGT (LW both).  Dynamic LDS: the weight images, then 32
// floats per wave (the tile's column amounts, handed from the sample lanes to the row registers).
template <int KS, int AH1, int AN2, int AH2, int AN3, int BH1, int BN2, int BH2, int BN3, int NGT, int MODE, bool XIN,
          int NT = kMlp32Threads, int WPE = 1>
__global__ __launch_bounds__(NT, WPE) void mlp32_kernel(Mlp32Args a)
{
  constexpr bool kPair = MODE == MLP_LW_PAIR || MODE == MLP_SW_PAIR;
  extern __shared__ floatx4 lds4[];
  const float *imgA = (const float *)lds4;
  const float *imgB = imgA + a.imgA_floats;
  float *cds = (float *)lds4 + a.imgA_floats + (kPair ? a.imgB_floats : 0);
  constexpr Img32 LA = img32_layout(KS, AH1, AN2, AH2, AN3, NGT);
  constexpr Img32 LB = img32_layout(KS, BH1, BN2, BH2, BN3, NGT);
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nwaves = blockDim.x >> 6;
  const int nx = a.nx, ngpt = a.ngpt;
  const int ntiles = (a.nbatch + 31) / 32;
  const int tstride = gridDim.x * nwaves;
  const uint32_t nb4 = 4u * (uint32_t)a.nbatch;

  // Layer-1 B operand of step s: input k = 2s + h of sample s0 + j.  XIN: raw[s] holds the state value input k is
  // formed from (s = 0: tlay / play; s = 1: h2o / o3; s > 1: gas k), raw[KS..KS+2] = h2o, p(lev ilay), p(lev ilay+1)
  constexpr int NR = XIN ? KS + 3 : KS;
  auto load_x = [&](int tl, float (&xv)[NR]) {
    const uint32_t s = (uint32_t)tl * 32u + (uint32_t)j;  // loads past the batch return 0
    if constexpr (XIN) {
      const uint32_t nlay = (uint32_t)a.nlay;
      const uint32_t icol = s / nlay, ilay = s - icol * nlay;
      const uint32_t o2 = 4u * s;
      // inputs 2t (lane half 0) and 2t+1 (half 1): one descriptor per array (uniform), each half reading its own
      auto pair = [&](int k0, const float *p0, uint32_t r0, uint32_t f0, const float *p1, uint32_t r1, uint32_t f1) {
        (void)k0;
        const Buf b0(p0, r0), b1(p1, r1);
        const float v0 = b0.ld(h ? kOOB : f0), v1 = b1.ld(h ? f1 : kOOB);
        return h ? v1 : v0;
      };
      xv[0] = pair(0, a.tlay, nb4, o2, a.play, nb4, o2);
      if constexpr (kMlpPackedIn && MODE == MLP_LW_PAIR) {
        // code c of input k: records (c == 3 ? batch : c == 2 ? layers : c) x 4 bytes; offset s*4 (2-D) or ilay*4
        auto gp = [&](int k) {
          const float *p = a.gas.p[k];
          asm volatile("" : "+s"(p));  // loaded where it is used, not held across the tile loop
          return p;
        };
        auto code = [&](int k) { return (a.gcode[k >> 4] >> (2 * (k & 15))) & 3u; };
        auto rec = [&](uint32_t c) { return c == 3u ? nb4 : (c == 2u ? 4u * nlay : 4u * c); };
        auto off = [&](uint32_t c) { return c == 3u ? 4u * s : (c == 2u ? 4u * ilay : 0u); };
        if constexpr (KS > 1) xv[1] = pair(2, gp(2), rec(code(2)), o2, gp(3), rec(code(3)), o2);
#pragma unroll
        for (int t = 2; t < KS; t++) {
          const int k0 = 2 * t, k1 = 2 * t + 1;
          const uint32_t c0 = code(k0), c1 = code(k1);
          xv[t] = pair(k0, gp(k0), rec(c0), off(c0), gp(k1), rec(c1), off(c1));
        }
      } else {
        if constexpr (KS > 1) xv[1] = pair(2, a.gas.p[2], a.grec[2], o2, a.gas.p[3], a.grec[3], o2);
#pragma unroll
        for (int t = 2; t < KS; t++) {
          const int k0 = 2 * t, k1 = 2 * t + 1;
          xv[t] = pair(k0, a.gas.p[k0], a.grec[k0], s * a.gsm[k0] + ilay * a.glm[k0], a.gas.p[k1], a.grec[k1],
                       s * a.gsm[k1] + ilay * a.glm[k1]);
        }
      }
      const Buf bh(a.h2o, nb4), bl(a.plev, 4u * (nlay + 1u) * (uint32_t)a.ncol);
      const uint32_t pl = 4u * (icol * (nlay + 1u) + ilay);
      xv[KS] = bh.ld(o2);
      xv[KS + 1] = bl.ld(s < (uint32_t)a.nbatch ? pl : kOOB);
      const float p1 = bl.ld(s < (uint32_t)a.nbatch ? pl + 4u : kOOB);
      xv[KS + 2] = s < (uint32_t)a.nbatch ? p1 : 1.0f;
    } else {
      const Buf bx(a.x, nb4 * (uint32_t)nx);
#pragma unroll
      for (int t = 0; t < KS; t++) {
        const int k = 2 * t + h;
        xv[t] = bx.ld(k < nx ? 4u * (s * (uint32_t)nx + (uint32_t)k) : kOOB);
      }
    }
  };
  // XIN: compute_nn_inputs (nn_inputs_kernel's expressions) in place, with the scaling constants of network A's image
  // (the host checks that they are the ones it was given); returns col_dry.  No branch: log is formed on every lane
  // and selected, and inputs past nx scale a zero raw value by (0 - 0) / 1.
  auto form_x = [&](float (&xv)[NR], const float *xs) -> float {
    if constexpr (XIN) {
      const float *mn = xs + h * 16, *rg = xs + 32 + h * 16;
      const float lg = ref_logf_nb(xv[0]);
      xv[0] = ((h ? lg : xv[0]) - mn[0]) / rg[0];
      if constexpr (KS > 1) xv[1] = (sqrtf(sqrtf(xv[1])) - mn[1]) / rg[1];
#pragma unroll
      for (int t = 2; t < KS; t++) xv[t] = (xv[t] - mn[t]) / rg[t];
      return col_dry_of(xv[KS], xv[KS + 1], xv[KS + 2]);
    } else {
      return 0.0f;
    }
  };

  float xn[NR];  // the next tile's inputs, loaded before this tile's stores
  load_x(blockIdx.x * nwaves + wave, xn);
  {
    // The weight images into LDS, kStage loads in flight per thread, with the first tile's inputs already on their way
    // (issued above: after the barrier they would wait for the staging).  A load-then-store loop waits out every
    // load's latency in turn: the LW pair's 108 KB took 13 such round trips per block before the first tile.  C3
    // (alone, round 6): LW network -4 %; the first tile's loads first: steps -0.5 % (profiles/r06/mlpstage_*.txt)
    constexpr int kStage = 8;
    const int n4 = (a.imgA_floats + (kPair ? a.imgB_floats : 0)) / 4, nA4 = a.imgA_floats / 4;
    const floatx4 *srcA = (const floatx4 *)a.imgA, *srcB = (const floatx4 *)a.imgB;
    for (int i0 = threadIdx.x; i0 < n4; i0 += kStage * (int)blockDim.x) {
      floatx4 v[kStage];
#pragma unroll
      for (int u = 0; u < kStage; u++) {
        const int i = min(i0 + u * (int)blockDim.x, n4 - 1);  // clamped: every load issues, past-the-end ones unused
        v[u] = i < nA4 ? srcA[i] : srcB[i - nA4];
      }
#pragma unroll
      for (int u = 0; u < kStage; u++) {
        const int i = i0 + u * (int)blockDim.x;
        if (i < n4) lds4[i] = v[u];
      }
    }
  }
  __syncthreads();
  for (int tile = blockIdx.x * nwaves + wave; tile < ntiles; tile += tstride) {
    float xv[NR];
#pragma unroll
    for (int t = 0; t < NR; t++) xv[t] = xn[t];
    load_x(tile + tstride, xn);
    // The weight images are loop-invariant: left visible, their LDS reads are hoisted out of the tile loop and
    // spilled to scratch.  An offset the compiler cannot see through keeps them inside, next to their MFMAs.
    int lds_off = 0;
    asm volatile("" : "+s"(lds_off));
    const float *iA = imgA + lds_off, *iB = imgB + lds_off;
    const float cd_in = form_x(xv, iA + LA.xs);
    float x1[KS];
#pragma unroll
    for (int t = 0; t < KS; t++) x1[t] = xv[t];
    float hA[AN3];
    mlp32_hidden<KS, AH1, AN2, AH2, AN3, NGT>(iA, x1, lane, hA);
    float hB[kPair ? BN3 : 1];
    if constexpr (kPair) mlp32_hidden<KS, BH1, BN2, BH2, BN3, NGT>(iB, x1, lane, hB);
    // wave-uniform by construction; readfirstlane lets the compiler keep the output descriptors in SGPRs (it treats
    // the loop index as divergent and would wrap every store in a waterfall loop)
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane(tile * 32);
    const uint32_t nvalid = min(32u, (uint32_t)a.nbatch - s0);
    float cd;
    if constexpr (XIN) {
      cd = cd_in;
    } else {
      const Buf bc(a.col_dry, nb4);
      cd = bc.ld(4u * (s0 + (uint32_t)j));
    }
    // this tile's rows of the outputs: (nvalid, ngpt) floats.  Lane (c, h) stores rows R(r) = (r&3) + 8(r>>2) + 4h at
    // g-point 32go + c: vo[r] = its byte offset at go = 0 (go adds 128 bytes each), out of range past the batch
    const uint32_t rows = nvalid * (uint32_t)ngpt * 4u;
    const Buf o0(a.out0 + (size_t)s0 * ngpt, rows), o1(a.out1 + (size_t)s0 * ngpt, rows);
    // SW: g (zero) when the caller asked for it; an empty range drops the stores otherwise
    const Buf o2(a.out2 ? a.out2 + (size_t)s0 * ngpt : a.out0, a.out2 ? rows : 0u);
    // the column amounts of rows R(r): sample j's lanes put theirs in the wave's slot, the row registers read them back
    float *slot = cds + wave * 32;
    slot[j] = cd;  // both lane halves write sample j's (equal) value
    __builtin_amdgcn_wave_barrier();
    float cdr[16];
    uint32_t vo[16];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const floatx4 v = *(const floatx4 *)&slot[8 * b + 4 * h];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t R = (uint32_t)(8 * b + 4 * h + i);
        cdr[4 * b + i] = v[i];
        vo[4 * b + i] = R < nvalid ? 4u * (R * (uint32_t)ngpt + (uint32_t)j) : kOOB;
      }
    }
    auto out_tile = [&](int go) {
      const floatx16 yA = mfma_chain_t<AN3>(iA + LA.l3, go, hA, lane);
      floatx16 yB = {};
      if constexpr (kPair) yB = mfma_chain_t<BN3>(iB + LB.l3, go, hB, lane);
      const int g = 32 * go + j;
      const float bA = iA[LA.b3 + g], sdA = iA[LA.sd + g], mnA = iA[LA.mn + g];
      if constexpr (MODE == MLP_SW_PAIR) {
        // tau = tau_abs + tau_ray, ssa = tau_ray / tau, g = 0 (predict_nn_sw_blas with the combine,
        // rrtmgp/kernels/mo_gas_optics_kernels.F90:869-953; mo_gas_optics_rrtmgp.F90:560-567)
        const float bB = iB[LB.b3 + g], sdB = iB[LB.sd + g], mnB = iB[LB.mn + g];
#pragma unroll
        for (int r = 0; r < 16; r++) {
          float ta = sdA * (yA[r] + bA);
          ta = ta + mnA;
          const float vabs = pow8(ta) * cdr[r];
          float tr = sdB * (yB[r] + bB);
          tr = tr + mnB;
          const float vray = pow8(tr) * cdr[r];
          const float tot = vabs + vray, ssa = vray / tot;
          const uint32_t off = vo[r] + 128u * go;
          o0.st(tot, off);
          o1.st(ssa, off);
        }
        // g = 0 only when the caller asked for the array (the fused step and the class layer's NN path pass none):
        // one uniform branch per g-tile instead of a dropped store per element
        if (a.out2) {
#pragma unroll
          for (int r = 0; r < 16; r++) o2.st(0.0f, vo[r] + 128u * go);
        }
      } else if constexpr (kPair) {
        const float bB = iB[LB.b3 + g];
#pragma unroll
        for (int r = 0; r < 16; r++) {
          float t = sdA * (yA[r] + bA);
          t = t + mnA;
          const float p = yB[r] + bB;
          const float tau = pow8(t) * cdr[r], pf = p * p;
          const uint32_t off = vo[r] + 128u * go;
          o0.st(tau, off);
          o1.st(pf, off);
        }
      } else {  // MLP_LW_BOTH: outputs [0, ngpt) -> tau, [ngpt, 2 ngpt) -> pfrac (mo_gas_optics_kernels.F90:754-766);
                // ngpt % 32 == 0, so a g-tile is all tau or all pfrac
        const bool is_tau = 32 * go < ngpt;
        const uint32_t gshift = is_tau ? 0u : 4u * (uint32_t)ngpt;
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const float y = yA[r] + bA;
          float t = sdA * y;
          t = t + mnA;
          const float tau = pow8(t) * cdr[r], pf = y * y;
          const uint32_t off = vo[r] + 128u * go - gshift;
          o0.st(tau, is_tau ? off : kOOB);
          o1.st(pf, is_tau ? kOOB : off);
        }
      }
    };
#pragma unroll 1
    for (int go = 0; go < NGT; go++) out_tile(go);
  }
}

constexpr int kOccDevices = 64;

template <int KS, int AH1, int AN2, int AH2, int AN3, int BH1, int BN2, int BH2, int BN3, int NGT, int MODE, bool XIN,
          int NT = kMlp32Threads, int WPE = 1>
static int launch32(rrtmgpnn_context *ctx, Mlp32Args &a)
{
  auto kern = mlp32_kernel<KS, AH1, AN2, AH2, AN3, BH1, BN2, BH2, BN3, NGT, MODE, XIN, NT, WPE>;
  const size_t lds = sizeof(float) * ((size_t)(a.imgA_floats + (MODE != MLP_LW_BOTH ? a.imgB_floats : 0)) +
                                      32 * (NT / 64));
  if (lds > 160 * 1024) return RRTMGPNN_ERR_UNSUPPORTED;
  if (lds > 64 * 1024)
    if (int rc = raise_lds_limit((const void *)kern)) return rc;
  const long long ntiles = ((long long)a.nbatch + 31) / 32;
  const int wpb = NT / 64;
  int per_cu = std::min(std::max(1, (int)((160 * 1024) / std::max<size_t>(lds, 1))), 2048 / NT);
  const long long want = (ntiles + wpb - 1) / wpb;
  // Blocks a CU actually holds (registers included).  When the tiles fill less than two rounds of resident blocks, a
  // grid of one round strides them and loads each weight image once per CU, instead of a partial second round that
  // loads it again for little work (the SW pair at C3: 184 VGPRs, one 8-wave block per CU, 422 blocks: step -1 %).
  // With many rounds the blocks' turnover lets the overlapped LW chain share the CUs (C4: one round was 1 % slower).
  // Cached per (instance, device): contexts of several host threads launch concurrently, and a function's occupancy
  // is a property of the device it runs on.
  static std::atomic<int> occ_cache[kOccDevices];
  int occ = -1;
  if (ctx->device >= 0 && ctx->device < kOccDevices) {
    occ = occ_cache[ctx->device].load(std::memory_order_relaxed);
    if (!occ) {
      int nb = 0;
      occ = (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void *)kern, NT, lds) == hipSuccess && nb > 0)
                ? nb : -1;
      occ_cache[ctx->device].store(occ, std::memory_order_relaxed);
    }
  }
  if (occ > 0 && want <= 2LL * occ * ctx->num_cus) per_cu = std::min(per_cu, occ);
  // rrtmgpnn_context_set_mlp_max_cus: at most that many CUs' worth of blocks (the waves stride the tiles)
  const int cus = ctx->mlp_max_cus > 0 ? std::min(ctx->mlp_max_cus, ctx->num_cus) : ctx->num_cus;
  const long long grid = std::max<long long>(1, std::min<long long>(want, (long long)cus * per_cu));
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), lds, ctx->stream, a);
  RRTMGPNN_LAUNCH_CHECK("mlp32_kernel");
  return RRTMGPNN_OK;
}

static bool shape32(const rrtmgpnn_network *n, int KS, int HT1, int N2, int HT2, int N3, int NGT)
{
  return n && n->d_packed32 && n->s32[0] == KS && n->s32[1] == HT1 && n->s32[2] == N2 && n->s32[3] == HT2 &&
         n->s32[4] == N3 && n->s32[5] == NGT;
}

// The LW modes on the 32x32x2 kernel for the shipped shapes with the shipped activations (softsign, softsign,
// linear); RRTMGPNN_ERR_UNSUPPORTED (no error set) otherwise, and the caller runs the 16x16x4 kernel.
int launch_mlp32(rrtmgpnn_context *ctx, MlpMode mode, const rrtmgpnn_network *A, const rrtmgpnn_network *B,
                 long long nbatch, int ngpt, const float *x, const float *col_dry, float *out0, float *out1,
                 float *out2, const MlpInputs *in)
{
  const int kmode = ctx->mlp_kernel >= 0 ? ctx->mlp_kernel : g_mlp_kernel_default;
  if (kmode == 1 || (mode != MLP_LW_PAIR && mode != MLP_LW_BOTH && mode != MLP_SW_PAIR))
    return RRTMGPNN_ERR_UNSUPPORTED;
  const bool pair = mode != MLP_LW_BOTH;
  auto std_acts = [](const rrtmgpnn_network *n) {
    return n->act[0] == RRTMGPNN_ACT_SOFTSIGN && n->act[1] == RRTMGPNN_ACT_SOFTSIGN && n->act[2] == RRTMGPNN_ACT_LINEAR;
  };
  if (!A || !std_acts(A) || (pair && (!B || !std_acts(B)))) return RRTMGPNN_ERR_UNSUPPORTED;
  Mlp32Args a{};
  a.x = x; a.col_dry = col_dry; a.out0 = out0; a.out1 = out1; a.out2 = out2;
  a.imgA = A->d_packed32; a.imgA_floats = A->packed32_floats;
  a.imgB = pair ? B->d_packed32 : nullptr;
  a.imgB_floats = pair ? B->packed32_floats : 0;
  a.nx = A->dims[0]; a.ngpt = ngpt;
  if (in) {
    a.play = in->play; a.tlay = in->tlay; a.plev = in->plev; a.h2o = in->h2o; a.nlay = in->nlay;
    a.gas = in->gas;
  }
  a.ncol = in && in->nlay > 0 ? (int)(nbatch / in->nlay) : 0;
  // 16-byte stores, and every descriptor's range below kOOB
  auto al16 = [](const float *p) { return ((uintptr_t)p & 15) == 0; };
  if (ngpt % 32 != 0 || !al16(out0) || !out1 || !al16(out1)) return RRTMGPNN_ERR_UNSUPPORTED;
  if (A->s32[5] * 32 != (pair ? ngpt : 2 * ngpt) || (pair && B->s32[5] != A->s32[5]))
    return RRTMGPNN_ERR_UNSUPPORTED;  // full g-tiles
  if ((unsigned long long)nbatch * 4ull * (unsigned long long)std::max(1, A->dims[0]) >= kMaxRecords ||
      32ull * 4ull * (unsigned long long)ngpt >= kMaxRecords)
    return RRTMGPNN_ERR_UNSUPPORTED;
  if (in && (unsigned long long)(nbatch / std::max(1, in->nlay) + 1) * (in->nlay + 1) * 4ull >= kMaxRecords)
    return RRTMGPNN_ERR_UNSUPPORTED;
  a.nbatch = (int)nbatch;
  const bool xin = in != nullptr;
  if (in)  // the kernel scales with A's image: it must hold the constants the caller passed
    for (int k = 0; k < a.nx; k++)
      if (k >= (int)A->in_min.size() || k >= (int)A->in_max.size() || A->in_min[k] != in->mn[k] ||
          A->in_max[k] != in->mx[k])
        return RRTMGPNN_ERR_UNSUPPORTED;
  if (in)
    for (int k = 0; k < kMaxInputs; k++) {
      const int nd = in->gas.nd[k];
      const bool on = k < a.nx && in->gas.p[k];
      a.gsm[k] = nd == 2 ? 4u : 0u;
      a.glm[k] = nd == 1 ? 4u : 0u;
      a.grec[k] = !on ? 0u : (nd == 2 ? 4u * (uint32_t)nbatch : (nd == 1 ? 4u * (uint32_t)in->nlay : 4u));
      const uint32_t code = !on ? 0u : (nd == 2 ? 3u : (nd == 1 ? 2u : 1u));
      a.gcode[k >> 4] |= code << (2 * (k & 15));
    }
  if (mode == MLP_LW_PAIR && shape32(A, 9, 2, 29, 2, 29, 8) && shape32(B, 9, 1, 8, 1, 8, 8)) {
    // the shipped g256 pair: absorption 18-58-58-256, Planck fraction 18-16-16-256
    if (xin) return launch32<9, 2, 29, 2, 29, 1, 8, 1, 8, 8, MLP_LW_PAIR, true>(ctx, a);
    return launch32<9, 2, 29, 2, 29, 1, 8, 1, 8, 8, MLP_LW_PAIR, false>(ctx, a);
  }
  if (mode == MLP_SW_PAIR && shape32(A, 4, 1, 8, 1, 8, 7) && shape32(B, 4, 1, 8, 1, 8, 7)) {
    // the shipped g224 pair: absorption and Rayleigh 7-16-16-224
    if (xin) return launch32<4, 1, 8, 1, 8, 1, 8, 1, 8, 7, MLP_SW_PAIR, true, kSwNT, kSwWPE>(ctx, a);
    return launch32<4, 1, 8, 1, 8, 1, 8, 1, 8, 7, MLP_SW_PAIR, false, kSwNT, kSwWPE>(ctx, a);
  }
  if (mode == MLP_LW_BOTH && !xin && shape32(A, 9, 2, 32, 2, 32, 8)) {
    // the shipped g128 single model: 18-64-64-256
    return launch32<9, 2, 32, 2, 32, 1, 1, 1, 1, 8, MLP_LW_BOTH, false>(ctx, a);
  }
  return RRTMGPNN_ERR_UNSUPPORTED;
}

}  // namespace rrtmgpnn
