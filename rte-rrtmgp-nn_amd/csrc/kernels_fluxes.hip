// kernels_fluxes.hip -- the RFMIP driver's per-block SW boundary conditions and the post-processing of the broadband
// fluxes.
//
//  * sw_boundary_kernel  : the per-block work of examples/rfmip-clear-sky/rrtmgp_rfmip_sw.F90 between gas_optics and
//                          rte_sw (:403-434), with gas_optics_ext's toa_src(igpt, icol) = solar_source(igpt)
//                          (rrtmgp/mo_gas_optics_rrtmgp.F90:594-599) in front of it: per column def_tsi = the sum of
//                          toa_src over g-points in g order, toa = toa_src * tsi / def_tsi, the spectrally constant
//                          surface albedo expanded to every g-point, mu0 = merge(cos(sza * deg_to_rad), 1, usecol)
//                          with usecol = sza < 90 - 2 spacing(90) (rrtmgp_rfmip_sw.F90:236-238) and glibc's cosf
//                          (libm_ref.hpp ref_cosf).  A block holds kBcCols columns; def_tsi in the reference's
//                          sequential order, then the block writes the (ngpt, kBcCols) slabs.  The benchmarked step
//                          forms the same values in the checkpointed SW solver's prologue instead
//                          (rrtmgpnn_sw_solver_2stream_rfmip, kernels_sw_ck.hip); this kernel serves the class layer
//                          and the other SW solver kernels.
//
//  * heating_rate_kernel : layer heating rates from the level fluxes and pressures, in the fork's (nlay+1, ncol)
//                          level-fastest flux layout.  Two forms, both term by term:
//      K/s   (extensions/mo_heating_rates.F90:48-52, compute_heating_rate):
//              ((up(l+1) - up(l) - dn(l+1) + dn(l)) * grav) / (cp_dry * (p(l+1) - p(l)))
//      K/day (examples/rrtmgp-nn-training/rrtmgp_lw_eval_nn_rfmip.F90:624-653, calc_heating_rate, the tolerance
//             report's form): scaling * ((dn - up)(l+1) - (dn - up)(l)) / (p(l+1) - p(l)),
//             scaling = -(24 * 3600 * grav / 1004) formed in fp32 on the host
//
// Elementwise and HBM-bound: one thread per (layer, column), layer fastest, so a wave reads 65 contiguous levels of
// each array and writes 64 contiguous layers.  -ffp-contract=off keeps the reference's roundings.
#include "internal.hpp"
#include "libm_ref.hpp"

namespace rrtmgpnn {

constexpr int kBcCols = 16;

// toa_src(igpt, icol) = solar_source(igpt) for every column (gas_optics_ext), so every column's def_tsi is the same
// sequential sum: one lane forms it per block, over the source staged in LDS (a sum over dependent global loads took
// 18 us at C3)
__global__ void __launch_bounds__(256) sw_boundary_kernel(int ngpt, int ncol, const float *__restrict__ solar_source,
                                                          const float *__restrict__ tsi,
                                                          const float *__restrict__ sfc_alb,
                                                          const float *__restrict__ sza, float deg_to_rad,
                                                          float sza_max, float *__restrict__ toa,
                                                          float *__restrict__ alb, float *__restrict__ mu0)
{
  __shared__ float src[kSwBoundaryMaxG];
  __shared__ float def_tsi;
  const int c0 = blockIdx.x * kBcCols, t = threadIdx.x;
  for (int g = t; g < ngpt; g += blockDim.x) src[g] = solar_source[g];
  __syncthreads();
  if (t == 0) {
    float s = 0.0f;  // def_tsi_s = def_tsi_s + toa_flux(igpt, icol), igpt = 1..ngpt, in that order
    int g = 0;
    for (; g + 8 <= ngpt; g += 8) {  // eight LDS reads in flight, then the eight dependent adds
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = src[g + j];
#pragma unroll
      for (int j = 0; j < 8; j++) s = s + v[j];
    }
    for (; g < ngpt; g++) s = s + src[g];
    def_tsi = s;
  }
  if (t < kBcCols && c0 + t < ncol) {
    const float z = sza[c0 + t];
    mu0[c0 + t] = z < sza_max ? ref_cosf(z * deg_to_rad) : 1.0f;
  }
  __syncthreads();
  const float d = def_tsi;
  const int nc = min(kBcCols, ncol - c0);
  for (int i = t; i < nc * ngpt; i += blockDim.x) {
    const int c = i / ngpt, g = i - c * ngpt;
    const size_t k = (size_t)(c0 + c) * ngpt + g;
    toa[k] = src[g] * tsi[c0 + c] / d;
    alb[k] = sfc_alb[c0 + c];
  }
}

SwBcDev sw_boundary_device(const SwBc *bc)
{
  // deg_to_rad = acos(-1._wp) / 180._wp in working precision (rrtmgp_rfmip_sw.F90:106); the usecol bound
  // 90 - 2 spacing(90) = 90 - 2^-16 (spacing(90.) = 2^-17 in fp32)
  volatile float pi = 3.14159265358979323846f;
  return SwBcDev{bc->solar_source, bc->tsi, bc->sfc_alb, bc->sza, pi / 180.0f, 90.0f - 2.0f * 0x1p-17f};
}

int launch_sw_boundary(rrtmgpnn_context *ctx, int ngpt, int ncol, const float *solar_source, const float *tsi,
                       const float *sfc_alb, const float *sza, float *toa, float *alb, float *mu0)
{
  if (ncol == 0) return RRTMGPNN_OK;
  if (ngpt > kSwBoundaryMaxG) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw_boundary_rfmip: ngpt > 1024");
  const SwBc bc{solar_source, tsi, sfc_alb, sza, toa, alb, mu0};
  const SwBcDev d = sw_boundary_device(&bc);
  hipLaunchKernelGGL(sw_boundary_kernel, dim3((unsigned)((ncol + kBcCols - 1) / kBcCols)), dim3(256), 0, ctx->stream,
                     ngpt, ncol, solar_source, tsi, sfc_alb, sza, d.deg_to_rad, d.sza_max, toa, alb, mu0);
  RRTMGPNN_LAUNCH_CHECK("sw_boundary_kernel");
  return RRTMGPNN_OK;
}

template <bool kDay>
__global__ void __launch_bounds__(256) heating_rate_kernel(long long n, int nlay, float c0, float c1,
                                                          const float *__restrict__ up, const float *__restrict__ dn,
                                                          const float *__restrict__ plev, float *__restrict__ hr)
{
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long col = i / nlay;
  const int l = (int)(i - col * nlay);
  const long long k = col * (nlay + 1) + l;  // levels l and l + 1 of this column
  const float dp = plev[k + 1] - plev[k];
  if constexpr (kDay) {
    const float dF = (dn[k + 1] - up[k + 1]) - (dn[k] - up[k]);
    hr[i] = c0 * dF / dp;  // c0 = scaling
  } else {
    hr[i] = (up[k + 1] - up[k] - dn[k + 1] + dn[k]) * c0 / (c1 * dp);  // c0 = grav, c1 = cp_dry
  }
}

int launch_heating_rate(rrtmgpnn_context *ctx, int ncol, int nlay, int k_day, float c0, float c1, const float *up,
                        const float *dn, const float *plev, float *hr)
{
  const long long n = (long long)ncol * nlay;
  if (n == 0) return RRTMGPNN_OK;
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (k_day)
    hipLaunchKernelGGL(heating_rate_kernel<true>, grid, block, 0, ctx->stream, n, nlay, c0, c1, up, dn, plev, hr);
  else
    hipLaunchKernelGGL(heating_rate_kernel<false>, grid, block, 0, ctx->stream, n, nlay, c0, c1, up, dn, plev, hr);
  RRTMGPNN_LAUNCH_CHECK("heating_rate_kernel");
  return RRTMGPNN_OK;
}

}  // namespace rrtmgpnn
