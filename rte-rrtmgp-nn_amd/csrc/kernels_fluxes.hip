// kernels_fluxes.hip -- post-processing of the broadband fluxes.
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

namespace rrtmgpnn {

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
