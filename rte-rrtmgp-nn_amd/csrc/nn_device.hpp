// nn_device.hpp -- device expressions shared by the MLP kernels (kernels_nn.hip: 16x16x4 tiles, kernels_nn32.hip:
// 32x32x2 tiles), so that both give the same bits: the column amount of get_col_dry, the output scaling's 8th power,
// softsign, and the input scaling of compute_nn_inputs.
#pragma once
#include "internal.hpp"
#include "libm_ref.hpp"

namespace rrtmgpnn {

struct NnInArgs {
  float mn[kMaxInputs];
  float mx[kMaxInputs];
};

// get_col_dry (rrtmgp/mo_gas_optics_rrtmgp.F90:1662-1707) for one (layer, column): h2o vmr v and the layer's two
// level pressures
__device__ __forceinline__ float col_dry_of(float v, float p_a, float p_b)
{
  const float m_dry = 0.028964f, m_h2o = 0.018016f, avogad = 6.02214076e23f, grav = 9.80665f;
  float delta_plev = fabsf(p_a - p_b);
  float fact = 1.0f / (1.0f + v);
  float m_air = (m_dry + m_h2o * v) * fact;
  return 10.0f * delta_plev * avogad * fact / (1000.0f * m_air * 100.0f * grav);
}

// (std*y + mean)^8 of output_sgemm_tau (neural/mod_network_rrtmgp.F90:309-312) as three squarings
__device__ __forceinline__ float pow8(float t)
{
  float t2 = t * t, t4 = t2 * t2;
  return t4 * t4;
}

// softsign (neural/mod_activation.F90:107-128) with libm_ref.hpp div_softsign (reciprocal and two residual
// corrections), equal to the IEEE quotient x / (|x| + 1) for every |x| < 2^126, checked exhaustively on the GPU
__device__ __forceinline__ float softsign(float x) { return div_softsign(x, fabsf(x) + 1.0f); }

}  // namespace rrtmgpnn
