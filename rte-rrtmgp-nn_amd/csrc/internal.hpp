// internal.hpp -- shared declarations of the rrtmgpnn runtime (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/rrtmgpnn.h"

namespace rrtmgpnn {

void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define RRTMGPNN_HIP(call)                                                                           \
  do {                                                                                               \
    hipError_t e_ = (call);                                                                          \
    if (e_ != hipSuccess)                                                                            \
      return ::rrtmgpnn::fail(RRTMGPNN_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Launch-error check after a kernel launch.
#define RRTMGPNN_LAUNCH_CHECK(name)                                                                  \
  do {                                                                                               \
    hipError_t e_ = hipGetLastError();                                                               \
    if (e_ != hipSuccess)                                                                            \
      return ::rrtmgpnn::fail(RRTMGPNN_ERR_DEVICE, std::string(name) + " launch: " + hipGetErrorString(e_)); \
  } while (0)

constexpr int kMaxLayers = 7;   // network layers (excluding input)
constexpr int kMaxInputs = 32;  // NN input features
constexpr int kMaxBands = 64;
extern int g_sw_kernel_default;  // rrtmgpnn_context_set_sw_kernel(NULL, mode)
extern int g_mlp_kernel_default;  // rrtmgpnn_context_set_mlp_kernel(NULL, mode)
// Raise a kernel's dynamic-LDS limit to 160 KiB on the current device, once per (kernel, device): a function
// attribute is per device, so a second GPU of the same process gets its own call.  Thread-safe; after the first
// call for a (kernel, device) pair it makes no HIP call (hipGraph captures stay attribute-free).
int raise_lds_limit(const void *kernel);

}  // namespace rrtmgpnn

// Device workspace owned by a context: grown on demand, never shrunk, so steady-state calls
// (and hipGraph capture of them) perform no allocation.  A call made while the context's stream is being
// captured pins the buffer (ws_pinned): the graph holds its address, so a later call that would grow it fails
// with RRTMGPNN_ERR_ARGUMENT instead of freeing memory the graph still writes (rrtmgpnn_context_unpin_workspace
// once the graph is destroyed; or give the graph a context of its own).
struct rrtmgpnn_context {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int num_cus = 256;
  int sw_kernel = -1;  // SW two-stream kernel: 0 by ngpt, 1 / 2 g-points per lane, -1 the library default
  int mlp_max_cus = 0;  // rrtmgpnn_context_set_mlp_max_cus: CUs' worth of network blocks, 0 = all
  int mlp_kernel = -1;  // LW network tiling: 0 32x32x2 where instantiated, 1 16x16x4, -1 the library default
  // Per-call solver extras, set by the *_gpt entry points for the duration of one call (rte_lw's lw_Ds and
  // ty_fluxes_flexible's g-point outputs, (ngpt, nlay+1, ncol) each); the other entries leave them null.
  struct SolverExtras {
    const float *lw_Ds = nullptr;
    float *gpt_up = nullptr, *gpt_dn = nullptr, *gpt_dir = nullptr;
  } extras;
  void *ws = nullptr;
  size_t ws_bytes = 0;
  bool ws_pinned = false;
  int workspace(size_t bytes, void **out);
  // device data environment (present.cpp): a caching pool of device buffers and the host -> device map
  struct Present {
    void *dev = nullptr;
    size_t bytes = 0;
    int state = 0;  // 0 host newer, 1 both current, 2 device newer
    uint64_t gen = 0;  // the host array's process-wide generation this copy was made at (present.cpp)
  };
  std::multimap<size_t, void *> pool_free;      // capacity -> buffer
  std::unordered_map<void *, size_t> pool_live;  // buffer -> capacity
  std::unordered_map<const void *, Present> present;
  int pool_get(size_t bytes, void **out);
  void pool_put(void *p);
  void pool_clear();
  // pinned staging ring for host <-> device copies of pageable host arrays: the host side is one memcpy into the
  // ring, the DMA runs asynchronously on the stream; the ring is reused after sync(), which also completes the
  // device-to-host copies queued in pending_d2h
  void *pin = nullptr;
  size_t pin_cap = 0, pin_head = 0;
  struct PendingD2H {
    void *dst;
    const void *src;
    size_t bytes;
  };
  std::vector<PendingD2H> pending_d2h;
  int h2d(void *dst, const void *host, size_t bytes);
  int d2h(void *host, const void *dev, size_t bytes);
  int sync();
};

// A network: host copy of the model + device images.
//   d_raw    : plain weights (n_in, n_out) per layer + biases (generic forward path)
//   d_packed : MFMA operand image for the fused 3-layer kernel (see kernels_nn.hip)
struct rrtmgpnn_network {
  int device = 0;
  int nlayers = 0;
  int dims[rrtmgpnn::kMaxLayers + 1] = {0};
  int act[rrtmgpnn::kMaxLayers] = {0};
  std::vector<std::vector<float>> w, b;
  std::vector<float> in_min, in_max, out_mean, out_std;
  std::vector<std::string> input_names;
  float *d_raw = nullptr;
  size_t raw_w_off[rrtmgpnn::kMaxLayers] = {0}, raw_b_off[rrtmgpnn::kMaxLayers] = {0};
  // packed MFMA image (3-layer networks only)
  float *d_packed = nullptr;
  int packed_floats = 0;
  int k1s = 0, h1t = 0, h2t = 0, ngt = 0;
  int off_l1 = 0, off_l2 = 0, off_l3 = 0, off_b1 = 0, off_b2 = 0, off_b3 = 0, off_std = 0, off_mean = 0;
  // packed image of the 32x32x2 kernel (kernels_nn32.hip; 3-layer networks with hidden widths <= 64):
  // s32 = KS, HT1, N2, HT2, N3, NGT
  float *d_packed32 = nullptr;
  int packed32_floats = 0;
  int s32[6] = {0};
  bool has_out_scaling() const { return !out_mean.empty(); }
};

// Cloud optics (extensions/cloud_optics/mo_cloud_optics.F90 ty_cloud_optics): one device buffer holding
// the LUT or Pade tables in the file's Fortran layout; off[] are float offsets into it
//   LUT : ext/ssa/asy liquid (nsize_liq, nband) [0..2], ice (nsize_ice, nband, nrghice) [3..5]
//   Pade: ext/ssa/asy liquid (nband, nsizereg, ncoef) [0..2], ice (..., nrghice) [3..5], size-regime
//         bounds [6..11]
struct rrtmgpnn_cloud_optics {
  int device = 0;
  int lut_mode = 1;
  int nband = 0, nsize_liq = 0, nsize_ice = 0, nrghice = 0, nsizereg = 0, ncoef_ext = 0, ncoef_ssa = 0;
  int icergh = 1;
  float radliq_lwr = 0, radliq_upr = 0, radice_lwr = 0, radice_upr = 0, liq_step = 0, ice_step = 0;
  std::vector<float> band_lims_wvn;
  float *d_tab = nullptr;
  size_t off[12] = {0};
};

namespace rrtmgpnn {
// kernels_clouds.hip
struct BandArgs;
int launch_cloud_optics(rrtmgpnn_context *ctx, const rrtmgpnn_cloud_optics *co, int ncol, int nlay, const float *clwp,
                        const float *ciwp, const float *reliq, const float *reice, float *tau, float *ssa, float *g);
int launch_increment_bybnd(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, const BandArgs *bands, float *tau1,
                           float *ssa1, float *g1, const float *tau2, const float *ssa2, const float *g2);
int launch_heating_rate(rrtmgpnn_context *ctx, int ncol, int nlay, int k_day, float c0, float c1, const float *up,
                        const float *dn, const float *plev, float *hr);
int launch_sw_boundary(rrtmgpnn_context *ctx, int ngpt, int ncol, const float *solar_source, const float *tsi,
                       const float *sfc_alb, const float *sza, float *toa, float *alb, float *mu0);
// the RFMIP driver's SW boundary conditions as inputs of a solver launch (rrtmgpnn_sw_solver_2stream_rfmip): the
// checkpointed solver forms them in its prologue; the other solver kernels get them from launch_sw_boundary, into
// toa / alb / mu0 (scratch)
struct SwBc {
  const float *solar_source, *tsi, *sfc_alb, *sza;
  float *toa, *alb, *mu0;
};
// the device-side part: the inputs and the driver's two constants (deg_to_rad, the usecol bound)
struct SwBcDev {
  const float *solar_source, *tsi, *sfc_alb, *sza;
  float deg_to_rad, sza_max;
};
SwBcDev sw_boundary_device(const SwBc *bc);
constexpr int kSwBoundaryMaxG = 1024;
int launch_delta_scale(rrtmgpnn_context *ctx, long long n, float *tau, float *ssa, float *g, const float *fwd);
// kernels_nn.hip
struct GasArgs {
  const float *p[kMaxInputs];
  int nd[kMaxInputs];
};
int launch_nn_inputs(rrtmgpnn_context *ctx, int ncol, int nlay, int nx, const float *play, const float *tlay,
                     const GasArgs &gas, const float *in_min_max /*host 2*nx*/, float *out);
int launch_col_dry(rrtmgpnn_context *ctx, int ncol, int nlay, const float *h2o, const float *plev, float *col_dry);
int launch_tlev(rrtmgpnn_context *ctx, int ncol, int nlay, const float *play, const float *plev, const float *tlay,
                float *tlev);
enum MlpMode { MLP_PLAIN = 0, MLP_LW_PAIR = 1, MLP_SW_PAIR = 2, MLP_SW_ABS = 3, MLP_LW_BOTH = 4 };
// state the MLP kernel forms its inputs from (fused gas optics): compute_nn_inputs + get_col_dry in-kernel
struct MlpInputs {
  const float *play, *tlay, *plev, *h2o;
  int nlay;
  GasArgs gas;
  float mn[kMaxInputs], mx[kMaxInputs];
};
int launch_mlp(rrtmgpnn_context *ctx, MlpMode mode, const rrtmgpnn_network *A, const rrtmgpnn_network *B,
               long long nbatch, int ngpt, const float *x, const float *col_dry, float *out0, float *out1,
               float *out2, const MlpInputs *in = nullptr);
int launch_mlp_generic(rrtmgpnn_context *ctx, const rrtmgpnn_network *net, long long nbatch, const float *x,
                       float *out);
int pack_network(rrtmgpnn_network *net);
// kernels_nn32.hip: the LW pair, LW both and SW pair modes on v_mfma_f32_32x32x2_f32; RRTMGPNN_ERR_UNSUPPORTED (no error set) when no instance
// exists for the networks (launch_mlp then runs the 16x16x4 kernel)
int pack_network32(rrtmgpnn_network *net);
int launch_mlp32(rrtmgpnn_context *ctx, MlpMode mode, const rrtmgpnn_network *A, const rrtmgpnn_network *B,
                 long long nbatch, int ngpt, const float *x, const float *col_dry, float *out0, float *out1,
                 float *out2, const MlpInputs *in);
// kernels_rte.hip
struct BandArgs {
  int lims[2 * kMaxBands];
  int nbnd;
};
int launch_planck_source(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ntemp, const float *tlay,
                         const float *tlev, const float *tsfc, int sfc_lay, const BandArgs &bands,
                         float temp_ref_min, float totplnk_delta, const float *totplnk, float *sfc_source,
                         float *sfc_source_Jac, float *pfrac, float *lev_source);
int launch_lw_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus, const float *Ds,
                     const float *wts, const float *inc_flux, const float *tau, const float *lay_source,
                     const float *lev_source, const float *sfc_emis, const float *sfc_source, float *flux_up,
                     float *flux_dn);
int launch_lw_noscat_planck(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                            const float *Ds, const float *wts, const float *inc_flux, const float *tau,
                            const float *pfrac, int ntemp, const float *tlay, const float *tlev, const float *tsfc,
                            int sfc_lay, const BandArgs &bands, float temp_ref_min, float totplnk_delta,
                            const float *totplnk, bool emis_by_band, const float *sfc_emis, const float *tau_bnd,
                            float *flux_up, float *flux_dn);
// bands != nullptr: atmosphere incremented by the band-resolved 2str set (tau, ssa, g)_bnd in-kernel
int launch_sw_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                      const float *inc_flux_dif, const float *tau, const float *ssa, const float *g,
                      const float *mu0, const float *alb_dir, const float *alb_dif, const BandArgs *bands,
                      const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, float *flux_up,
                      float *flux_dn, float *flux_dir, const SwBc *bc = nullptr);
// kernels_sw_x2.hip (called by launch_sw_2stream for even ngpt; ws sized by it)
size_t sw_2stream_x2_layer_planes(bool inc);
int launch_sw_2stream_x2(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                         const float *inc_flux_dif, const float *tau, const float *ssa, const float *g,
                         const float *mu0, const float *alb_dir, const float *alb_dif, const BandArgs *bands,
                         const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, void *ws, float *flux_up,
                         float *flux_dn, float *flux_dir);
int launch_sw_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                     const float *tau, const float *mu0, float *flux_dir);
// kernels_sw_ck.hip (checkpointed passes; called by launch_sw_2stream for even ngpt in mode 3)
// the checkpointed SW kernel's small-grid instance applies (clear sky, g = 0, no g-point outputs, the grid in one round)
bool sw_ck_small(const rrtmgpnn_context *ctx, int ngpt, int ncol, bool has_g, bool inc, bool gpt);
// planes: the large-grid instances' workspace planes (kCkTnNN, kCkTnInc, ...); false after that allocation failed
size_t sw_2stream_ck_ws_floats(int ngpt, int nlay, int ncol, bool small, bool inc, bool nn, bool planes = true);
int launch_sw_2stream_ck(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                         const float *inc_flux_dif, const float *tau, const float *ssa, const float *g,
                         const float *mu0, const float *alb_dir, const float *alb_dif, const BandArgs *bands,
                         const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, void *ws, float *flux_up,
                         float *flux_dn, float *flux_dir, bool planes = true, const SwBcDev *bc = nullptr);
// kernels_lw_scat.hip
int launch_lw_rescl(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus, const float *Ds,
                    const float *wts, const float *inc_flux, const float *tau, const float *ssa, const float *g,
                    const float *lay_source, const float *lev_source, const float *sfc_emis, const float *sfc_source,
                    float *flux_up, float *flux_dn);
int launch_lw_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                      const float *tau, const float *ssa, const float *g, const float *lev_source,
                      const float *sfc_emis, const float *sfc_source, float *flux_up, float *flux_dn);
int launch_expand(rrtmgpnn_context *ctx, int nband, int ngpt, int ncol, const BandArgs &bands, const float *in,
                  float *out);
}  // namespace rrtmgpnn
