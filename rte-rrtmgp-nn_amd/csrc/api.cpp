// api.cpp -- the C ABI (include/rrtmgpnn.h): contexts, networks, argument checking and dispatch.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "datafile.hpp"
#include "internal.hpp"

namespace rrtmgpnn {

static thread_local std::string g_last_error;
int g_sw_kernel_default = 0;
int g_mlp_kernel_default = 0;

void set_error(const std::string &msg) { g_last_error = msg; }

int fail(int code, const std::string &msg)
{
  g_last_error = msg;
  return code;
}

int raise_lds_limit(const void *kernel)
{
  static std::mutex mu;
  static std::set<std::pair<const void *, int>> done;
  int dev = 0;
  RRTMGPNN_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  if (done.count({kernel, dev})) return RRTMGPNN_OK;
  RRTMGPNN_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  done.insert({kernel, dev});
  return RRTMGPNN_OK;
}

// activation names of neural/mod_layer.F90:64-121 (set_activation) -> the codes of network_create
static int activation_code(std::string n)
{
  while (!n.empty() && (n.back() == ' ' || n.back() == '\0')) n.pop_back();
  size_t i = n.find_first_not_of(' ');
  n = i == std::string::npos ? "" : n.substr(i);
  static const char *names[] = {"linear", "softsign", "relu", "sigmoid", "hard_sigmoid", "tanh", "gaussian"};
  for (int k = 0; k < 7; k++)
    if (n == names[k]) return k;
  return -1;
}

static int finalize_network(rrtmgpnn_network *net)
{
  // raw device image: all weights then all biases
  size_t total = 0;
  for (int n = 0; n < net->nlayers; n++) {
    net->raw_w_off[n] = total;
    total += net->w[n].size();
  }
  for (int n = 0; n < net->nlayers; n++) {
    net->raw_b_off[n] = total;
    total += net->b[n].size();
  }
  std::vector<float> raw(total);
  for (int n = 0; n < net->nlayers; n++) {
    std::memcpy(raw.data() + net->raw_w_off[n], net->w[n].data(), net->w[n].size() * 4);
    std::memcpy(raw.data() + net->raw_b_off[n], net->b[n].data(), net->b[n].size() * 4);
  }
  RRTMGPNN_HIP(hipSetDevice(net->device));
  RRTMGPNN_HIP(hipMalloc(&net->d_raw, total * 4));
  RRTMGPNN_HIP(hipMemcpy(net->d_raw, raw.data(), total * 4, hipMemcpyHostToDevice));
  if (int rc = pack_network(net)) return rc;
  return pack_network32(net);
}

static int check_ctx(rrtmgpnn_context *ctx)
{
  if (!ctx) return fail(RRTMGPNN_ERR_ARGUMENT, "null context");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return fail(RRTMGPNN_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return RRTMGPNN_OK;
}

static int band_args(int nbnd, const int *lims, int ngpt, BandArgs &b)
{
  if (nbnd < 1 || nbnd > kMaxBands || !lims) return fail(RRTMGPNN_ERR_ARGUMENT, "band limits: need 1..64 bands");
  b.nbnd = nbnd;
  for (int i = 0; i < nbnd; i++) {
    b.lims[2 * i] = lims[2 * i];
    b.lims[2 * i + 1] = lims[2 * i + 1];
    if (lims[2 * i] < 1 || lims[2 * i + 1] > ngpt || lims[2 * i] > lims[2 * i + 1])
      return fail(RRTMGPNN_ERR_ARGUMENT, "band limits out of range [1, ngpt]");
  }
  return RRTMGPNN_OK;
}

// the fused increments give every g-point a band: refuse band limits that leave one out
static int bands_cover(const BandArgs &b, int ngpt)
{
  for (int g = 1; g <= ngpt; g++) {
    bool in = false;
    for (int i = 0; i < b.nbnd && !in; i++) in = g >= b.lims[2 * i] && g <= b.lims[2 * i + 1];
    if (!in) return fail(RRTMGPNN_ERR_ARGUMENT, "band limits leave g-points outside every band");
  }
  return RRTMGPNN_OK;
}

}  // namespace rrtmgpnn

using namespace rrtmgpnn;

int rrtmgpnn_context::workspace(size_t bytes, void **out)
{
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) == hipSuccess && cap == hipStreamCaptureStatusActive) {
    if (bytes > ws_bytes)
      return fail(RRTMGPNN_ERR_ARGUMENT, "workspace would grow inside a hipGraph capture: issue the call once "
                                         "eagerly before capturing");
    ws_pinned = true;  // the captured graph holds this address from now on
  }
  if (bytes > ws_bytes && ws_pinned)
    return fail(RRTMGPNN_ERR_ARGUMENT, "workspace is pinned by a captured hipGraph and too small for this call: use "
                                       "another context, or rrtmgpnn_context_unpin_workspace after destroying the graph");
  if (bytes > ws_bytes) {
    if (ws) {
      (void)hipStreamSynchronize(stream);
      (void)hipFree(ws);
      ws = nullptr;
      ws_bytes = 0;
    }
    hipError_t e = hipMalloc(&ws, bytes);
    if (e != hipSuccess) return fail(RRTMGPNN_ERR_DEVICE, std::string("workspace hipMalloc: ") + hipGetErrorString(e));
    ws_bytes = bytes;
  }
  *out = ws;
  return RRTMGPNN_OK;
}

extern "C" {

int rrtmgpnn_version(void) { return 1; }

const char *rrtmgpnn_last_error(void) { return g_last_error.c_str(); }

int rrtmgpnn_context_create(int device, void *hip_stream, rrtmgpnn_context **ctx)
{
  if (!ctx) return fail(RRTMGPNN_ERR_ARGUMENT, "ctx out-pointer is null");
  int ndev = 0;
  RRTMGPNN_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(RRTMGPNN_ERR_ARGUMENT, "device ordinal out of range");
  RRTMGPNN_HIP(hipSetDevice(device));
  rrtmgpnn_context *c = new rrtmgpnn_context();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
  c->stream = (hipStream_t)hip_stream;  // NULL = the device's default (null) stream
  *ctx = c;
  return RRTMGPNN_OK;
}

int rrtmgpnn_context_destroy(rrtmgpnn_context *ctx)
{
  if (!ctx) return RRTMGPNN_OK;
  (void)hipSetDevice(ctx->device);
  ctx->pool_clear();
  if (ctx->ws) (void)hipFree(ctx->ws);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return RRTMGPNN_OK;
}

int rrtmgpnn_context_unpin_workspace(rrtmgpnn_context *ctx)
{
  if (int rc = check_ctx(ctx)) return rc;
  ctx->ws_pinned = false;
  return RRTMGPNN_OK;
}

int rrtmgpnn_context_set_sw_kernel(rrtmgpnn_context *ctx, int mode)
{
  if (mode < 0 || mode > 3) return fail(RRTMGPNN_ERR_ARGUMENT, "sw kernel mode must be 0, 1, 2 or 3");
  if (!ctx) {
    rrtmgpnn::g_sw_kernel_default = mode;
    return RRTMGPNN_OK;
  }
  if (int rc = check_ctx(ctx)) return rc;
  ctx->sw_kernel = mode;
  return RRTMGPNN_OK;
}

int rrtmgpnn_context_set_mlp_kernel(rrtmgpnn_context *ctx, int mode)
{
  if (mode < 0 || mode > 1) return fail(RRTMGPNN_ERR_ARGUMENT, "mlp kernel mode must be 0 or 1");
  if (!ctx) {
    rrtmgpnn::g_mlp_kernel_default = mode;
    return RRTMGPNN_OK;
  }
  if (int rc = check_ctx(ctx)) return rc;
  ctx->mlp_kernel = mode;
  return RRTMGPNN_OK;
}

int rrtmgpnn_context_set_mlp_max_cus(rrtmgpnn_context *ctx, int cus)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (cus < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "mlp max cus must be >= 0");
  ctx->mlp_max_cus = cus;
  return RRTMGPNN_OK;
}

int rrtmgpnn_context_get_mlp_max_cus(rrtmgpnn_context *ctx, int *cus)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!cus) return fail(RRTMGPNN_ERR_ARGUMENT, "null cus");
  *cus = ctx->mlp_max_cus;
  return RRTMGPNN_OK;
}

int rrtmgpnn_context_set_stream(rrtmgpnn_context *ctx, void *hip_stream)
{
  if (int rc = check_ctx(ctx)) return rc;
  // The device data environment orders every use of a pooled buffer, a pinned-ring slice and a queued device-to-host
  // copy on the context's one stream: finish the old stream's work (and the pending copies, resetting the ring)
  // before work on the new stream can be handed those buffers, whoever owns the old stream -- also when the new stream
  // is being captured into a hipGraph (the old stream's queued copies and ring slices must be complete before the
  // capture's nodes reuse them).  Only a capturing old stream is left alone: a capture cannot be synchronised, and
  // the graph orders its own nodes.
  hipStreamCaptureStatus cap_old = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(ctx->stream, &cap_old);
  (void)hipGetLastError();
  if ((ctx->stream != (hipStream_t)hip_stream || ctx->own_stream) && cap_old == hipStreamCaptureStatusNone)
    if (int rc = ctx->sync()) return rc;
  if (ctx->own_stream) {
    (void)hipStreamDestroy(ctx->stream);
    ctx->own_stream = false;
  }
  ctx->stream = (hipStream_t)hip_stream;
  return RRTMGPNN_OK;
}

void *rrtmgpnn_context_stream(rrtmgpnn_context *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int rrtmgpnn_context_synchronize(rrtmgpnn_context *ctx)
{
  if (int rc = check_ctx(ctx)) return rc;
  return ctx->sync();  // also completes queued rrtmgpnn_copy_d2h copies
}

int rrtmgpnn_malloc(rrtmgpnn_context *ctx, long long bytes, void **dptr)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!dptr || bytes < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "malloc: bad arguments");
  RRTMGPNN_HIP(hipMalloc(dptr, (size_t)(bytes ? bytes : 4)));
  return RRTMGPNN_OK;
}

int rrtmgpnn_free(rrtmgpnn_context *ctx, void *dptr)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (dptr) RRTMGPNN_HIP(hipFree(dptr));
  return RRTMGPNN_OK;
}

int rrtmgpnn_memcpy_h2d(rrtmgpnn_context *ctx, void *dst, const void *src, long long bytes)
{
  if (int rc = check_ctx(ctx)) return rc;
  RRTMGPNN_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
  RRTMGPNN_HIP(hipStreamSynchronize(ctx->stream));
  return RRTMGPNN_OK;
}

int rrtmgpnn_memcpy_d2h(rrtmgpnn_context *ctx, void *dst, const void *src, long long bytes)
{
  if (int rc = check_ctx(ctx)) return rc;
  RRTMGPNN_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
  RRTMGPNN_HIP(hipStreamSynchronize(ctx->stream));
  return RRTMGPNN_OK;
}

// ---- networks ----
int rrtmgpnn_network_load(rrtmgpnn_context *ctx, const char *path, rrtmgpnn_network **net)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!path || !net) return fail(RRTMGPNN_ERR_ARGUMENT, "network_load: null argument");
  DataFile df;
  if (int rc = read_data_file(path, df)) return rc;
  auto &m = df.vars;
  std::vector<int> dims, act;
  std::vector<char> names;
  const bool nc = df.has("nn_dimsize");  // the reference's netCDF model file (mod_network_rrtmgp.F90:58-122)
  const char *kmin = nc ? "nn_input_coeffs_min" : "input_min", *kmax = nc ? "nn_input_coeffs_max" : "input_max";
  const char *kmean = nc ? "nn_output_coeffs_mean" : "output_mean", *kstd = nc ? "nn_output_coeffs_std" : "output_std";
  if (nc) {
    for (const char *k : {"nn_activation_char", "nn_input_coeffs_min", "nn_input_coeffs_max"})
      if (!df.has(k)) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": missing " + k);
    std::vector<int> hidden = to_int(m["nn_dimsize"]);
    dims.push_back((int)m["nn_input_coeffs_min"].count());  // nn_dim_input
    dims.insert(dims.end(), hidden.begin(), hidden.end());
    const DataVar &ac = m["nn_activation_char"];  // (num_layers, string_len) characters
    const size_t len = ac.dims.size() == 2 ? (size_t)ac.dims[1] : 0;
    for (size_t n = 0; len && n < (size_t)ac.dims[0]; n++) {
      const int code = activation_code(std::string(&ac.data[n * len], len));
      if (code < 0) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": unknown activation function");
      act.push_back(code);
    }
    if (df.has("nn_inputs_char")) {  // (nx, 32) characters, the layout of network_create's input_names
      const DataVar &ic = m["nn_inputs_char"];
      if (ic.dims.size() == 2 && ic.dims[1] == 32) names = ic.data;
    }
  } else {
    for (const char *k : {"dims", "activation", "input_min", "input_max"})
      if (!df.has(k)) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": missing " + k);
    dims = to_int(m["dims"]);
    act = to_int(m["activation"]);
    if (df.has("input_names")) names = m["input_names"].data;
  }
  int nl = (int)dims.size() - 1;
  if (nl < 1 || nl > kMaxLayers || (int)act.size() != nl) return fail(RRTMGPNN_ERR_IO, "network_load: bad dims");
  std::vector<std::vector<float>> W(nl), B(nl);
  std::vector<const float *> wp(nl), bp(nl);
  for (int n = 0; n < nl; n++) {
    std::string wn = (nc ? "nn_weights_" : "w") + std::to_string(n + 1), bn = (nc ? "nn_bias_" : "b") + std::to_string(n + 1);
    if (!df.has(wn) || !df.has(bn)) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": missing layer " + wn);
    W[n] = to_float(m[wn]);  // file (C) order (n_in, n_out) in both formats
    B[n] = to_float(m[bn]);
    if (W[n].size() != (size_t)dims[n] * dims[n + 1] || B[n].size() != (size_t)dims[n + 1])
      return fail(RRTMGPNN_ERR_IO, std::string(path) + ": layer size mismatch");
    wp[n] = W[n].data();
    bp[n] = B[n].data();
  }
  std::vector<float> mn = to_float(m[kmin]), mx = to_float(m[kmax]);
  std::vector<float> om, os;
  if (df.has(kmean) && df.has(kstd)) {
    om = to_float(m[kmean]);
    os = to_float(m[kstd]);
  }
  return rrtmgpnn_network_create(ctx, nl, dims.data(), act.data(), wp.data(), bp.data(), mn.data(), mx.data(),
                                 om.empty() ? nullptr : om.data(), os.empty() ? nullptr : os.data(),
                                 names.empty() ? nullptr : names.data(), net);
}

int rrtmgpnn_network_create(rrtmgpnn_context *ctx, int nlayers, const int *dims, const int *activations,
                            const float *const *weights, const float *const *biases, const float *input_min,
                            const float *input_max, const float *output_mean, const float *output_std,
                            const char *input_names, rrtmgpnn_network **out)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!out || !dims || !activations || !weights || !biases || !input_min || !input_max)
    return fail(RRTMGPNN_ERR_ARGUMENT, "network_create: null argument");
  if (nlayers < 1 || nlayers > kMaxLayers) return fail(RRTMGPNN_ERR_ARGUMENT, "network_create: 1..7 layers");
  if (dims[0] < 1 || dims[0] > kMaxInputs) return fail(RRTMGPNN_ERR_ARGUMENT, "network_create: 1..32 inputs");
  rrtmgpnn_network *net = new rrtmgpnn_network();
  net->device = ctx->device;
  net->nlayers = nlayers;
  for (int n = 0; n <= nlayers; n++) net->dims[n] = dims[n];
  for (int n = 0; n < nlayers; n++) net->act[n] = activations[n];
  net->w.resize(nlayers);
  net->b.resize(nlayers);
  for (int n = 0; n < nlayers; n++) {
    if (dims[n + 1] < 1) {
      delete net;
      return fail(RRTMGPNN_ERR_ARGUMENT, "network_create: empty layer");
    }
    net->w[n].assign(weights[n], weights[n] + (size_t)dims[n] * dims[n + 1]);
    net->b[n].assign(biases[n], biases[n] + dims[n + 1]);
  }
  int nx = dims[0], ny = dims[nlayers];
  net->in_min.assign(input_min, input_min + nx);
  net->in_max.assign(input_max, input_max + nx);
  if (output_mean && output_std) {
    net->out_mean.assign(output_mean, output_mean + ny);
    net->out_std.assign(output_std, output_std + ny);
  }
  for (int i = 0; i < nx; i++) {
    std::string s;
    if (input_names) {
      s.assign(input_names + 32 * i, 32);
      size_t e = s.find_last_not_of(" \0", std::string::npos, 2);
      s = (e == std::string::npos) ? std::string() : s.substr(0, e + 1);
    }
    net->input_names.push_back(s);
  }
  if (int rc = finalize_network(net)) {
    rrtmgpnn_network_destroy(net);
    return rc;
  }
  *out = net;
  return RRTMGPNN_OK;
}

int rrtmgpnn_network_destroy(rrtmgpnn_network *net)
{
  if (!net) return RRTMGPNN_OK;
  (void)hipSetDevice(net->device);
  if (net->d_raw) (void)hipFree(net->d_raw);
  if (net->d_packed) (void)hipFree(net->d_packed);
  if (net->d_packed32) (void)hipFree(net->d_packed32);
  delete net;
  return RRTMGPNN_OK;
}

int rrtmgpnn_network_get_dims(const rrtmgpnn_network *net, int *nlayers, int dims[8])
{
  if (!net || !nlayers || !dims) return fail(RRTMGPNN_ERR_ARGUMENT, "get_dims: null argument");
  *nlayers = net->nlayers;
  for (int n = 0; n < 8; n++) dims[n] = n <= net->nlayers ? net->dims[n] : 0;
  return RRTMGPNN_OK;
}

int rrtmgpnn_network_get_input_name(const rrtmgpnn_network *net, int i, char *buf, int buflen)
{
  if (!net || !buf || buflen < 1 || i < 0 || i >= net->dims[0])
    return fail(RRTMGPNN_ERR_ARGUMENT, "get_input_name: bad argument");
  std::snprintf(buf, (size_t)buflen, "%s", net->input_names[i].c_str());
  return RRTMGPNN_OK;
}

int rrtmgpnn_network_get_input_scaling(const rrtmgpnn_network *net, float *mn, float *mx)
{
  if (!net || !mn || !mx) return fail(RRTMGPNN_ERR_ARGUMENT, "get_input_scaling: null argument");
  for (int i = 0; i < net->dims[0]; i++) {
    mn[i] = net->in_min[i];
    mx[i] = net->in_max[i];
  }
  return RRTMGPNN_OK;
}

// ---- gas optics ----
int rrtmgpnn_compute_nn_inputs(rrtmgpnn_context *ctx, int ncol, int nlay, int ninputs, const float *play,
                               const float *tlay, const float *const *gas_conc, const int *gas_ndims,
                               const rrtmgpnn_network *net, float *nn_inputs)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!net || !play || !tlay || !gas_conc || !gas_ndims || !nn_inputs || ncol < 0 || nlay < 1)
    return fail(RRTMGPNN_ERR_ARGUMENT, "compute_nn_inputs: bad argument");
  if (ninputs != net->dims[0] || ninputs < 4 || ninputs > kMaxInputs)
    return fail(RRTMGPNN_ERR_ARGUMENT, "compute_nn_inputs: ninputs does not match the network");
  if (!gas_conc[2] || !gas_conc[3] || gas_ndims[2] != 2 || gas_ndims[3] != 2)
    return fail(RRTMGPNN_ERR_ARGUMENT, "compute_nn_inputs: inputs 3 (h2o) and 4 (o3) must be 2-D (nlay,ncol)");
  GasArgs g{};
  for (int k = 0; k < ninputs; k++) {
    g.p[k] = k >= 2 ? gas_conc[k] : nullptr;
    g.nd[k] = k >= 2 ? gas_ndims[k] : 0;
    if (k >= 2 && g.p[k] && (g.nd[k] < 0 || g.nd[k] > 2))
      return fail(RRTMGPNN_ERR_ARGUMENT, "compute_nn_inputs: gas_ndims must be 0, 1 or 2");
  }
  std::vector<float> mm(2 * ninputs);
  for (int k = 0; k < ninputs; k++) {
    mm[k] = net->in_min[k];
    mm[ninputs + k] = net->in_max[k];
  }
  return launch_nn_inputs(ctx, ncol, nlay, ninputs, play, tlay, g, mm.data(), nn_inputs);
}

int rrtmgpnn_get_col_dry(rrtmgpnn_context *ctx, int ncol, int nlay, const float *vmr_h2o, const float *plev,
                         float *col_dry)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!vmr_h2o || !plev || !col_dry || ncol < 0 || nlay < 1) return fail(RRTMGPNN_ERR_ARGUMENT, "get_col_dry: bad argument");
  return launch_col_dry(ctx, ncol, nlay, vmr_h2o, plev, col_dry);
}

int rrtmgpnn_interpolate_tlev(rrtmgpnn_context *ctx, int ncol, int nlay, const float *play, const float *plev,
                              const float *tlay, float *tlev)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!play || !plev || !tlay || !tlev || ncol < 0 || nlay < 2)
    return fail(RRTMGPNN_ERR_ARGUMENT, "interpolate_tlev: bad argument (needs nlay >= 2)");
  return launch_tlev(ctx, ncol, nlay, play, plev, tlay, tlev);
}

int rrtmgpnn_predict_nn_lw(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs, const float *nn_inputs,
                           const float *col_dry, const rrtmgpnn_network *const *nets, int nnets, float *tau,
                           float *pfrac)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!nets || !nn_inputs || !col_dry || !tau || !pfrac || ncol < 0 || nlay < 1 || ngpt < 1)
    return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_lw: bad argument");
  long long N = (long long)ncol * nlay;
  if (nnets == 2) {
    const rrtmgpnn_network *A = nets[0], *B = nets[1];
    if (!A || !B) return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_lw: null network");
    if (A->dims[0] != ninputs || B->dims[0] != ninputs || A->dims[A->nlayers] != ngpt || B->dims[B->nlayers] != ngpt)
      return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_lw: network sizes do not match (ninputs, ngpt)");
    if (!A->has_out_scaling())
      return fail(RRTMGPNN_ERR_ARGUMENT, "output_sgemm_tau: NN output scaling coefficients missing");
    return launch_mlp(ctx, MLP_LW_PAIR, A, B, N, ngpt, nn_inputs, col_dry, tau, pfrac, nullptr);
  } else if (nnets == 1) {
    const rrtmgpnn_network *A = nets[0];
    if (!A || A->dims[0] != ninputs || A->dims[A->nlayers] != 2 * ngpt)
      return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_lw: single model must have 2*ngpt outputs");
    if (!A->has_out_scaling())
      return fail(RRTMGPNN_ERR_ARGUMENT, "output_sgemm_lw: NN output scaling coefficients missing");
    return launch_mlp(ctx, MLP_LW_BOTH, A, nullptr, N, ngpt, nn_inputs, col_dry, tau, pfrac, nullptr);
  }
  return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_lw: nnets must be 1 or 2");
}

// Fused gas optics (NN path): the inputs of compute_nn_inputs and get_col_dry are formed inside the MLP kernel.
static int fused_inputs(const char *who, const rrtmgpnn_network *net, int ninputs, int nlay, const float *play,
                        const float *tlay, const float *plev, const float *vmr_h2o, const float *const *gas_conc,
                        const int *gas_ndims, MlpInputs &in)
{
  if (!net || !play || !tlay || !plev || !vmr_h2o || !gas_conc || !gas_ndims || nlay < 1)
    return fail(RRTMGPNN_ERR_ARGUMENT, std::string(who) + ": bad argument");
  if (ninputs != net->dims[0] || ninputs < 4 || ninputs > kMaxInputs)
    return fail(RRTMGPNN_ERR_ARGUMENT, std::string(who) + ": ninputs does not match the network");
  if (!gas_conc[2] || !gas_conc[3] || gas_ndims[2] != 2 || gas_ndims[3] != 2)
    return fail(RRTMGPNN_ERR_ARGUMENT, std::string(who) + ": inputs 3 (h2o) and 4 (o3) must be 2-D (nlay,ncol)");
  in = MlpInputs{};
  in.play = play; in.tlay = tlay; in.plev = plev; in.h2o = vmr_h2o; in.nlay = nlay;
  for (int k = 0; k < ninputs; k++) {
    in.gas.p[k] = k >= 2 ? gas_conc[k] : nullptr;
    in.gas.nd[k] = k >= 2 ? gas_ndims[k] : 0;
    if (k >= 2 && in.gas.p[k] && (in.gas.nd[k] < 0 || in.gas.nd[k] > 2))
      return fail(RRTMGPNN_ERR_ARGUMENT, std::string(who) + ": gas_ndims must be 0, 1 or 2");
    in.mn[k] = net->in_min[k];
    in.mx[k] = net->in_max[k];
  }
  return RRTMGPNN_OK;
}

// no in-kernel-input instance for these networks: compute_nn_inputs + get_col_dry into the context workspace, then
// the MLP on them (the same kernels as the separate entries)
static int fused_fallback(rrtmgpnn_context *ctx, int ncol, int nlay, const MlpInputs &in, int ninputs,
                          const float **x, const float **col_dry)
{
  const size_t N = (size_t)ncol * nlay;
  void *ws = nullptr;
  if (int rc = ctx->workspace(sizeof(float) * N * (ninputs + 1), &ws)) return rc;
  float *xw = (float *)ws, *cw = xw + N * ninputs;
  std::vector<float> mm(2 * ninputs);
  for (int k = 0; k < ninputs; k++) { mm[k] = in.mn[k]; mm[ninputs + k] = in.mx[k]; }
  if (int rc = launch_nn_inputs(ctx, ncol, nlay, ninputs, in.play, in.tlay, in.gas, mm.data(), xw)) return rc;
  if (int rc = launch_col_dry(ctx, ncol, nlay, in.h2o, in.plev, cw)) return rc;
  *x = xw;
  *col_dry = cw;
  return RRTMGPNN_OK;
}

int rrtmgpnn_gas_optics_lw_nn(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs, const float *play,
                              const float *tlay, const float *plev, const float *vmr_h2o,
                              const float *const *gas_conc, const int *gas_ndims,
                              const rrtmgpnn_network *const *nets, int nnets, float *tau, float *pfrac)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!nets || !nets[0] || !tau || !pfrac || ncol < 0 || ngpt < 1 || (nnets != 1 && nnets != 2))
    return fail(RRTMGPNN_ERR_ARGUMENT, "gas_optics_lw_nn: bad argument");
  MlpInputs in;
  if (int rc = fused_inputs("gas_optics_lw_nn", nets[0], ninputs, nlay, play, tlay, plev, vmr_h2o, gas_conc, gas_ndims,
                            in))
    return rc;
  if (ncol == 0) return RRTMGPNN_OK;
  const long long N = (long long)ncol * nlay;
  if (nnets == 2) {
    const rrtmgpnn_network *A = nets[0], *B = nets[1];
    if (!B || B->dims[0] != ninputs || A->dims[A->nlayers] != ngpt || B->dims[B->nlayers] != ngpt)
      return fail(RRTMGPNN_ERR_ARGUMENT, "gas_optics_lw_nn: network sizes do not match (ninputs, ngpt)");
    if (!A->has_out_scaling()) return fail(RRTMGPNN_ERR_ARGUMENT, "output_sgemm_tau: NN output scaling coefficients missing");
    const int rc = launch_mlp(ctx, MLP_LW_PAIR, A, B, N, ngpt, nullptr, nullptr, tau, pfrac, nullptr, &in);
    if (rc != RRTMGPNN_ERR_UNSUPPORTED) return rc;
  }
  const float *x = nullptr, *cd = nullptr;
  if (int rc = fused_fallback(ctx, ncol, nlay, in, ninputs, &x, &cd)) return rc;
  return rrtmgpnn_predict_nn_lw(ctx, ncol, nlay, ngpt, ninputs, x, cd, nets, nnets, tau, pfrac);
}

int rrtmgpnn_gas_optics_sw_nn(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs, const float *play,
                              const float *tlay, const float *plev, const float *vmr_h2o,
                              const float *const *gas_conc, const int *gas_ndims,
                              const rrtmgpnn_network *const *nets, float *tau, float *ssa, float *g)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!nets || !nets[0] || !tau || ncol < 0 || ngpt < 1) return fail(RRTMGPNN_ERR_ARGUMENT, "gas_optics_sw_nn: bad argument");
  MlpInputs in;
  if (int rc = fused_inputs("gas_optics_sw_nn", nets[0], ninputs, nlay, play, tlay, plev, vmr_h2o, gas_conc, gas_ndims,
                            in))
    return rc;
  if (ncol == 0) return RRTMGPNN_OK;
  const long long N = (long long)ncol * nlay;
  const rrtmgpnn_network *A = nets[0], *B = ssa ? nets[1] : nullptr;
  if (ssa) {
    if (!B || B->dims[0] != ninputs || A->dims[A->nlayers] != ngpt || B->dims[B->nlayers] != ngpt ||
        !A->has_out_scaling() || !B->has_out_scaling())
      return fail(RRTMGPNN_ERR_ARGUMENT, "gas_optics_sw_nn: absorption / Rayleigh networks missing or inconsistent");
    const int rc = launch_mlp(ctx, MLP_SW_PAIR, A, B, N, ngpt, nullptr, nullptr, tau, ssa, g, &in);
    if (rc != RRTMGPNN_ERR_UNSUPPORTED) return rc;
  }
  const float *x = nullptr, *cd = nullptr;
  if (int rc = fused_fallback(ctx, ncol, nlay, in, ninputs, &x, &cd)) return rc;
  return rrtmgpnn_predict_nn_sw(ctx, ncol, nlay, ngpt, ninputs, x, cd, nets, tau, ssa, g);
}

int rrtmgpnn_predict_nn_sw(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs, const float *nn_inputs,
                           const float *col_dry, const rrtmgpnn_network *const *nets, float *tau, float *ssa, float *g)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!nets || !nets[0] || !nn_inputs || !col_dry || !tau || ncol < 0 || nlay < 1 || ngpt < 1)
    return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_sw: bad argument");
  const rrtmgpnn_network *A = nets[0];
  if (A->dims[0] != ninputs || A->dims[A->nlayers] != ngpt)
    return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_sw: network sizes do not match (ninputs, ngpt)");
  if (!A->has_out_scaling()) return fail(RRTMGPNN_ERR_ARGUMENT, "output_sgemm_tau: NN output scaling coefficients missing");
  long long N = (long long)ncol * nlay;
  if (!ssa) return launch_mlp(ctx, MLP_SW_ABS, A, nullptr, N, ngpt, nn_inputs, col_dry, tau, nullptr, nullptr);
  const rrtmgpnn_network *B = nets[1];
  if (!B || B->dims[0] != ninputs || B->dims[B->nlayers] != ngpt || !B->has_out_scaling())
    return fail(RRTMGPNN_ERR_ARGUMENT, "predict_nn_sw: Rayleigh network missing or inconsistent");
  return launch_mlp(ctx, MLP_SW_PAIR, A, B, N, ngpt, nn_inputs, col_dry, tau, ssa, g);
}

int rrtmgpnn_network_forward(rrtmgpnn_context *ctx, const rrtmgpnn_network *net, long long nbatch, const float *x,
                             float *out)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!net || !x || !out || nbatch < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "network_forward: bad argument");
  if (net->d_packed) return launch_mlp(ctx, MLP_PLAIN, net, nullptr, nbatch, net->dims[net->nlayers], x, nullptr, out, nullptr, nullptr);
  return launch_mlp_generic(ctx, net, nbatch, x, out);
}

int rrtmgpnn_compute_planck_source_nn(rrtmgpnn_context *ctx, int ncol, int nlay, int nbnd, int ngpt, int nPlanckTemp,
                                      const float *tlay, const float *tlev, const float *tsfc, int sfc_lay,
                                      const int *band_lims_gpt, float temp_ref_min, float totplnk_delta,
                                      const float *totplnk, float *sfc_source, float *sfc_source_Jac, float *pfrac,
                                      float *lev_source)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!tlay || !tlev || !tsfc || !totplnk || !sfc_source || !sfc_source_Jac || !pfrac || !lev_source || ncol < 0 ||
      nlay < 1 || ngpt < 1 || nPlanckTemp < 2 || sfc_lay < 1 || sfc_lay > nlay || !(totplnk_delta > 0.0f))
    return fail(RRTMGPNN_ERR_ARGUMENT, "compute_planck_source_nn: bad argument");
  BandArgs b;
  if (int rc = band_args(nbnd, band_lims_gpt, ngpt, b)) return rc;
  return launch_planck_source(ctx, ncol, nlay, ngpt, nPlanckTemp, tlay, tlev, tsfc, sfc_lay, b, temp_ref_min,
                              totplnk_delta, totplnk, sfc_source, sfc_source_Jac, pfrac, lev_source);
}

int rrtmgpnn_lw_solver_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                              const float *Ds, const float *weights, const float *inc_flux, const float *tau,
                              const float *lay_source, const float *lev_source, const float *sfc_emis_gpt,
                              const float *sfc_source, float *flux_up, float *flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!Ds || !weights || !tau || !lay_source || !lev_source || !sfc_emis_gpt || !sfc_source || !flux_up || !flux_dn ||
      ngpt < 1 || nlay < 1 || ncol < 0)
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw_solver_noscat: bad argument");
  return launch_lw_noscat(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, lay_source, lev_source,
                          sfc_emis_gpt, sfc_source, flux_up, flux_dn);
}

int rrtmgpnn_lw_solver_noscat_planck(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                     const float *Ds, const float *weights, const float *inc_flux, const float *tau,
                                     const float *pfrac, int nbnd, int nPlanckTemp, const float *tlay,
                                     const float *tlev, const float *tsfc, int sfc_lay, const int *band_lims_gpt,
                                     float temp_ref_min, float totplnk_delta, const float *totplnk,
                                     int emis_by_band, const float *sfc_emis, float *flux_up, float *flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!Ds || !weights || !tau || !pfrac || !tlay || !tlev || !tsfc || !totplnk || !sfc_emis || !flux_up ||
      !flux_dn || ngpt < 1 || nlay < 1 || ncol < 0 || nPlanckTemp < 2 || sfc_lay < 1 || sfc_lay > nlay ||
      !(totplnk_delta > 0.0f))
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw_solver_noscat_planck: bad argument");
  BandArgs b;
  if (int rc = band_args(nbnd, band_lims_gpt, ngpt, b)) return rc;
  if (emis_by_band)
    if (int rc = bands_cover(b, ngpt)) return rc;
  return launch_lw_noscat_planck(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, pfrac,
                                 nPlanckTemp, tlay, tlev, tsfc, sfc_lay, b, temp_ref_min, totplnk_delta, totplnk,
                                 emis_by_band != 0, sfc_emis, nullptr, flux_up, flux_dn);
}

int rrtmgpnn_lw_solver_noscat_planck_inc(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                         int nmus, const float *Ds, const float *weights, const float *inc_flux,
                                         const float *tau, const float *tau_bnd, const float *pfrac, int nbnd,
                                         int nPlanckTemp, const float *tlay, const float *tlev, const float *tsfc,
                                         int sfc_lay, const int *band_lims_gpt, float temp_ref_min,
                                         float totplnk_delta, const float *totplnk, int emis_by_band,
                                         const float *sfc_emis, float *flux_up, float *flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!Ds || !weights || !tau || !tau_bnd || !pfrac || !tlay || !tlev || !tsfc || !totplnk || !sfc_emis ||
      !flux_up || !flux_dn || ngpt < 1 || nlay < 1 || ncol < 0 || nPlanckTemp < 2 || sfc_lay < 1 || sfc_lay > nlay ||
      !(totplnk_delta > 0.0f))
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw_solver_noscat_planck_inc: bad argument");
  BandArgs b;
  if (int rc = band_args(nbnd, band_lims_gpt, ngpt, b)) return rc;
  if (int rc = bands_cover(b, ngpt)) return rc;
  return launch_lw_noscat_planck(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, pfrac,
                                 nPlanckTemp, tlay, tlev, tsfc, sfc_lay, b, temp_ref_min, totplnk_delta, totplnk,
                                 emis_by_band != 0, sfc_emis, tau_bnd, flux_up, flux_dn);
}

int rrtmgpnn_lw_solver_1rescl(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                              const float *Ds, const float *weights, const float *inc_flux, const float *tau,
                              const float *ssa, const float *g, const float *lay_source, const float *lev_source,
                              const float *sfc_emis_gpt, const float *sfc_source, float *flux_up, float *flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!Ds || !weights || !tau || !ssa || !g || !lay_source || !lev_source || !sfc_emis_gpt || !sfc_source ||
      !flux_up || !flux_dn || ngpt < 1 || nlay < 1 || ncol < 0)
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw_solver_1rescl: bad argument");
  return launch_lw_rescl(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, ssa, g, lay_source,
                         lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn);
}

int rrtmgpnn_lw_solver_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                               const float *inc_flux, const float *tau, const float *ssa, const float *g,
                               const float *lev_source, const float *sfc_emis_gpt, const float *sfc_source,
                               float *flux_up, float *flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!tau || !ssa || !g || !lev_source || !sfc_emis_gpt || !sfc_source || !flux_up || !flux_dn || ngpt < 1 ||
      nlay < 1 || ncol < 0)
    return fail(RRTMGPNN_ERR_ARGUMENT, "lw_solver_2stream: bad argument");
  return launch_lw_2stream(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, ssa, g, lev_source, sfc_emis_gpt,
                           sfc_source, flux_up, flux_dn);
}

int rrtmgpnn_sw_solver_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                               const float *inc_flux, const float *inc_flux_dif, const float *tau, const float *ssa,
                               const float *g, const float *mu0, const float *sfc_alb_dir_gpt,
                               const float *sfc_alb_dif_gpt, float *flux_up, float *flux_dn, float *flux_dir)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!inc_flux || !tau || !ssa || !mu0 || !sfc_alb_dir_gpt || !sfc_alb_dif_gpt || !flux_up || !flux_dn ||
      !flux_dir || ngpt < 1 || nlay < 1 || ncol < 0)
    return fail(RRTMGPNN_ERR_ARGUMENT, "sw_solver_2stream: bad argument");
  return launch_sw_2stream(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g, mu0, sfc_alb_dir_gpt,
                           sfc_alb_dif_gpt, nullptr, nullptr, nullptr, nullptr, flux_up, flux_dn, flux_dir);
}

// ---- the *_gpt entries: the call above with rte_lw's lw_Ds and ty_fluxes_flexible's g-point outputs, handed to the
// launch through the context for this one call ----
namespace {
struct ExtrasScope {
  rrtmgpnn_context *c;
  ExtrasScope(rrtmgpnn_context *ctx, const float *ds, float *up, float *dn, float *dir) : c(ctx)
  {
    c->extras.lw_Ds = ds;
    c->extras.gpt_up = up;
    c->extras.gpt_dn = dn;
    c->extras.gpt_dir = dir;
  }
  ~ExtrasScope() { c->extras = rrtmgpnn_context::SolverExtras{}; }
};
int lw_ds_check(int nmus, const float *lw_Ds)
{
  if (lw_Ds && nmus != 1)
    return fail(RRTMGPNN_ERR_ARGUMENT, "rte_lw: providing lw_Ds incompatible with specifying n_gauss_angles");
  return RRTMGPNN_OK;
}
}  // namespace

int rrtmgpnn_lw_solver_noscat_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                  const float *Ds, const float *weights, const float *lw_Ds, const float *inc_flux,
                                  const float *tau, const float *lay_source, const float *lev_source,
                                  const float *sfc_emis_gpt, const float *sfc_source, float *flux_up, float *flux_dn,
                                  float *gpt_flux_up, float *gpt_flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (int rc = lw_ds_check(nmus, lw_Ds)) return rc;
  ExtrasScope x(ctx, lw_Ds, gpt_flux_up, gpt_flux_dn, nullptr);
  return rrtmgpnn_lw_solver_noscat(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, lay_source,
                                   lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn);
}

int rrtmgpnn_lw_solver_noscat_planck_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                         const float *Ds, const float *weights, const float *lw_Ds,
                                         const float *inc_flux, const float *tau, const float *pfrac, int nbnd,
                                         int nPlanckTemp, const float *tlay, const float *tlev, const float *tsfc,
                                         int sfc_lay, const int *band_lims_gpt, float temp_ref_min,
                                         float totplnk_delta, const float *totplnk, int emis_by_band,
                                         const float *sfc_emis, float *flux_up, float *flux_dn, float *gpt_flux_up,
                                         float *gpt_flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (int rc = lw_ds_check(nmus, lw_Ds)) return rc;
  ExtrasScope x(ctx, lw_Ds, gpt_flux_up, gpt_flux_dn, nullptr);
  return rrtmgpnn_lw_solver_noscat_planck(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, pfrac,
                                          nbnd, nPlanckTemp, tlay, tlev, tsfc, sfc_lay, band_lims_gpt, temp_ref_min,
                                          totplnk_delta, totplnk, emis_by_band, sfc_emis, flux_up, flux_dn);
}

int rrtmgpnn_sw_solver_2stream_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                   const float *inc_flux, const float *inc_flux_dif, const float *tau,
                                   const float *ssa, const float *g, const float *mu0, const float *sfc_alb_dir_gpt,
                                   const float *sfc_alb_dif_gpt, float *flux_up, float *flux_dn, float *flux_dir,
                                   float *gpt_flux_up, float *gpt_flux_dn, float *gpt_flux_dir)
{
  if (int rc = check_ctx(ctx)) return rc;
  ExtrasScope x(ctx, nullptr, gpt_flux_up, gpt_flux_dn, gpt_flux_dir);
  return rrtmgpnn_sw_solver_2stream(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g, mu0,
                                    sfc_alb_dir_gpt, sfc_alb_dif_gpt, flux_up, flux_dn, flux_dir);
}

int rrtmgpnn_sw_solver_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                              const float *tau, const float *mu0, float *flux_dir)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!inc_flux || !tau || !mu0 || !flux_dir || ngpt < 1 || nlay < 1 || ncol < 0)
    return fail(RRTMGPNN_ERR_ARGUMENT, "sw_solver_noscat: bad argument");
  return launch_sw_noscat(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, mu0, flux_dir);
}

int rrtmgpnn_lw_solver_1rescl_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                  const float *Ds, const float *weights, const float *inc_flux, const float *tau,
                                  const float *ssa, const float *g, const float *lay_source, const float *lev_source,
                                  const float *sfc_emis_gpt, const float *sfc_source, float *flux_up, float *flux_dn,
                                  float *gpt_flux_up, float *gpt_flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  ExtrasScope x(ctx, nullptr, gpt_flux_up, gpt_flux_dn, nullptr);
  return rrtmgpnn_lw_solver_1rescl(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, ssa, g,
                                   lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn);
}

int rrtmgpnn_lw_solver_2stream_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                   const float *inc_flux, const float *tau, const float *ssa, const float *g,
                                   const float *lev_source, const float *sfc_emis_gpt, const float *sfc_source,
                                   float *flux_up, float *flux_dn, float *gpt_flux_up, float *gpt_flux_dn)
{
  if (int rc = check_ctx(ctx)) return rc;
  ExtrasScope x(ctx, nullptr, gpt_flux_up, gpt_flux_dn, nullptr);
  return rrtmgpnn_lw_solver_2stream(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, ssa, g, lev_source, sfc_emis_gpt,
                                    sfc_source, flux_up, flux_dn);
}

int rrtmgpnn_sw_solver_noscat_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                  const float *inc_flux, const float *tau, const float *mu0, float *flux_dir,
                                  float *gpt_flux_dir)
{
  if (int rc = check_ctx(ctx)) return rc;
  ExtrasScope x(ctx, nullptr, nullptr, nullptr, gpt_flux_dir);
  return rrtmgpnn_sw_solver_noscat(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, mu0, flux_dir);
}

int rrtmgpnn_sw_solver_2stream_inc(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                   const float *inc_flux, const float *inc_flux_dif, const float *tau,
                                   const float *ssa, const float *g, int nbnd, const int *band_lims_gpt,
                                   const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, const float *mu0,
                                   const float *sfc_alb_dir_gpt, const float *sfc_alb_dif_gpt, float *flux_up,
                                   float *flux_dn, float *flux_dir)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!inc_flux || !tau || !ssa || !tau_bnd || !ssa_bnd || !g_bnd || !mu0 || !sfc_alb_dir_gpt || !sfc_alb_dif_gpt ||
      !flux_up || !flux_dn || !flux_dir || ngpt < 1 || nlay < 1 || ncol < 0)
    return fail(RRTMGPNN_ERR_ARGUMENT, "sw_solver_2stream_inc: bad argument");
  BandArgs b;
  if (int rc = band_args(nbnd, band_lims_gpt, ngpt, b)) return rc;
  if (int rc = bands_cover(b, ngpt)) return rc;
  return launch_sw_2stream(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, g, mu0, sfc_alb_dir_gpt,
                           sfc_alb_dif_gpt, &b, tau_bnd, ssa_bnd, g_bnd, flux_up, flux_dn, flux_dir);
}

int rrtmgpnn_expand_band_to_gpt(rrtmgpnn_context *ctx, int nband, int ngpt, int ncol, const int *band_lims_gpt,
                                const float *arr_in, float *arr_out)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!arr_in || !arr_out || ncol < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "expand: bad argument");
  BandArgs b;
  if (int rc = band_args(nband, band_lims_gpt, ngpt, b)) return rc;
  return launch_expand(ctx, nband, ngpt, ncol, b, arr_in, arr_out);
}

// ---- cloud optics --------------------------------------------------------------------------------
static int cloud_upload(rrtmgpnn_context *ctx, rrtmgpnn_cloud_optics *c, const std::vector<const float *> &src,
                        const std::vector<size_t> &counts)
{
  size_t total = 0;
  for (size_t k = 0; k < src.size(); k++) {
    c->off[k] = total;
    total += counts[k];
  }
  std::vector<float> img(total);
  for (size_t k = 0; k < src.size(); k++) std::memcpy(img.data() + c->off[k], src[k], sizeof(float) * counts[k]);
  RRTMGPNN_HIP(hipSetDevice(ctx->device));
  RRTMGPNN_HIP(hipMalloc(&c->d_tab, sizeof(float) * total));
  RRTMGPNN_HIP(hipMemcpy(c->d_tab, img.data(), sizeof(float) * total, hipMemcpyHostToDevice));
  return RRTMGPNN_OK;
}

int rrtmgpnn_cloud_optics_create_lut(rrtmgpnn_context *ctx, int nband, const float *band_lims_wvn, int nsize_liq,
                                     int nsize_ice, int nrghice, float radliq_lwr, float radliq_upr,
                                     float radice_lwr, float radice_upr, const float *lut_extliq,
                                     const float *lut_ssaliq, const float *lut_asyliq, const float *lut_extice,
                                     const float *lut_ssaice, const float *lut_asyice, rrtmgpnn_cloud_optics **co)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!co || nband < 1 || nband > 256 || nsize_liq < 2 || nsize_ice < 2 || nrghice < 1 || !lut_extliq || !lut_ssaliq ||
      !lut_asyliq || !lut_extice || !lut_ssaice || !lut_asyice)
    return fail(RRTMGPNN_ERR_ARGUMENT, "cloud_optics_create_lut: bad argument");
  auto *c = new rrtmgpnn_cloud_optics();
  c->device = ctx->device;
  c->lut_mode = 1;
  c->nband = nband;
  c->nsize_liq = nsize_liq;
  c->nsize_ice = nsize_ice;
  c->nrghice = nrghice;
  c->radliq_lwr = radliq_lwr; c->radliq_upr = radliq_upr;
  c->radice_lwr = radice_lwr; c->radice_upr = radice_upr;
  // load_lut (mo_cloud_optics.F90:141-142): step sizes in working precision
  c->liq_step = (radliq_upr - radliq_lwr) / (float)(nsize_liq - 1);
  c->ice_step = (radice_upr - radice_lwr) / (float)(nsize_ice - 1);
  if (band_lims_wvn) c->band_lims_wvn.assign(band_lims_wvn, band_lims_wvn + 2 * nband);
  const size_t nl = (size_t)nsize_liq * nband, ni = (size_t)nsize_ice * nband * nrghice;
  if (int rc = cloud_upload(ctx, c, {lut_extliq, lut_ssaliq, lut_asyliq, lut_extice, lut_ssaice, lut_asyice},
                            {nl, nl, nl, ni, ni, ni})) {
    delete c;
    return rc;
  }
  *co = c;
  return RRTMGPNN_OK;
}

int rrtmgpnn_cloud_optics_create_pade(rrtmgpnn_context *ctx, int nband, const float *band_lims_wvn, int nsizereg,
                                      int ncoef_ext, int ncoef_ssa, int nrghice, const float *pade_extliq,
                                      const float *pade_ssaliq, const float *pade_asyliq, const float *pade_extice,
                                      const float *pade_ssaice, const float *pade_asyice,
                                      const float *sizreg_extliq, const float *sizreg_ssaliq,
                                      const float *sizreg_asyliq, const float *sizreg_extice,
                                      const float *sizreg_ssaice, const float *sizreg_asyice,
                                      rrtmgpnn_cloud_optics **co)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!co || nband < 1 || nband > 256 || nrghice < 1 || !pade_extliq || !pade_ssaliq || !pade_asyliq || !pade_extice ||
      !pade_ssaice || !pade_asyice || !sizreg_extliq || !sizreg_ssaliq || !sizreg_asyliq || !sizreg_extice ||
      !sizreg_ssaice || !sizreg_asyice)
    return fail(RRTMGPNN_ERR_ARGUMENT, "cloud_optics_create_pade: bad argument");
  if (nsizereg != 3)
    return fail(RRTMGPNN_ERR_ARGUMENT, "cloud_optics%init(): Expecting precisely three size regimes for Pade approximants");
  if (ncoef_ext != 6 || ncoef_ssa != 5)
    return fail(RRTMGPNN_ERR_UNSUPPORTED, "cloud_optics: Pade approximants of order [2/3] (ext) and [2/2] (ssa, g) only");
  auto *c = new rrtmgpnn_cloud_optics();
  c->device = ctx->device;
  c->lut_mode = 0;
  c->nband = nband;
  c->nrghice = nrghice;
  c->nsizereg = nsizereg;
  c->ncoef_ext = ncoef_ext;
  c->ncoef_ssa = ncoef_ssa;
  const int nbound = nsizereg + 1;
  // load_pade (:250-253): radius limits from the extinction size regimes
  c->radliq_lwr = sizreg_extliq[0]; c->radliq_upr = sizreg_extliq[nbound - 1];
  c->radice_lwr = sizreg_extice[0]; c->radice_upr = sizreg_extice[nbound - 1];
  if (band_lims_wvn) c->band_lims_wvn.assign(band_lims_wvn, band_lims_wvn + 2 * nband);
  const size_t le = (size_t)nband * nsizereg * ncoef_ext, ls = (size_t)nband * nsizereg * ncoef_ssa;
  const size_t nb = (size_t)nbound;
  if (int rc = cloud_upload(ctx, c,
                            {pade_extliq, pade_ssaliq, pade_asyliq, pade_extice, pade_ssaice, pade_asyice,
                             sizreg_extliq, sizreg_ssaliq, sizreg_asyliq, sizreg_extice, sizreg_ssaice, sizreg_asyice},
                            {le, ls, ls, le * nrghice, ls * nrghice, ls * nrghice, nb, nb, nb, nb, nb, nb})) {
    delete c;
    return rc;
  }
  *co = c;
  return RRTMGPNN_OK;
}

int rrtmgpnn_cloud_optics_load(rrtmgpnn_context *ctx, const char *path, int use_lut, rrtmgpnn_cloud_optics **co)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!path || !co) return fail(RRTMGPNN_ERR_ARGUMENT, "cloud_optics_load: null argument");
  DataFile df;  // RBIN conversion or the coefficient file itself (classic netCDF)
  if (int rc = read_data_file(path, df)) return rc;
  auto &m = df.vars;
  auto need = [&](const char *k) -> const DataVar * {
    auto it = m.find(k);
    return it == m.end() ? nullptr : &it->second;
  };
  const DataVar *bl = need("bnd_limits_wavenumber");
  if (!bl || bl->dims.size() != 2) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": missing bnd_limits_wavenumber");
  const int nband = bl->dims[0];
  std::vector<float> blw = to_float(*bl);
  auto F = [&](const char *k) { return to_float(m[k]); };
  if (use_lut) {
    for (const char *k : {"lut_extliq", "lut_ssaliq", "lut_asyliq", "lut_extice", "lut_ssaice", "lut_asyice",
                          "radliq_lwr", "radliq_upr", "radice_lwr", "radice_upr"})
      if (!need(k)) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": missing " + k);
    const auto &li = m["lut_extice"];
    if (li.dims.size() != 3 || m["lut_extliq"].dims.size() != 2) return fail(RRTMGPNN_ERR_IO, "cloud_optics_load: bad LUT shape");
    std::vector<float> a = F("lut_extliq"), b = F("lut_ssaliq"), c = F("lut_asyliq"), d = F("lut_extice"),
                       e = F("lut_ssaice"), f = F("lut_asyice");
    return rrtmgpnn_cloud_optics_create_lut(ctx, nband, blw.data(), m["lut_extliq"].dims[1], li.dims[2], li.dims[0],
                                            F("radliq_lwr")[0], F("radliq_upr")[0], F("radice_lwr")[0],
                                            F("radice_upr")[0], a.data(), b.data(), c.data(), d.data(), e.data(),
                                            f.data(), co);
  }
  for (const char *k : {"pade_extliq", "pade_ssaliq", "pade_asyliq", "pade_extice", "pade_ssaice", "pade_asyice",
                        "pade_sizreg_extliq", "pade_sizreg_ssaliq", "pade_sizreg_asyliq", "pade_sizreg_extice",
                        "pade_sizreg_ssaice", "pade_sizreg_asyice"})
    if (!need(k)) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": missing " + k);
  const auto &pe = m["pade_extice"];
  if (pe.dims.size() != 4 || m["pade_ssaliq"].dims.size() != 3) return fail(RRTMGPNN_ERR_IO, "cloud_optics_load: bad Pade shape");
  std::vector<float> a = F("pade_extliq"), b = F("pade_ssaliq"), c = F("pade_asyliq"), d = F("pade_extice"),
                     e = F("pade_ssaice"), f = F("pade_asyice"), s1 = F("pade_sizreg_extliq"),
                     s2 = F("pade_sizreg_ssaliq"), s3 = F("pade_sizreg_asyliq"), s4 = F("pade_sizreg_extice"),
                     s5 = F("pade_sizreg_ssaice"), s6 = F("pade_sizreg_asyice");
  return rrtmgpnn_cloud_optics_create_pade(ctx, nband, blw.data(), pe.dims[2], pe.dims[1], m["pade_ssaliq"].dims[0],
                                           pe.dims[0], a.data(), b.data(), c.data(), d.data(), e.data(), f.data(),
                                           s1.data(), s2.data(), s3.data(), s4.data(), s5.data(), s6.data(), co);
}

int rrtmgpnn_cloud_optics_set_ice_roughness(rrtmgpnn_cloud_optics *co, int icergh)
{
  if (!co) return fail(RRTMGPNN_ERR_ARGUMENT, "cloud_optics_set_ice_roughness(): can't set before initialization");
  if (icergh < 1 || icergh > co->nrghice)
    return fail(RRTMGPNN_ERR_ARGUMENT, "cloud optics: cloud ice surface roughness flag is out of bounds");
  co->icergh = icergh;
  return RRTMGPNN_OK;
}

int rrtmgpnn_cloud_optics_get(const rrtmgpnn_cloud_optics *co, int *nband, int *nrghice, float radii[4])
{
  if (!co) return fail(RRTMGPNN_ERR_ARGUMENT, "cloud_optics_get: null handle");
  if (nband) *nband = co->nband;
  if (nrghice) *nrghice = co->nrghice;
  if (radii) {
    radii[0] = co->radliq_lwr; radii[1] = co->radliq_upr; radii[2] = co->radice_lwr; radii[3] = co->radice_upr;
  }
  return RRTMGPNN_OK;
}

int rrtmgpnn_cloud_optics_destroy(rrtmgpnn_cloud_optics *co)
{
  if (!co) return RRTMGPNN_OK;
  if (co->d_tab) {
    (void)hipSetDevice(co->device);
    (void)hipFree(co->d_tab);
  }
  delete co;
  return RRTMGPNN_OK;
}

int rrtmgpnn_cloud_optics_compute(rrtmgpnn_context *ctx, const rrtmgpnn_cloud_optics *co, int ncol, int nlay,
                                  const float *clwp, const float *ciwp, const float *reliq, const float *reice,
                                  float *tau, float *ssa, float *g)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!co || !co->d_tab) return fail(RRTMGPNN_ERR_ARGUMENT, "cloud optics: no data has been initialized");
  if (!clwp || !ciwp || !reliq || !reice || !tau || ncol < 0 || nlay < 0 || (ssa && !g))
    return fail(RRTMGPNN_ERR_ARGUMENT, "cloud optics: bad argument");
  return launch_cloud_optics(ctx, co, ncol, nlay, clwp, ciwp, reliq, reice, tau, ssa, g);
}

int rrtmgpnn_increment_bybnd(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int nband, const int *band_lims_gpt,
                             float *tau_io, float *ssa_io, float *g_io, const float *tau_in, const float *ssa_in,
                             const float *g_in)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!tau_io || !tau_in || ncol < 0 || nlay < 0 || ngpt < 1 || (ssa_io && !g_io) || (ssa_in && !g_in))
    return fail(RRTMGPNN_ERR_ARGUMENT, "increment: bad argument");
  BandArgs b;
  if (int rc = band_args(nband, band_lims_gpt, ngpt, b)) return rc;
  return launch_increment_bybnd(ctx, ncol, nlay, ngpt, &b, tau_io, ssa_io, g_io, tau_in, ssa_in, g_in);
}

int rrtmgpnn_increment(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, float *tau_io, float *ssa_io, float *g_io,
                       const float *tau_in, const float *ssa_in, const float *g_in)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!tau_io || !tau_in || ncol < 0 || nlay < 0 || ngpt < 1 || (ssa_io && !g_io) || (ssa_in && !g_in))
    return fail(RRTMGPNN_ERR_ARGUMENT, "increment: bad argument");
  return launch_increment_bybnd(ctx, ncol, nlay, ngpt, nullptr, tau_io, ssa_io, g_io, tau_in, ssa_in, g_in);
}

int rrtmgpnn_delta_scale_2str(rrtmgpnn_context *ctx, long long n, float *tau, float *ssa, float *g, const float *fwd)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!tau || !ssa || !g || n < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "delta_scale: bad argument");
  return launch_delta_scale(ctx, n, tau, ssa, g, fwd);
}

// ---- heating rates (a-20) ----
int rrtmgpnn_compute_heating_rate(rrtmgpnn_context *ctx, int ncol, int nlay, const float *flux_up, const float *flux_dn,
                                  const float *plev, float *heating_rate)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!flux_up || !flux_dn || !plev || !heating_rate || ncol < 0 || nlay < 1)
    return fail(RRTMGPNN_ERR_ARGUMENT, "heating_rate: bad argument");
  // mo_rrtmgp_constants.F90:50,53
  return launch_heating_rate(ctx, ncol, nlay, 0, 9.80665f, 1004.64f, flux_up, flux_dn, plev, heating_rate);
}

int rrtmgpnn_calc_heating_rate_k_day(rrtmgpnn_context *ctx, int ncol, int nlay, const float *flux_up,
                                     const float *flux_dn, const float *plev, float *hr_k_day)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!flux_up || !flux_dn || !plev || !hr_k_day || ncol < 0 || nlay < 1)
    return fail(RRTMGPNN_ERR_ARGUMENT, "calc_heating_rate: bad argument");
  // scaling = -(24.0_wp * 3600.0_wp * grav / SpecificHeatDryAir), each operation rounded to fp32
  volatile float day = 24.0f * 3600.0f, t = day * 9.80665f;
  const float scaling = -(t / 1004.0f);
  return launch_heating_rate(ctx, ncol, nlay, 1, scaling, 0.0f, flux_up, flux_dn, plev, hr_k_day);
}

int rrtmgpnn_sw_boundary_rfmip(rrtmgpnn_context *ctx, int ngpt, int ncol, const float *solar_source, const float *tsi,
                               const float *sfc_alb, const float *sza, float *toa_flux, float *sfc_alb_gpt, float *mu0)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (ngpt < 1 || ncol < 0 || !solar_source || !tsi || !sfc_alb || !sza || !toa_flux || !sfc_alb_gpt || !mu0)
    return fail(RRTMGPNN_ERR_ARGUMENT, "sw_boundary_rfmip: bad argument");
  return launch_sw_boundary(ctx, ngpt, ncol, solar_source, tsi, sfc_alb, sza, toa_flux, sfc_alb_gpt, mu0);
}

int rrtmgpnn_sw_solver_2stream_rfmip(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                     const float *solar_source, const float *tsi, const float *sfc_alb, const float *sza,
                                     const float *tau, const float *ssa, const float *g, int nbnd,
                                     const int *band_lims_gpt, const float *tau_bnd, const float *ssa_bnd,
                                     const float *g_bnd, float *toa_flux, float *sfc_alb_gpt, float *mu0,
                                     float *flux_up, float *flux_dn, float *flux_dir)
{
  if (int rc = check_ctx(ctx)) return rc;
  if (!solar_source || !tsi || !sfc_alb || !sza || !tau || !ssa || !toa_flux || !sfc_alb_gpt || !mu0 || !flux_up ||
      !flux_dn || !flux_dir || ngpt < 1 || nlay < 1 || ncol < 0 || nbnd < 0 ||
      (nbnd > 0 && (!tau_bnd || !ssa_bnd || !g_bnd)))
    return fail(RRTMGPNN_ERR_ARGUMENT, "sw_solver_2stream_rfmip: bad argument");
  if (ngpt > kSwBoundaryMaxG) return fail(RRTMGPNN_ERR_UNSUPPORTED, "sw_solver_2stream_rfmip: ngpt > 1024");
  const SwBc bc{solar_source, tsi, sfc_alb, sza, toa_flux, sfc_alb_gpt, mu0};
  BandArgs b;
  if (nbnd > 0) {
    if (int rc = band_args(nbnd, band_lims_gpt, ngpt, b)) return rc;
    if (int rc = bands_cover(b, ngpt)) return rc;
  }
  // inc_flux / mu0 / albedos: the scratch arrays, which the solver reads only when it does not form them itself
  return launch_sw_2stream(ctx, ngpt, nlay, ncol, top_at_1, toa_flux, nullptr, tau, ssa, g, mu0, sfc_alb_gpt,
                           sfc_alb_gpt, nbnd > 0 ? &b : nullptr, tau_bnd, ssa_bnd, g_bnd, flux_up, flux_dn, flux_dir,
                           &bc);
}

// ---- data files: RBIN, classic netCDF, netCDF-4 (datafile.cpp) ----
struct rrtmgpnn_file {
  DataFile df;
  std::vector<std::string> names;
};

int rrtmgpnn_file_open(const char *path, rrtmgpnn_file **f)
{
  if (!path || !f) return fail(RRTMGPNN_ERR_ARGUMENT, "file_open: null argument");
  rrtmgpnn_file *h = new rrtmgpnn_file();
  if (int rc = read_data_file(path, h->df)) {
    delete h;
    return rc;
  }
  for (const auto &kv : h->df.vars) h->names.push_back(kv.first);
  *f = h;
  return RRTMGPNN_OK;
}

int rrtmgpnn_file_close(rrtmgpnn_file *f)
{
  delete f;
  return RRTMGPNN_OK;
}

int rrtmgpnn_file_nvars(const rrtmgpnn_file *f, int *nvars)
{
  if (!f || !nvars) return fail(RRTMGPNN_ERR_ARGUMENT, "file_nvars: null argument");
  *nvars = (int)f->names.size();
  return RRTMGPNN_OK;
}

int rrtmgpnn_file_var_name(const rrtmgpnn_file *f, int i, char *name, int len)
{
  if (!f || !name || len < 1 || i < 0 || i >= (int)f->names.size())
    return fail(RRTMGPNN_ERR_ARGUMENT, "file_var_name: bad argument");
  std::snprintf(name, (size_t)len, "%s", f->names[i].c_str());
  return RRTMGPNN_OK;
}

int rrtmgpnn_file_var(const rrtmgpnn_file *f, const char *name, int *dtype, int *ndim, long long *dims)
{
  if (!f || !name) return fail(RRTMGPNN_ERR_ARGUMENT, "file_var: null argument");
  auto it = f->df.vars.find(name);
  if (it == f->df.vars.end()) return fail(RRTMGPNN_ERR_IO, std::string("file: no variable ") + name);
  if (dtype) *dtype = it->second.dtype;
  if (ndim) *ndim = (int)it->second.dims.size();
  if (dims)
    for (size_t k = 0; k < it->second.dims.size(); k++) dims[k] = it->second.dims[k];
  return RRTMGPNN_OK;
}

int rrtmgpnn_file_read(const rrtmgpnn_file *f, const char *name, int dtype, void *out, long long count)
{
  if (!f || !name || !out || count < 0) return fail(RRTMGPNN_ERR_ARGUMENT, "file_read: bad argument");
  auto it = f->df.vars.find(name);
  if (it == f->df.vars.end()) return fail(RRTMGPNN_ERR_IO, std::string("file: no variable ") + name);
  const DataVar &v = it->second;
  if ((long long)v.count() != count) return fail(RRTMGPNN_ERR_ARGUMENT, std::string("file_read: ") + name + ": size mismatch");
  if (dtype == kChar || v.dtype == kChar) {
    if (dtype != v.dtype) return fail(RRTMGPNN_ERR_ARGUMENT, std::string("file_read: ") + name + ": character/numeric mismatch");
    std::memcpy(out, v.data.data(), v.data.size());
  } else if (dtype == kF32) {
    std::vector<float> a = to_float(v);
    std::memcpy(out, a.data(), a.size() * 4);
  } else if (dtype == kI32) {
    std::vector<int> a = to_int(v);
    std::memcpy(out, a.data(), a.size() * 4);
  } else {
    return fail(RRTMGPNN_ERR_ARGUMENT, "file_read: dtype must be 0 (float32), 1 (int32) or 2 (char)");
  }
  return RRTMGPNN_OK;
}

int rrtmgpnn_file_att(const rrtmgpnn_file *f, const char *var, const char *att, char *text, int len)
{
  if (!f || !att || !text || len < 1) return fail(RRTMGPNN_ERR_ARGUMENT, "file_att: bad argument");
  auto it = f->df.atts.find(std::string(var ? var : "") + ":" + att);
  if (it == f->df.atts.end())
    return fail(RRTMGPNN_ERR_IO, std::string("file: no text attribute ") + (var ? var : "") + ":" + att);
  std::snprintf(text, (size_t)len, "%s", it->second.c_str());
  return RRTMGPNN_OK;
}

}  // extern "C"
