/*
 * rrtmgpnn.h -- C ABI of the MI355X-native RTE+RRTMGP-NN hot path.
 *
 * Plain pointers and sizes only (no torch / HIP types in the signatures): this is the
 * boundary the reference's Fortran class layer binds through ISO_C_BINDING
 * (see rte-rrtmgp-nn_amd/fortran/ and INTEGRATION.md).  All arrays use the reference's
 * Fortran column-major layout, g-point fastest:
 *     tau/lay_source/ssa/g      (ngpt, nlay,   ncol)
 *     lev_source                (ngpt, nlay+1, ncol)
 *     sfc_source/sfc_emis_gpt   (ngpt, ncol)
 *     play/tlay/col_dry/gases   (nlay, ncol)        plev/tlev (nlay+1, ncol)
 *     fluxes                    (nlay+1, ncol)
 * Array arguments are DEVICE pointers (hipMalloc'd or torch tensors) unless the comment
 * says "host".  Every call is asynchronous on the context's stream and reentrant across
 * contexts (one context per host thread / OpenMP block, as the reference drivers'
 * `!$OMP PARALLEL firstprivate(...)` loops require, rrtmgp_rfmip_lw.F90:364-367).
 *
 * Return value: RRTMGPNN_OK (0) or an error code; the message of the last failing call on
 * this host thread is rrtmgpnn_last_error().  The reference class layer returns
 * character(len=128) error_msg (empty on success); the Fortran glue maps one to the other.
 */
#ifndef RRTMGPNN_H
#define RRTMGPNN_H

#ifdef __cplusplus
extern "C" {
#endif

#define RRTMGPNN_OK               0
#define RRTMGPNN_ERR_ARGUMENT     1
#define RRTMGPNN_ERR_DEVICE       2
#define RRTMGPNN_ERR_IO           3
#define RRTMGPNN_ERR_UNSUPPORTED  4

#define RRTMGPNN_ACT_LINEAR       0
#define RRTMGPNN_ACT_SOFTSIGN     1
#define RRTMGPNN_ACT_RELU         2
#define RRTMGPNN_ACT_SIGMOID      3
#define RRTMGPNN_ACT_HARD_SIGMOID 4

typedef struct rrtmgpnn_context rrtmgpnn_context;
typedef struct rrtmgpnn_network rrtmgpnn_network;
typedef struct rrtmgpnn_cloud_optics rrtmgpnn_cloud_optics;
typedef struct rrtmgpnn_file rrtmgpnn_file;

/* ---- runtime ------------------------------------------------------------------------------ */
int         rrtmgpnn_version(void);
const char *rrtmgpnn_last_error(void);
/* Creates a context on `device` that enqueues on `hip_stream` (a hipStream_t; NULL = the legacy default
 * stream, ordered with every other default-stream operation). */
int rrtmgpnn_context_create(int device, void *hip_stream, rrtmgpnn_context **ctx);
int rrtmgpnn_context_destroy(rrtmgpnn_context *ctx);
int rrtmgpnn_context_set_stream(rrtmgpnn_context *ctx, void *hip_stream);
/* MI355X tuning, no reference counterpart: which SW two-stream kernel rrtmgpnn_sw_solver_2stream* launch.
 * 0 (default): mode 3 when ngpt is even, one g-point per lane otherwise.  1: one g-point per lane.  2: two g-points
 * per lane (packed fp32, two columns per block) with per-level workspace planes.  3: two g-points per lane with
 * checkpointed passes (beam / adding state stored every 3 levels instead of per level).  2 and 3 need even ngpt.
 * All kernels give bit-identical fluxes.  ctx == NULL sets the default of every context not set itself. */
int rrtmgpnn_context_set_sw_kernel(rrtmgpnn_context *ctx, int mode);
/* MI355X tuning, no reference counterpart: the MFMA tiling of the gas-optics networks (rrtmgpnn_predict_nn_lw/_sw,
 * rrtmgpnn_gas_optics_lw_nn/_sw_nn).  0 (default): v_mfma_f32_32x32x2_f32 tiles where an instance exists for the
 * networks (the shipped LW g256 pair, LW g128 single model and SW g224 pair, softsign/softsign/linear), 16x16x4
 * otherwise.  1: 16x16x4 tiles.
 * Bit-identical outputs either way.  ctx == NULL sets the default of every context not set itself. */
int rrtmgpnn_context_set_mlp_kernel(rrtmgpnn_context *ctx, int mode);
/* MI355X tuning, no reference counterpart: the gas-optics networks launched on this context use at most `cus` CUs'
 * worth of resident blocks (0, the default: every CU).  For a host that runs the LW and SW chains side by side on two
 * streams: an LW network confined to part of the chip leaves the other CUs to the SW solver from its start (each LW
 * network block holds a whole CU's LDS).  Bit-identical outputs. */
int rrtmgpnn_context_set_mlp_max_cus(rrtmgpnn_context *ctx, int cus);
/* The cap rrtmgpnn_context_set_mlp_max_cus left in force on this context (0: every CU). */
int rrtmgpnn_context_get_mlp_max_cus(rrtmgpnn_context *ctx, int *cus);
void *rrtmgpnn_context_stream(rrtmgpnn_context *ctx);
int rrtmgpnn_context_synchronize(rrtmgpnn_context *ctx);
/* The context's device workspace grows on demand.  A call issued while the context's stream is captured into a
 * hipGraph pins it (the graph holds its address): later calls that would need more fail with RRTMGPNN_ERR_ARGUMENT
 * instead of freeing memory the graph writes.  Unpin after destroying the graph (no reference counterpart). */
int rrtmgpnn_context_unpin_workspace(rrtmgpnn_context *ctx);
/* Device memory helpers for hosts without their own allocator (Fortran glue). */
int rrtmgpnn_malloc(rrtmgpnn_context *ctx, long long bytes, void **dptr);
int rrtmgpnn_free(rrtmgpnn_context *ctx, void *dptr);
int rrtmgpnn_memcpy_h2d(rrtmgpnn_context *ctx, void *dst, const void *src, long long bytes);
int rrtmgpnn_memcpy_d2h(rrtmgpnn_context *ctx, void *dst, const void *src, long long bytes);
/* A context whose work runs on a stream it creates and owns (non-blocking), so host threads with a context each
 * (OpenMP over blocks, rrtmgp_rfmip_lw.F90:364-367) run concurrently on the device.  No reference counterpart. */
int rrtmgpnn_context_create_owned(int device, rrtmgpnn_context **ctx);

/* ---- Device data environment of a context: the OpenACC data regions of the reference's GPU build ----
 * The reference keeps optical properties, sources and gas concentrations on the device between calls with
 * `!$acc enter data create/copyin` (ty_gas_concs%set_vmr, rrtmgp/mo_gas_concentrations.F90:166; the optical-property
 * and source constructors, examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:325-327; gas_optics,
 * rrtmgp/mo_gas_optics_rrtmgp.F90:281-426) and `!$acc update host` / `exit data delete`.  Here a context maps a
 * host array (its address and size) to a device copy from the context's pool, with a state: host newer, both
 * current, device newer.  All transfers are ordered on the context's stream; a context serves one host thread.
 * rrtmgpnn_present: the device copy of host[0, bytes); mode RRTMGPNN_PRESENT_READ uploads it first when the host
 *   copy is newer (created on first use, `copyin`); RRTMGPNN_PRESENT_WRITE marks the device copy newer (the caller's
 *   kernel writes it; `create`); both bits: upload if needed, then device newer.  A different size for the same
 *   address replaces the entry (host newer).
 * rrtmgpnn_present_update_host: copy a device-newer array back (`!$acc update host`) and wait for it.
 * rrtmgpnn_present_update_device: the host copy changed: it is uploaded at its next READ (`!$acc update device`),
 *   in every context of the process (the reference's OpenACC data environment is process-wide).
 * rrtmgpnn_present_delete: drop the entry (its buffer returns to the pool; `!$acc exit data delete`); no-op if absent.
 *   Every other context's copy of that host array is stale from then on and is uploaded again at its next READ.
 * Cross-thread contract of update_device / delete: the host copy wins in every context.  A copy another context holds
 *   as device newer (a kernel result not yet copied back with update_host) is discarded too; a thread that still needs
 *   such a result must update_host it before any thread updates or deletes the same host array.  The process-wide
 *   generation table behind this keeps one 16-byte entry per host address ever updated or deleted (bounded by the
 *   distinct addresses the host program's allocator hands out).
 * rrtmgpnn_stage_h2d / rrtmgpnn_scratch / rrtmgpnn_release: stream-ordered per-call buffers from the same pool
 *   (a call's inputs copied in, its intermediates); released buffers are reused by later work on the stream.
 * rrtmgpnn_copy_d2h / rrtmgpnn_copy_h2d / rrtmgpnn_copy_d2d: enqueue a copy on the context's stream (the device side complete after
 *   rrtmgpnn_context_synchronize; the host buffer of an H2D copy may be reused on return).
 * rrtmgpnn_memset_async: bytes of a device buffer set to `value`, on the context's stream. */
#define RRTMGPNN_PRESENT_READ  1
#define RRTMGPNN_PRESENT_WRITE 2
int rrtmgpnn_present(rrtmgpnn_context *ctx, const void *host, long long bytes, int mode, void **dptr);
int rrtmgpnn_present_update_host(rrtmgpnn_context *ctx, void *host);
int rrtmgpnn_present_update_device(rrtmgpnn_context *ctx, const void *host);
int rrtmgpnn_present_delete(rrtmgpnn_context *ctx, const void *host);
int rrtmgpnn_stage_h2d(rrtmgpnn_context *ctx, const void *host, long long bytes, void **dptr);
int rrtmgpnn_scratch(rrtmgpnn_context *ctx, long long bytes, void **dptr);
int rrtmgpnn_release(rrtmgpnn_context *ctx, void *dptr);
int rrtmgpnn_copy_d2h(rrtmgpnn_context *ctx, void *host, const void *dptr, long long bytes);
int rrtmgpnn_copy_h2d(rrtmgpnn_context *ctx, void *dptr, const void *host, long long bytes);
int rrtmgpnn_copy_d2d(rrtmgpnn_context *ctx, void *dst, const void *src, long long bytes);
int rrtmgpnn_memset_async(rrtmgpnn_context *ctx, void *dptr, int value, long long bytes);

/* ---- neural networks: replaces rrtmgp_network_type (neural/mod_network_rrtmgp.F90:34-122) ---- */
/* Load an RBIN model file (converted from the reference's netCDF model files). */
int rrtmgpnn_network_load(rrtmgpnn_context *ctx, const char *path, rrtmgpnn_network **net);
/* Build from host arrays.  weights[n] is layer n's kernel, (dims[n], dims[n+1]) C-order
 * (= the netCDF variable nn_weights_<n+1> = the reference's w_transposed memory).
 * output_mean/std may be NULL (Planck-fraction models). */
int rrtmgpnn_network_create(rrtmgpnn_context *ctx, int nlayers, const int *dims, const int *activations,
                            const float *const *weights, const float *const *biases,
                            const float *input_min, const float *input_max,
                            const float *output_mean, const float *output_std,
                            const char *input_names /* nx*32 chars, space padded, may be NULL */,
                            rrtmgpnn_network **net);
int rrtmgpnn_network_destroy(rrtmgpnn_network *net);
/* host outputs */
int rrtmgpnn_network_get_dims(const rrtmgpnn_network *net, int *nlayers, int dims[8]);
int rrtmgpnn_network_get_input_name(const rrtmgpnn_network *net, int i, char *buf, int buflen);
int rrtmgpnn_network_get_input_scaling(const rrtmgpnn_network *net, float *input_min, float *input_max);

/* ---- gas-optics kernels --------------------------------------------------------------------- */
/* compute_nn_inputs (rrtmgp/mo_gas_optics_rrtmgp.F90:618-798).  gas_conc[k] (k>=2) is a device
 * pointer to the concentration of input k with gas_ndims[k] in {0:(1), 1:(nlay), 2:(nlay,ncol)},
 * or NULL when the gas is absent (reference uses ref_vmr = 0, :757-758).  Entries 0,1 ignored.
 * gas_conc/gas_ndims are HOST arrays of length ninputs (<= 32).  nn_inputs (ninputs,nlay,ncol). */
int rrtmgpnn_compute_nn_inputs(rrtmgpnn_context *ctx, int ncol, int nlay, int ninputs,
                               const float *play, const float *tlay,
                               const float *const *gas_conc, const int *gas_ndims,
                               const rrtmgpnn_network *net, float *nn_inputs);
/* get_col_dry (rrtmgp/mo_gas_optics_rrtmgp.F90:1662-1707), g0 = grav. */
int rrtmgpnn_get_col_dry(rrtmgpnn_context *ctx, int ncol, int nlay, const float *vmr_h2o, const float *plev,
                         float *col_dry);
/* Level temperatures from layers (rrtmgp/mo_gas_optics_rrtmgp.F90:317-337). */
int rrtmgpnn_interpolate_tlev(rrtmgpnn_context *ctx, int ncol, int nlay, const float *play, const float *plev,
                              const float *tlay, float *tlev);
/* predict_nn_lw_blas (rrtmgp/kernels/mo_gas_optics_kernels.F90:690-774).  nnets == 2: nets[0] =
 * absorption (tau = (std*y+mean)^8 * col_dry), nets[1] = Planck fraction (pfrac = y^2);
 * nnets == 1: single "both" model with 2*ngpt outputs (:744-772). */
int rrtmgpnn_predict_nn_lw(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs,
                           const float *nn_inputs, const float *col_dry,
                           const rrtmgpnn_network *const *nets, int nnets, float *tau, float *pfrac);
/* predict_nn_sw_blas (:869-953) with INLINE_COMBINE: nets[0] absorption, nets[1] Rayleigh.
 * ssa == NULL -> tau = tau_abs only (1scl).  Otherwise tau = tau_abs + tau_ray, ssa = tau_ray/tau.
 * g != NULL -> zero-filled as gas_optics_ext does (mo_gas_optics_rrtmgp.F90:560-567). */
int rrtmgpnn_predict_nn_sw(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs,
                           const float *nn_inputs, const float *col_dry,
                           const rrtmgpnn_network *const *nets, float *tau, float *ssa, float *g);
/* Fused gas optics, NN path (MI355X): compute_nn_inputs + get_col_dry + predict_nn_lw in one kernel.  The network
 * inputs and the dry-air column amounts are formed per sample inside the MLP kernel with the expressions of
 * rrtmgpnn_compute_nn_inputs and rrtmgpnn_get_col_dry, so nn_inputs and col_dry never touch HBM; tau and pfrac are
 * bit-identical to the three separate calls (gas_optics_int's NN branch, rrtmgp/mo_gas_optics_rrtmgp.F90:342-391).
 * Arguments as those calls' (gas_conc / gas_ndims HOST arrays; vmr_h2o the h2o vmr get_col_dry reads).  Networks
 * without an in-kernel instance run the three kernels (nn_inputs and col_dry in the context workspace). */
int rrtmgpnn_gas_optics_lw_nn(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs, const float *play,
                              const float *tlay, const float *plev, const float *vmr_h2o,
                              const float *const *gas_conc, const int *gas_ndims,
                              const rrtmgpnn_network *const *nets, int nnets, float *tau, float *pfrac);
/* The same for the shortwave: compute_nn_inputs + get_col_dry + predict_nn_sw (gas_optics_ext's NN branch,
 * mo_gas_optics_rrtmgp.F90:433-602); ssa / g as rrtmgpnn_predict_nn_sw. */
int rrtmgpnn_gas_optics_sw_nn(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int ninputs, const float *play,
                              const float *tlay, const float *plev, const float *vmr_h2o,
                              const float *const *gas_conc, const int *gas_ndims,
                              const rrtmgpnn_network *const *nets, float *tau, float *ssa, float *g);
/* Generic MLP forward (network_type%output_sgemm_flat, neural/mod_network.F90:273-354):
 * out(ny, nbatch) = net(x(nx, nbatch)), last-layer activation applied, no post-processing. */
int rrtmgpnn_network_forward(rrtmgpnn_context *ctx, const rrtmgpnn_network *net, long long nbatch,
                             const float *x, float *out);
/* compute_Planck_source_nn (rrtmgp/kernels/mo_gas_optics_kernels.F90:615-683).  sfc_lay 1-based.
 * band_lims_gpt: HOST (2,nbnd) 1-based.  totplnk: DEVICE (nPlanckTemp, nbnd).
 * pfrac is overwritten with lay_source. */
int rrtmgpnn_compute_planck_source_nn(rrtmgpnn_context *ctx, int ncol, int nlay, int nbnd, int ngpt,
                                      int nPlanckTemp, const float *tlay, const float *tlev, const float *tsfc,
                                      int sfc_lay, const int *band_lims_gpt, float temp_ref_min,
                                      float totplnk_delta, const float *totplnk, float *sfc_source,
                                      float *sfc_source_Jac, float *pfrac, float *lev_source);

/* ---- RTE solvers ---------------------------------------------------------------------------- */
/* lw_solver_noscat_GaussQuad (rte/kernels/mo_rte_solver_kernels.F90:332-415) without rescaling or
 * Jacobians.  Ds, weights: HOST arrays of nmus (<= 4) entries.  inc_flux may be NULL (zero). */
int rrtmgpnn_lw_solver_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                              const float *Ds, const float *weights, const float *inc_flux,
                              const float *tau, const float *lay_source, const float *lev_source,
                              const float *sfc_emis_gpt, const float *sfc_source,
                              float *flux_up, float *flux_dn);
/* Fused clear-sky LW entry: compute_Planck_source_nn (rrtmgp/kernels/mo_gas_optics_kernels.F90:615-683)
 * + lw_solver_noscat_GaussQuad in one kernel.  Takes the Planck fraction (what predict_nn_lw writes into
 * lay_source) instead of lay/lev/sfc sources, forms every source in-kernel with the same products as
 * rrtmgpnn_compute_planck_source_nn, and never stores them: fluxes are bit-identical to
 * compute_planck_source_nn followed by lw_solver_noscat.  band_lims_gpt HOST (2,nbnd); totplnk DEVICE.
 * emis_by_band == 0: sfc_emis is (ngpt, ncol) per g-point; 1: (nbnd, ncol) by band, as rte_lw takes it, expanded
 * in-kernel (expand, rte/mo_rte_lw.F90:429-447: the same values, no band-to-g-point array in HBM). */
int rrtmgpnn_lw_solver_noscat_planck(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                     const float *Ds, const float *weights, const float *inc_flux, const float *tau,
                                     const float *pfrac, int nbnd, int nPlanckTemp, const float *tlay,
                                     const float *tlev, const float *tsfc, int sfc_lay, const int *band_lims_gpt,
                                     float temp_ref_min, float totplnk_delta, const float *totplnk,
                                     int emis_by_band, const float *sfc_emis, float *flux_up, float *flux_dn);
/* rrtmgpnn_lw_solver_noscat_planck with the atmosphere incremented by a band-resolved absorption optical depth
 * tau_bnd (nbnd, nlay, ncol), e.g. cloud optics: the same fluxes as rrtmgpnn_increment_bybnd (1scl by 1scl)
 * followed by rrtmgpnn_lw_solver_noscat_planck, but the g-point tau array is only read (it is left as it was). */
int rrtmgpnn_lw_solver_noscat_planck_inc(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                         int nmus, const float *Ds, const float *weights, const float *inc_flux,
                                         const float *tau, const float *tau_bnd, const float *pfrac, int nbnd,
                                         int nPlanckTemp, const float *tlay, const float *tlev, const float *tsfc,
                                         int sfc_lay, const int *band_lims_gpt, float temp_ref_min,
                                         float totplnk_delta, const float *totplnk, int emis_by_band,
                                         const float *sfc_emis, float *flux_up, float *flux_dn);
/* rte_lw on two-stream optical properties, default branch (rte/mo_rte_lw.F90:372-387): lw_solver_noscat_GaussQuad
 * with do_rescaling -- tau scaled by (1 - ssa + ssa(1-g)/2), a no-scattering pass down, then
 * lw_transport_1rescl up and down again with the adjustment terms (rte/kernels/mo_rte_solver_kernels.F90:209-233,
 * 1729-1795).  Arguments as rrtmgpnn_lw_solver_noscat plus ssa, g (ngpt, nlay, ncol). */
int rrtmgpnn_lw_solver_1rescl(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                              const float *Ds, const float *weights, const float *inc_flux, const float *tau,
                              const float *ssa, const float *g, const float *lay_source, const float *lev_source,
                              const float *sfc_emis_gpt, const float *sfc_source, float *flux_up, float *flux_dn);
/* rte_lw(..., use_2stream=.true.): lw_solver_2stream (rte/kernels/mo_rte_solver_kernels.F90:426-486) with
 * lw_two_stream (:1018-1069), lw_source_2str (:1112-1162) and adding (:1526-1637).  inc_flux (ngpt, ncol) is a flux
 * (NULL: zero); the layer sources are not used (as in the reference).  Broadband sums are sequential over g
 * (sum_broadband_nocol). */
int rrtmgpnn_lw_solver_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                               const float *inc_flux, const float *tau, const float *ssa, const float *g,
                               const float *lev_source, const float *sfc_emis_gpt, const float *sfc_source,
                               float *flux_up, float *flux_dn);
/* sw_solver_2stream (:541-692).  inc_flux_dif may be NULL (zero, rte/mo_rte_sw.F90:197-210).
 * g may be NULL: asymmetry parameter identically zero, as gas_optics_ext's NN branch produces
 * (mo_gas_optics_rrtmgp.F90:560-567) -- same fluxes as passing a zero-filled array. */
int rrtmgpnn_sw_solver_2stream(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                               const float *inc_flux, const float *inc_flux_dif,
                               const float *tau, const float *ssa, const float *g, const float *mu0,
                               const float *sfc_alb_dir_gpt, const float *sfc_alb_dif_gpt,
                               float *flux_up, float *flux_dn, float *flux_dir);
/* The solvers above with the outputs of ty_fluxes_flexible (rte/mo_fluxes.F90:57-67) and rte_lw's lw_Ds
 * (rte/mo_rte_lw.F90:80-81, 239-246, 329-341).  gpt_flux_* (ngpt, nlay+1, ncol) device arrays, NULL for none.
 * LW: both or neither of gpt_flux_up/dn; with one angle they receive the g-point RADIANCES and the broadband fluxes
 * are reduced from them as lw_solver_noscat does (quirk B-5), with several angles the angle-summed fluxes.  lw_Ds
 * (NULL: the Gauss angles): ngpt*ncol column-dependent secants read as D(igpt, icol) -- the kernel's layout; the
 * reference's rte_lw checks the extents as (ncol, ngpt) but passes the array unchanged (quirk B-12) -- with one angle
 * (nmus must be 1) of weight weights[0].  SW: all three of up, down (TOTAL: diffuse + direct, as the reference
 * stores it) and direct, and the broadband down flux summed from the total (the reference's save_gpt_flux order,
 * :660-684); even ngpt.  Bit-identical to the reference (tests/test_oracle.py, tests/test_gpu_gpt.py). */
int rrtmgpnn_lw_solver_noscat_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                  const float *Ds, const float *weights, const float *lw_Ds, const float *inc_flux,
                                  const float *tau, const float *lay_source, const float *lev_source,
                                  const float *sfc_emis_gpt, const float *sfc_source, float *flux_up, float *flux_dn,
                                  float *gpt_flux_up, float *gpt_flux_dn);
int rrtmgpnn_lw_solver_noscat_planck_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                         const float *Ds, const float *weights, const float *lw_Ds,
                                         const float *inc_flux, const float *tau, const float *pfrac, int nbnd,
                                         int nPlanckTemp, const float *tlay, const float *tlev, const float *tsfc,
                                         int sfc_lay, const int *band_lims_gpt, float temp_ref_min,
                                         float totplnk_delta, const float *totplnk, int emis_by_band,
                                         const float *sfc_emis, float *flux_up, float *flux_dn, float *gpt_flux_up,
                                         float *gpt_flux_dn);
int rrtmgpnn_sw_solver_2stream_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                   const float *inc_flux, const float *inc_flux_dif, const float *tau,
                                   const float *ssa, const float *g, const float *mu0, const float *sfc_alb_dir_gpt,
                                   const float *sfc_alb_dif_gpt, float *flux_up, float *flux_dn, float *flux_dir,
                                   float *gpt_flux_up, float *gpt_flux_dn, float *gpt_flux_dir);
/* rte_sw on absorption-only (1scl) properties (rte/mo_rte_sw.F90:213-222): apply_BC_factor (top level =
 * inc_flux * mu0, rte/kernels/mo_rte_solver_kernels.F90:1685-1704) and sw_solver_noscat (:496-532), broadband direct
 * flux (nlay+1, ncol) = sum over g of each column's direct beam (sum_broadband_nocol, sequential).  The reference's
 * rte_sw swaps the spectral and broadband arguments of sw_solver_noscat (quirk B-10) and the kernel sums column 1 for
 * every column (B-11): this entry follows the kernels' evident meaning; the spectral beam is the reference's bit for
 * bit (tests/test_oracle.py).  inc_flux (ngpt, ncol), tau (ngpt, nlay, ncol), mu0 (ncol). */
int rrtmgpnn_sw_solver_noscat(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                              const float *tau, const float *mu0, float *flux_dir);
/* The scattering LW solvers and the SW direct beam with ty_fluxes_flexible's g-point outputs (ngpt, nlay+1, ncol),
 * both or neither of gpt_flux_up/dn for LW.
 * 1rescl: what lw_solver_noscat_GaussQuad leaves in flux_up_gpt/flux_dn_gpt with do_rescaling (rte/mo_rte_lw.F90:
 *   377-387; kernels :179-281, 383-411): with one angle the radiances of the final up and down passes (quirk B-5),
 *   with several the angle-summed fluxes.
 * 2stream: the adding fluxes lw_solver_2stream forms per g-point (:454-485).
 * noscat (SW, 1scl): the spectral direct beam, top level = inc_flux * mu0 (apply_BC_factor + sw_solver_noscat; the
 *   reference's rte_sw passes a local array to apply_BC_factor when g-point fluxes are desired, :155-163, 218: this
 *   entry applies the boundary condition to the caller's array, the evident meaning, as for B-10/B-11).
 * Broadband outputs as the entries above, bit for bit (tests/test_gpu_gpt.py). */
int rrtmgpnn_lw_solver_1rescl_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                  const float *Ds, const float *weights, const float *inc_flux, const float *tau,
                                  const float *ssa, const float *g, const float *lay_source, const float *lev_source,
                                  const float *sfc_emis_gpt, const float *sfc_source, float *flux_up, float *flux_dn,
                                  float *gpt_flux_up, float *gpt_flux_dn);
int rrtmgpnn_lw_solver_2stream_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                   const float *inc_flux, const float *tau, const float *ssa, const float *g,
                                   const float *lev_source, const float *sfc_emis_gpt, const float *sfc_source,
                                   float *flux_up, float *flux_dn, float *gpt_flux_up, float *gpt_flux_dn);
int rrtmgpnn_sw_solver_noscat_gpt(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                  const float *inc_flux, const float *tau, const float *mu0, float *flux_dir,
                                  float *gpt_flux_dir);
/* rrtmgpnn_sw_solver_2stream of the atmosphere incremented by band-resolved two-stream properties
 * (tau, ssa, g)_bnd (nbnd, nlay, ncol) -- clouds%increment(atmos) (inc_2stream_by_2stream_bybnd,
 * rte/kernels/mo_optical_props_kernels.F90:430-463) fused into the solver: same fluxes, bit for bit, as
 * rrtmgpnn_increment_bybnd then rrtmgpnn_sw_solver_2stream; the inputs are left unchanged.  g may be NULL
 * (zero).  band_lims_gpt HOST (2, nbnd) and must put every g-point in a band. */
int rrtmgpnn_sw_solver_2stream_inc(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                   const float *inc_flux, const float *inc_flux_dif, const float *tau,
                                   const float *ssa, const float *g, int nbnd, const int *band_lims_gpt,
                                   const float *tau_bnd, const float *ssa_bnd, const float *g_bnd, const float *mu0,
                                   const float *sfc_alb_dir_gpt, const float *sfc_alb_dif_gpt, float *flux_up,
                                   float *flux_dn, float *flux_dir);
/* expand (rte/mo_rte_lw.F90:429-447): (nband,ncol) -> (ngpt,ncol).  band_lims_gpt HOST (2,nband). */
int rrtmgpnn_expand_band_to_gpt(rrtmgpnn_context *ctx, int nband, int ngpt, int ncol, const int *band_lims_gpt,
                                const float *arr_in, float *arr_out);

/* ---- all-sky: cloud optics, increment, delta scaling ------------------ */
/* ty_cloud_optics%load, LUT form (extensions/cloud_optics/mo_cloud_optics.F90:load_lut).  HOST arrays in the
 * coefficient file's Fortran layout: liquid (nsize_liq, nband), ice (nsize_ice, nband, nrghice).
 * band_lims_wvn (2, nband) may be NULL.  Ice roughness starts at 1 (set_ice_roughness). */
int rrtmgpnn_cloud_optics_create_lut(rrtmgpnn_context *ctx, int nband, const float *band_lims_wvn, int nsize_liq,
                                     int nsize_ice, int nrghice, float radliq_lwr, float radliq_upr,
                                     float radice_lwr, float radice_upr, const float *lut_extliq,
                                     const float *lut_ssaliq, const float *lut_asyliq, const float *lut_extice,
                                     const float *lut_ssaice, const float *lut_asyice, rrtmgpnn_cloud_optics **co);
/* Pade form (load_pade): coefficients (nband, nsizereg, ncoef[, nrghice]) with ncoef_ext = 6 ([2/3]
 * approximants) and ncoef_ssa = 5 ([2/2]); size-regime bounds (nsizereg + 1) each; nsizereg must be 3. */
int rrtmgpnn_cloud_optics_create_pade(rrtmgpnn_context *ctx, int nband, const float *band_lims_wvn, int nsizereg,
                                      int ncoef_ext, int ncoef_ssa, int nrghice, const float *pade_extliq,
                                      const float *pade_ssaliq, const float *pade_asyliq, const float *pade_extice,
                                      const float *pade_ssaice, const float *pade_asyice,
                                      const float *sizreg_extliq, const float *sizreg_ssaliq,
                                      const float *sizreg_asyliq, const float *sizreg_extice,
                                      const float *sizreg_ssaice, const float *sizreg_asyice,
                                      rrtmgpnn_cloud_optics **co);
/* Load the RBIN conversion of rrtmgp-cloud-optics-coeffs-{lw,sw}.nc; use_lut selects the method. */
int rrtmgpnn_cloud_optics_load(rrtmgpnn_context *ctx, const char *path, int use_lut, rrtmgpnn_cloud_optics **co);
int rrtmgpnn_cloud_optics_set_ice_roughness(rrtmgpnn_cloud_optics *co, int icergh);
/* host outputs: nband, nrghice, radii = {liq min, liq max, ice min, ice max} (get_min/max_radius_*) */
int rrtmgpnn_cloud_optics_get(const rrtmgpnn_cloud_optics *co, int *nband, int *nrghice, float radii[4]);
int rrtmgpnn_cloud_optics_destroy(rrtmgpnn_cloud_optics *co);
/* cloud_optics (:354-535): clwp, ciwp, reliq, reice (nlay, ncol) -> by band (nband, nlay, ncol).
 * ssa == NULL: 1scl, tau = absorption optical depth; otherwise 2str (tau, ssa, g; g required). */
int rrtmgpnn_cloud_optics_compute(rrtmgpnn_context *ctx, const rrtmgpnn_cloud_optics *co, int ncol, int nlay,
                                  const float *clwp, const float *ciwp, const float *reliq, const float *reice,
                                  float *tau, float *ssa, float *g);
/* ty_optical_props_arry%increment of g-point properties (ngpt, nlay, ncol) by band-resolved ones
 * (nband, nlay, ncol) (rte/mo_optical_props.F90:882-1023, inc_*_bybnd).  ssa_io == NULL: 1scl target;
 * ssa_in == NULL: 1scl increment.  band_lims_gpt HOST (2, nband). */
int rrtmgpnn_increment_bybnd(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, int nband, const int *band_lims_gpt,
                             float *tau_io, float *ssa_io, float *g_io, const float *tau_in, const float *ssa_in,
                             const float *g_in);
/* Same-resolution increment (increment_*_by_*, rte/kernels/mo_optical_props_kernels.F90:109-219):
 * both sets (ngpt, nlay, ncol); NULL ssa as above. */
int rrtmgpnn_increment(rrtmgpnn_context *ctx, int ncol, int nlay, int ngpt, float *tau_io, float *ssa_io, float *g_io,
                       const float *tau_in, const float *ssa_in, const float *g_in);
/* Heating rate [K/s] per layer, compute_heating_rate (extensions/mo_heating_rates.F90:26-53): grav = 9.80665,
 * cp_dry = 1004.64 (rrtmgp/mo_rrtmgp_constants.F90:50,53).  The extension predates this fork's layout; here fluxes and
 * plev are the fork's (nlay+1, ncol), level fastest, and heating_rate is (nlay, ncol). */
int rrtmgpnn_compute_heating_rate(rrtmgpnn_context *ctx, int ncol, int nlay, const float *flux_up, const float *flux_dn,
                                  const float *plev, float *heating_rate);
/* Heating rate [K/day] as the NN evaluation programs report it, calc_heating_rate
 * (examples/rrtmgp-nn-training/rrtmgp_lw_eval_nn_rfmip.F90:624-653): cp = 1004, -(86400 g / cp) d(F_dn - F_up) / dp.
 * Same layouts as rrtmgpnn_compute_heating_rate. */
int rrtmgpnn_calc_heating_rate_k_day(rrtmgpnn_context *ctx, int ncol, int nlay, const float *flux_up,
                                     const float *flux_dn, const float *plev, float *hr_k_day);
/* The RFMIP SW driver's per-block boundary conditions (examples/rfmip-clear-sky/rrtmgp_rfmip_sw.F90:403-434), with
 * gas_optics_ext's toa_src(igpt, icol) = solar_source(igpt) (rrtmgp/mo_gas_optics_rrtmgp.F90:594-599): per column
 * def_tsi = sum over g of toa_src in g order, toa_flux = toa_src * tsi / def_tsi, sfc_alb_gpt(g, icol) = sfc_alb(icol),
 * mu0 = merge(cos(sza * deg_to_rad), 1, usecol), usecol = sza < 90 - 2 spacing(90) (:236-238), cos with glibc's cosf
 * algorithm (the reference built here links it).  solar_source DEVICE (ngpt) after set_tsi; tsi, sfc_alb, sza DEVICE
 * (ncol); outputs DEVICE toa_flux and sfc_alb_gpt (ngpt, ncol), mu0 (ncol). */
int rrtmgpnn_sw_boundary_rfmip(rrtmgpnn_context *ctx, int ngpt, int ncol, const float *solar_source, const float *tsi,
                               const float *sfc_alb, const float *sza, float *toa_flux, float *sfc_alb_gpt, float *mu0);
/* rrtmgpnn_sw_boundary_rfmip followed by rrtmgpnn_sw_solver_2stream (nbnd == 0) or rrtmgpnn_sw_solver_2stream_inc
 * (nbnd > 0; band_lims_gpt, tau_bnd, ssa_bnd, g_bnd as there), with no diffuse incident flux and the albedo given for
 * both the direct and the diffuse beam, as the RFMIP and all-sky drivers call rte_sw (rrtmgp_rfmip_sw.F90:403-441):
 * the same fluxes, bit for bit.  The checkpointed solver forms the boundary conditions in its prologue (no separate
 * launch); the other solver kernels read them from toa_flux, sfc_alb_gpt and mu0 (DEVICE scratch, (ngpt, ncol),
 * (ngpt, ncol), (ncol); contents unspecified after the call). */
int rrtmgpnn_sw_solver_2stream_rfmip(rrtmgpnn_context *ctx, int ngpt, int nlay, int ncol, int top_at_1,
                                     const float *solar_source, const float *tsi, const float *sfc_alb, const float *sza,
                                     const float *tau, const float *ssa, const float *g, int nbnd,
                                     const int *band_lims_gpt, const float *tau_bnd, const float *ssa_bnd,
                                     const float *g_bnd, float *toa_flux, float *sfc_alb_gpt, float *mu0,
                                     float *flux_up, float *flux_dn, float *flux_dir);
/* ty_optical_props_2str%delta_scale([for]) (rte/mo_optical_props.F90:576-604; kernels
 * rte/kernels/mo_optical_props_kernels.F90:41-92) on n values in place.  fwd == NULL: f = g**2. */
int rrtmgpnn_delta_scale_2str(rrtmgpnn_context *ctx, long long n, float *tau, float *ssa, float *g, const float *fwd);

/* ---- data files ---------------------------------------------------------
 * Native readers for the files the path consumes, replacing the netCDF-Fortran calls of
 * neural/mod_network_rrtmgp.F90:58-122 (load_netcdf), examples/all-sky/mo_load_cloud_coefficients.F90 and
 * examples/rfmip-clear-sky/mo_rfmip_io.F90: classic netCDF (CDF-1/2/5, parsed natively), netCDF-4 (HDF5,
 * through libhdf5 bound at run time: RRTMGPNN_HDF5_LIB or the loader path) and this repository's RBIN.
 * rrtmgpnn_network_load and rrtmgpnn_cloud_optics_load accept all three.  A file is read whole on open;
 * dims are in file (C) order; dtype 0 float32 (floating-point variables, doubles rounded), 1 int32,
 * 2 char.  Variable-length strings and netCDF-4 dimension-only scales are not exposed.  Host memory only. */
int rrtmgpnn_file_open(const char *path, rrtmgpnn_file **f);
int rrtmgpnn_file_close(rrtmgpnn_file *f);
int rrtmgpnn_file_nvars(const rrtmgpnn_file *f, int *nvars);
int rrtmgpnn_file_var_name(const rrtmgpnn_file *f, int i, char *name, int len);
/* dims: room for 8 entries */
int rrtmgpnn_file_var(const rrtmgpnn_file *f, const char *name, int *dtype, int *ndim, long long *dims);
/* count = number of elements; numeric variables convert to the requested dtype (0 or 1) */
int rrtmgpnn_file_read(const rrtmgpnn_file *f, const char *name, int dtype, void *out, long long count);
/* text attribute `att` of variable `var` (NULL or "": global) */
int rrtmgpnn_file_att(const rrtmgpnn_file *f, const char *var, const char *att, char *text, int len);

#ifdef __cplusplus
}
#endif
#endif /* RRTMGPNN_H */
