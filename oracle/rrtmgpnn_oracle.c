/*
 * rrtmgpnn_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C99, float32 like the reference's default wp = c_float,
 * rte/mo_rte_kind.F90:29-33) of the RTE+RRTMGP-NN hot path.  It is the parity
 * checker for the HIP kernels and the "port" CPU baseline in bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product (rte-rrtmgp-nn_amd/) never does.
 *
 * Parity of this restatement is pinned against the reference itself:
 *   - RTE solvers (lw_solver_noscat[_GaussQuad], sw_solver_2stream, adding) and
 *     the MLP chain (network_type%output_sgemm_flat + MKL sgemm) are compiled
 *     from /root/reference sources by oracle/Makefile.ref into oracle/_ref/
 *     and compared in tests/test_oracle_vs_reference.py (container only); the
 *     comparison's outputs are frozen as RBIN fixtures under tests/golden.
 *   - compute_nn_inputs, get_col_dry, the NN post-processing and
 *     compute_Planck_source_nn live in reference modules that need netcdf
 *     (unbuildable here); they are restated below line-by-line and pinned by the
 *     known-answer property sum_g pfrac = 1 per band.
 *
 * Every function cites the reference lines it follows.  Array conventions are
 * the reference's Fortran column-major ones: x(a,b,c) is x[a + na*(b + nb*c)].
 * Compile with -ffp-contract=off: multiply-adds are written as fmaf() exactly
 * where the order is meant to be fused.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI_F 3.14159265358979323846f

/* ---------------------------------------------------------------------------------------------
 * NN inputs: rrtmgp/mo_gas_optics_rrtmgp.F90:618-798 (compute_nn_inputs)
 *   nn_inputs(1) = (tlay - min)/(max-min); (2) = (log(play) - ...); (3),(4) = (sqrt(sqrt(h2o/o3)) - ...)
 *   others: concentration scalar/1-D/2-D min-max scaled; missing gas -> ref_vmr = 0
 *   (nn_scenario_index local = 0 at :636 shadows the config module, :757-758).
 * gas[k] for k >= 2 (0-based): pointer to conc, gas_ndims[k] in {0,1,2}, or NULL = missing.
 * h2o (k=2) and o3 (k=3) must be 2-D (nlay,ncol).
 * ------------------------------------------------------------------------------------------- */
void orc_compute_nn_inputs(int ncol, int nlay, int nx, const float *play, const float *tlay,
                           const float *const *gas, const int *gas_ndims,
                           const float *in_min, const float *in_max, float *nn_inputs)
{
  for (int icol = 0; icol < ncol; icol++)
    for (int ilay = 0; ilay < nlay; ilay++) {
      size_t s = (size_t)ilay + (size_t)nlay * icol;
      float *o = nn_inputs + (size_t)nx * s;
      o[0] = (tlay[s] - in_min[0]) / (in_max[0] - in_min[0]);
      o[1] = (logf(play[s]) - in_min[1]) / (in_max[1] - in_min[1]);
      o[2] = (sqrtf(sqrtf(gas[2][s])) - in_min[2]) / (in_max[2] - in_min[2]);
      o[3] = (sqrtf(sqrtf(gas[3][s])) - in_min[3]) / (in_max[3] - in_min[3]);
      for (int k = 4; k < nx; k++) {
        float c;
        if (!gas[k]) c = 0.0f;
        else if (gas_ndims[k] == 0) c = gas[k][0];
        else if (gas_ndims[k] == 1) c = gas[k][ilay];
        else c = gas[k][s];
        o[k] = (c - in_min[k]) / (in_max[k] - in_min[k]);
      }
    }
}

/* rrtmgp/mo_gas_optics_rrtmgp.F90:1662-1707 (get_col_dry), constants mo_rrtmgp_constants.F90 */
void orc_get_col_dry(int ncol, int nlay, const float *vmr_h2o, const float *plev, float *col_dry)
{
  const float m_dry = 0.028964f, m_h2o = 0.018016f, avogad = 6.02214076e23f, grav = 9.80665f;
  for (int icol = 0; icol < ncol; icol++)
    for (int ilev = 0; ilev < nlay; ilev++) {
      const float *pl = plev + (size_t)(nlay + 1) * icol;
      float v = vmr_h2o[ilev + (size_t)nlay * icol];
      float delta_plev = fabsf(pl[ilev] - pl[ilev + 1]);
      float fact = 1.0f / (1.0f + v);
      float m_air = (m_dry + m_h2o * v) * fact;
      col_dry[ilev + (size_t)nlay * icol] =
          10.0f * delta_plev * avogad * fact / (1000.0f * m_air * 100.0f * grav);
    }
}

/* Level temperatures when gas_optics_int is called without tlev: rrtmgp/mo_gas_optics_rrtmgp.F90:317-337.
 * Pressure-weighted interpolation inside the column, linear extrapolation in pressure at both ends; Fortran
 * evaluates a*b/c as (a*b)/c and a*b*c as (a*b)*c, left to right.  play/tlay (nlay,ncol), plev/tlev (nlay+1,ncol). */
void orc_interpolate_tlev(int ncol, int nlay, const float *play, const float *plev, const float *tlay, float *tlev)
{
  for (int icol = 0; icol < ncol; icol++) {
    const float *pa = play + (size_t)nlay * icol, *ta = tlay + (size_t)nlay * icol;
    const float *pv = plev + (size_t)(nlay + 1) * icol;
    float *tv = tlev + (size_t)(nlay + 1) * icol;
    tv[0] = ta[0] + ((pv[0] - pa[0]) * (ta[1] - ta[0])) / (pa[1] - pa[0]);                           /* :327 */
    for (int l = 1; l < nlay; l++)                                                                     /* :328-332 */
      tv[l] = ((pa[l - 1] * ta[l - 1]) * (pv[l] - pa[l]) + (pa[l] * ta[l]) * (pa[l - 1] - pv[l])) /
              (pv[l] * (pa[l - 1] - pa[l]));
    tv[nlay] = ta[nlay - 1] + ((pv[nlay] - pa[nlay - 1]) * (ta[nlay - 1] - ta[nlay - 2])) /           /* :333-334 */
                                  (pa[nlay - 1] - pa[nlay - 2]);
  }
}

/* neural/mod_activation.F90:107-184 (bias_and_activation variants) */
static float activate(int act, float x)
{
  switch (act) {
  case 1: return x / (fabsf(x) + 1.0f);                          /* softsign  :111-118 */
  case 2: return fmaxf(0.0f, x);                                 /* relu      :52-60   */
  case 3: return 1.0f / (1.0f + expf(-x));                       /* sigmoid   :79-86   */
  case 4: return fmaxf(0.0f, fminf(1.0f, 0.2f * x + 0.5f));      /* hard_sigmoid       */
  case 5: return tanhf(x);
  case 6: return expf(-x * x);
  default: return x;                                             /* linear    :163-184 */
  }
}

/* ---------------------------------------------------------------------------------------------
 * Generic MLP forward, neural/mod_network.F90:273-354 (output_sgemm_flat) and
 * neural/mod_network_rrtmgp.F90:125-236: a_{n} = act_n(W_n^T a_{n-1} + b_n).
 * W[n] is stored (n_in, n_out) C-order (= the netCDF kernel, = w_transposed Fortran).
 * The sum is an fmaf chain over ascending k (the GPU MFMA kernel reproduces this order).
 * x(nx, nbatch), out(ny, nbatch); nbatch samples.
 * ------------------------------------------------------------------------------------------- */
void orc_mlp_forward(int nlayers, const int *dims, const float *const *W, const float *const *b,
                     const int *act, long nbatch, const float *x, float *out)
{
  int maxd = 0;
  for (int n = 0; n <= nlayers; n++) if (dims[n] > maxd) maxd = dims[n];
#pragma omp parallel
  {
    float *a0 = (float *)malloc(sizeof(float) * maxd), *a1 = (float *)malloc(sizeof(float) * maxd);
#pragma omp for schedule(static)
    for (long j = 0; j < nbatch; j++) {
      const float *in = x + (size_t)dims[0] * j;
      for (int n = 0; n < nlayers; n++) {
        int nin = dims[n], nout = dims[n + 1];
        float *dst = (n == nlayers - 1) ? out + (size_t)nout * j : ((n & 1) ? a1 : a0);
        const float *w = W[n];
        for (int i = 0; i < nout; i++) {
          float acc = 0.0f;
          for (int k = 0; k < nin; k++) acc = fmaf(w[(size_t)k * nout + i], in[k], acc);
          dst[i] = activate(act[n], acc + b[n][i]);
        }
        in = dst;
      }
    }
    free(a0); free(a1);
  }
}

/* (sigma*y + mu)^8 * coldry; neural/mod_network_rrtmgp.F90:209-219; y already includes bias
 * (the caller's MLP applied the linear last-layer activation).  Optional SW combine
 * :224-229 when tau_abs != NULL: tau_tot = tau_abs + tau_ray, ssa = tau_ray/tau_tot. */
void orc_nn_tau_post(int ngpt, long nbatch, float *y, const float *mean, const float *std,
                     const float *coldry, float *tau_abs_to_tot)
{
  for (long j = 0; j < nbatch; j++)
    for (int i = 0; i < ngpt; i++) {
      size_t idx = (size_t)i + (size_t)ngpt * j;
      float t = std[i] * y[idx] + mean[i];
      float t2 = t * t, t4 = t2 * t2, t8 = t4 * t4;
      float v = t8 * coldry[j];
      if (tau_abs_to_tot) {
        tau_abs_to_tot[idx] = tau_abs_to_tot[idx] + v;
        v = v / tau_abs_to_tot[idx];
      }
      y[idx] = v;
    }
}

/* pfrac = y^2 ; neural/mod_network_rrtmgp.F90:309-312 */
void orc_square(long n, float *y)
{
  for (long i = 0; i < n; i++) y[i] = y[i] * y[i];
}

/* The single-model ("both") branch of predict_nn_lw_blas_sp: rrtmgp/kernels/mo_gas_optics_kernels.F90:744-772 on
 * the output of output_sgemm_lw (neural/mod_network_rrtmgp.F90:319-409: the MLP with the linear last layer, no
 * scaling).  y (2*ngpt, nbatch): rows 1..ngpt are the scaled absorption output, rows ngpt+1..2*ngpt the square root
 * of the Planck fraction.  tau = (ystd*y + ymeans)**8 then tau*col_dry (:760-764; ystd/ymeans are the first ngpt
 * output coefficients, :752-753); pfrac = y(igpt+ngpt)*y(igpt+ngpt) (:766). */
void orc_nn_both_post(int ngpt, long nbatch, const float *y, const float *mean, const float *std,
                      const float *coldry, float *tau, float *pfrac)
{
  for (long j = 0; j < nbatch; j++)
    for (int i = 0; i < ngpt; i++) {
      const float *yj = y + (size_t)2 * ngpt * j;
      float t = std[i] * yj[i] + mean[i];
      float t2 = t * t, t4 = t2 * t2, t8 = t4 * t4;
      tau[(size_t)ngpt * j + i] = t8 * coldry[j];
      pfrac[(size_t)ngpt * j + i] = yj[i + ngpt] * yj[i + ngpt];
    }
}

/* rrtmgp/kernels/mo_gas_optics_kernels.F90:1024-1043 (interpolate1D) */
static void interpolate1D(float val, float offset, float delta, int ntemp, int nbnd,
                          const float *table, float *res)
{
  float val0 = (val - offset) / delta;
  int iv = (int)val0; /* Fortran int(): truncation toward zero */
  float frac = val0 - (float)iv;
  int index = iv + 1;
  if (index < 1) index = 1;
  if (index > ntemp - 1) index = ntemp - 1;
  for (int b = 0; b < nbnd; b++) {
    const float *t = table + (size_t)ntemp * b; /* totplnk(nPlanckTemp, nbnd) */
    res[b] = t[index - 1] + frac * (t[index] - t[index - 1]);
  }
}

/* rrtmgp/kernels/mo_gas_optics_kernels.F90:615-683 (compute_Planck_source_nn)
 * sfc_lay is 1-based (mo_gas_optics_rrtmgp.F90:402: merge(1,nlay,play(1,1) > play(nlay,1))).
 * band_lims_gpt(2,nbnd) 1-based.  pfrac is overwritten with lay_source. */
void orc_planck_source_nn(int ncol, int nlay, int nbnd, int ngpt, int ntemp,
                          const float *tlay, const float *tlev, const float *tsfc, int sfc_lay,
                          const int *band_lims_gpt, float temp_ref_min, float totplnk_delta,
                          const float *totplnk, float *sfc_source, float *sfc_source_Jac,
                          float *pfrac, float *lev_source)
{
  float *pf_sfc = (float *)malloc(sizeof(float) * nbnd * 4);
  float *pf_sfcJ = pf_sfc + nbnd, *pf_lev = pf_sfc + 2 * nbnd, *pf_lay = pf_sfc + 3 * nbnd;
  for (int icol = 0; icol < ncol; icol++) {
    const float *tl = tlev + (size_t)(nlay + 1) * icol;
    interpolate1D(tsfc[icol], temp_ref_min, totplnk_delta, ntemp, nbnd, totplnk, pf_sfc);
    interpolate1D(tsfc[icol] + 1.0f, temp_ref_min, totplnk_delta, ntemp, nbnd, totplnk, pf_sfcJ);
    interpolate1D(tl[nlay], temp_ref_min, totplnk_delta, ntemp, nbnd, totplnk, pf_lev);
    float *pf = pfrac + (size_t)ngpt * nlay * icol;
    float *lv = lev_source + (size_t)ngpt * (nlay + 1) * icol;
    for (int b = 0; b < nbnd; b++)
      for (int g = band_lims_gpt[2 * b] - 1; g < band_lims_gpt[2 * b + 1]; g++) {
        lv[g + (size_t)ngpt * nlay] = pf[g + (size_t)ngpt * (nlay - 1)] * pf_lev[b];
        float ps = pf[g + (size_t)ngpt * (sfc_lay - 1)];
        sfc_source[g + (size_t)ngpt * icol] = ps * pf_sfc[b];
        sfc_source_Jac[g + (size_t)ngpt * icol] = ps * (pf_sfcJ[b] - pf_sfc[b]);
      }
    for (int ilay = 0; ilay < nlay; ilay++) {
      interpolate1D(tl[ilay], temp_ref_min, totplnk_delta, ntemp, nbnd, totplnk, pf_lev);
      interpolate1D(tlay[ilay + (size_t)nlay * icol], temp_ref_min, totplnk_delta, ntemp, nbnd, totplnk, pf_lay);
      for (int b = 0; b < nbnd; b++)
        for (int g = band_lims_gpt[2 * b] - 1; g < band_lims_gpt[2 * b + 1]; g++) {
          size_t i = g + (size_t)ngpt * ilay;
          lv[i] = pf[i] * pf_lev[b];
          pf[i] = pf[i] * pf_lay[b];
        }
    }
  }
  free(pf_sfc);
}

/* ---------------------------------------------------------------------------------------------
 * LW no-scattering solver, one angle: rte/kernels/mo_rte_solver_kernels.F90:119-330
 * with lw_source_noscat :742-776 (top-at-1 indexing hard-coded: Appendix B-1 quirk, reproduced),
 * lw_transport_noscat_dn :982-1009, lw_transport_noscat_up :950-980.
 * If gpt_up/gpt_dn are non-NULL the g-point radiances*fac are ACCUMULATED into them (nmus>1 path,
 * :383-412); otherwise broadband fluxes are written with the 4-way partial sums (:296-318).
 * ------------------------------------------------------------------------------------------- */
static void lw_noscat_col(int ngpt, int nlay, int top_at_1, float D, const float *Dv, float weight,
                          const float *inc, const float *tau, const float *lay, const float *lev,
                          const float *emis, const float *sfc, float *radn_up, float *radn_dn,
                          float *tau_loc, float *trans, float *src_up, float *src_dn,
                          const float *ssa, const float *gg, float *An, float *Cn)
{
  const float tau_thresh = sqrtf(FLT_EPSILON);
  int top = top_at_1 ? 0 : nlay, sfcl = top_at_1 ? nlay : 0;
  for (int g = 0; g < ngpt; g++)
    radn_dn[g + (size_t)ngpt * top] = inc[g] / (2.0f * PI_F * weight);
  if (ssa) { /* do_rescaling (:209-233): scattering folded into an effective optical depth (Tang et al.) */
    for (int l = 0; l < nlay; l++)
      for (int g = 0; g < ngpt; g++) {
        size_t i = g + (size_t)ngpt * l;
        float ssal = ssa[i];
        float wb = ssal * (1.0f - gg[i]) * 0.5f;
        float scaleTau = (1.0f - ssal + wb);
        Cn[i] = 0.4f * wb / scaleTau;
        tau_loc[i] = tau[i] * (Dv ? Dv[g] : D) * scaleTau;
        trans[i] = expf(-tau_loc[i]);
        An[i] = (1.0f - trans[i] * trans[i]);
      }
  } else
  for (int l = 0; l < nlay; l++)
    for (int g = 0; g < ngpt; g++) {
      size_t i = g + (size_t)ngpt * l;
      tau_loc[i] = tau[i] * (Dv ? Dv[g] : D);  /* D(igpt, icol): the Gauss secant, or lw_Ds (rte/mo_rte_lw.F90:329-341) */
      trans[i] = expf(-tau_loc[i]);
    }
  for (int l = 0; l < nlay; l++)
    for (int g = 0; g < ngpt; g++) {
      size_t i = g + (size_t)ngpt * l;
      float t = tau_loc[i], T = trans[i], fact;
      if (t > tau_thresh) fact = (1.0f - T) / t - T;
      else fact = t * (0.5f - 1.0f / 3.0f * t);
      float lvdn = lev[g + (size_t)ngpt * (l + 1)], lvup = lev[i], ly = lay[i];
      src_dn[i] = (1.0f - T) * lvdn + 2.0f * fact * (ly - lvdn);
      src_up[i] = (1.0f - T) * lvup + 2.0f * fact * (ly - lvup);
    }
  if (top_at_1) {
    for (int l = 1; l <= nlay; l++)
      for (int g = 0; g < ngpt; g++)
        radn_dn[g + (size_t)ngpt * l] = trans[g + (size_t)ngpt * (l - 1)] * radn_dn[g + (size_t)ngpt * (l - 1)] +
                                        src_dn[g + (size_t)ngpt * (l - 1)];
  } else {
    for (int l = nlay - 1; l >= 0; l--)
      for (int g = 0; g < ngpt; g++)
        radn_dn[g + (size_t)ngpt * l] = trans[g + (size_t)ngpt * l] * radn_dn[g + (size_t)ngpt * (l + 1)] +
                                        src_dn[g + (size_t)ngpt * l];
  }
  for (int g = 0; g < ngpt; g++) {
    size_t i = g + (size_t)ngpt * sfcl;
    radn_up[i] = radn_dn[i] * (1.0f - emis[g]) + emis[g] * sfc[g];
  }
  if (ssa) { /* lw_transport_1rescl :1729-1795: up with adjustment from radn_dn, then down again from radn_up */
    if (top_at_1) {
      for (int l = nlay - 1; l >= 0; l--)
        for (int g = 0; g < ngpt; g++) {
          size_t i = g + (size_t)ngpt * l;
          float adj = Cn[i] * (An[i] * radn_dn[i] - trans[i] * src_dn[i] - src_up[i]);
          radn_up[i] = trans[i] * radn_up[i + ngpt] + src_up[i] + adj;
        }
      for (int l = 0; l < nlay; l++)
        for (int g = 0; g < ngpt; g++) {
          size_t i = g + (size_t)ngpt * l;
          float adj = Cn[i] * (An[i] * radn_up[i] - trans[i] * src_up[i] - src_dn[i]);
          radn_dn[i + ngpt] = trans[i] * radn_dn[i] + src_dn[i] + adj;
        }
    } else {
      for (int l = 0; l < nlay; l++)
        for (int g = 0; g < ngpt; g++) {
          size_t i = g + (size_t)ngpt * l;
          float adj = Cn[i] * (An[i] * radn_dn[i + ngpt] - trans[i] * src_dn[i] - src_up[i]);
          radn_up[i + ngpt] = trans[i] * radn_up[i] + src_up[i] + adj;
        }
      for (int l = nlay - 1; l >= 0; l--)
        for (int g = 0; g < ngpt; g++) {
          size_t i = g + (size_t)ngpt * l;
          float adj = Cn[i] * (An[i] * radn_up[i] - trans[i] * src_up[i] - src_dn[i]);
          radn_dn[i] = trans[i] * radn_dn[i + ngpt] + src_dn[i] + adj;
        }
    }
    return;
  }
  if (top_at_1) {
    for (int l = nlay - 1; l >= 0; l--)
      for (int g = 0; g < ngpt; g++)
        radn_up[g + (size_t)ngpt * l] = trans[g + (size_t)ngpt * l] * radn_up[g + (size_t)ngpt * (l + 1)] +
                                        src_up[g + (size_t)ngpt * l];
  } else {
    for (int l = 1; l <= nlay; l++)
      for (int g = 0; g < ngpt; g++)
        radn_up[g + (size_t)ngpt * l] = trans[g + (size_t)ngpt * (l - 1)] * radn_up[g + (size_t)ngpt * (l - 1)] +
                                        src_up[g + (size_t)ngpt * (l - 1)];
  }
}

/* lw_solver_noscat_GaussQuad :332-415 (+ lw_solver_noscat per angle); compute_Jac = false
 * (rte/mo_rte_rrtmgp_config.F90:28). Ds/weights have nmus entries.  ssa/g NULL: do_rescaling = false;
 * otherwise the rescaled solution rte_lw uses for 2str optical properties (rte/mo_rte_lw.F90:372-387).
 * lw_Ds (may be NULL): rte_lw's column-dependent secants (rte/mo_rte_lw.F90:329-341): lw_solver_noscat with one angle,
 * D(igpt, icol) = lw_Ds[igpt + ngpt*icol] (the kernel's layout; rte_lw checks the extents as (ncol, ngpt), quirk B-12)
 * and the weight of Ds[0]/weights[0].  gpt_up/gpt_dn (may be NULL, (ngpt, nlay+1, ncol)): save_gpt_flux -- with one
 * angle the g-point RADIANCES (radn_up => flux_up_gpt, no fac: quirk B-5, :183-196, :262-267), with several the
 * fluxes sum over angles of fac*radn (:383-407). */
void orc_lw_solver_noscat_ext(int ngpt, int nlay, int ncol, int top_at_1, int nmus, const float *Ds,
                              const float *weights, const float *lw_Ds, const float *inc_flux, const float *tau,
                              const float *ssa, const float *g, const float *lay_source, const float *lev_source,
                              const float *sfc_emis, const float *sfc_source, float *flux_up, float *flux_dn,
                              float *gpt_up, float *gpt_dn)
{
  if (lw_Ds) nmus = 1;
#pragma omp parallel
  {
    size_t nl = (size_t)ngpt * nlay, nv = (size_t)ngpt * (nlay + 1);
    float *buf = (float *)malloc(sizeof(float) * (6 * nl + 4 * nv));
    float *tau_loc = buf, *trans = buf + nl, *su = buf + 2 * nl, *sd = buf + 3 * nl;
    float *ru = buf + 4 * nl, *rd = ru + nv, *acc_u = rd + nv, *acc_d = acc_u + nv;
    float *An = acc_d + nv, *Cn = An + nl;
#pragma omp for schedule(static)
    for (int icol = 0; icol < ncol; icol++) {
      const float *tc = tau + nl * icol, *lc = lay_source + nl * icol, *vc = lev_source + nv * icol;
      const float *ec = sfc_emis + (size_t)ngpt * icol, *sc = sfc_source + (size_t)ngpt * icol;
      const float *ic = inc_flux + (size_t)ngpt * icol;
      const float *dv = lw_Ds ? lw_Ds + (size_t)ngpt * icol : NULL;
      float *fu = flux_up + (size_t)(nlay + 1) * icol, *fd = flux_dn + (size_t)(nlay + 1) * icol;
      float *au = gpt_up ? gpt_up + nv * icol : acc_u, *ad = gpt_dn ? gpt_dn + nv * icol : acc_d;
      for (int imu = 0; imu < nmus; imu++) {
        lw_noscat_col(ngpt, nlay, top_at_1, Ds[imu], dv, weights[imu], ic, tc, lc, vc, ec, sc, ru, rd,
                      tau_loc, trans, su, sd, ssa ? ssa + nl * icol : NULL, ssa ? g + nl * icol : NULL, An, Cn);
        float fac = 2.0f * PI_F * weights[imu];
        if (nmus == 1) {
          if (gpt_up)
            for (size_t i = 0; i < nv; i++) { au[i] = ru[i]; ad[i] = rd[i]; }
          for (int l = 0; l <= nlay; l++) {
            if (ngpt % 4 == 0) {
              float su4[4] = {0, 0, 0, 0}, sd4[4] = {0, 0, 0, 0};
              for (int g = 0; g < ngpt; g += 4)
                for (int j = 0; j < 4; j++) {
                  su4[j] = su4[j] + fac * ru[g + j + (size_t)ngpt * l];
                  sd4[j] = sd4[j] + fac * rd[g + j + (size_t)ngpt * l];
                }
              fu[l] = su4[0] + su4[1] + su4[2] + su4[3];
              fd[l] = sd4[0] + sd4[1] + sd4[2] + sd4[3];
            } else {
              float a = 0, b = 0;
              for (int g = 0; g < ngpt; g++) { a += ru[g + (size_t)ngpt * l]; b += rd[g + (size_t)ngpt * l]; }
              fu[l] = a; fd[l] = b;   /* quirk Appendix B-5: radiances, no fac, when ngpt%4 != 0 */
            }
          }
        } else {
          for (size_t i = 0; i < nv; i++) {
            if (imu == 0) { au[i] = fac * ru[i]; ad[i] = fac * rd[i]; }
            else { au[i] = au[i] + fac * ru[i]; ad[i] = ad[i] + fac * rd[i]; }
          }
        }
      }
      if (nmus > 1) /* sum_broadband rte/kernels/mo_fluxes_broadband_kernels.F90:31-39 */
        for (int l = 0; l <= nlay; l++) {
          float a = 0, b = 0;
          for (int g = 0; g < ngpt; g++) { a += au[g + (size_t)ngpt * l]; b += ad[g + (size_t)ngpt * l]; }
          fu[l] = a; fd[l] = b;
        }
    }
    free(buf);
  }
}

void orc_lw_solver_1rescl_gaussquad(int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                    const float *Ds, const float *weights, const float *inc_flux,
                                    const float *tau, const float *ssa, const float *g, const float *lay_source,
                                    const float *lev_source, const float *sfc_emis, const float *sfc_source,
                                    float *flux_up, float *flux_dn)
{
  orc_lw_solver_noscat_ext(ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, NULL, inc_flux, tau, ssa, g, lay_source,
                           lev_source, sfc_emis, sfc_source, flux_up, flux_dn, NULL, NULL);
}

void orc_lw_solver_noscat_gaussquad(int ngpt, int nlay, int ncol, int top_at_1, int nmus,
                                    const float *Ds, const float *weights, const float *inc_flux,
                                    const float *tau, const float *lay_source, const float *lev_source,
                                    const float *sfc_emis, const float *sfc_source,
                                    float *flux_up, float *flux_dn)
{
  orc_lw_solver_1rescl_gaussquad(ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, tau, NULL, NULL,
                                 lay_source, lev_source, sfc_emis, sfc_source, flux_up, flux_dn);
}

/* adding (rte/kernels/mo_rte_solver_kernels.F90:1526-1637) for one column; flux_dn holds the incident
 * diffuse flux at the top level on entry.  Shared by the SW and LW two-stream solvers. */
static void adding_col(int ngpt, int nlay, int top_at_1, const float *albedo_sfc, const float *Rdif,
                       const float *Tdif, const float *src_dn, const float *src_up, const float *src_sfc,
                       float *rup, float *rdn, float *albedo, float *src, float *denom)
{
  if (top_at_1) {
    for (int i = 0; i < ngpt; i++) {
      albedo[i + (size_t)ngpt * nlay] = albedo_sfc[i];
      src[i + (size_t)ngpt * nlay] = src_sfc[i];
    }
    for (int l = nlay - 1; l >= 0; l--)
      for (int i = 0; i < ngpt; i++) {
        size_t x = i + (size_t)ngpt * l, xp = x + ngpt;
        denom[x] = 1.0f / (1.0f - Rdif[x] * albedo[xp]);
        albedo[x] = Rdif[x] + Tdif[x] * Tdif[x] * albedo[xp] * denom[x];
        src[x] = src_up[x] + Tdif[x] * denom[x] * (src[xp] + albedo[xp] * src_dn[x]);
      }
    for (int i = 0; i < ngpt; i++) rup[i] = rdn[i] * albedo[i] + src[i];
    for (int l = 1; l <= nlay; l++)
      for (int i = 0; i < ngpt; i++) {
        size_t x = i + (size_t)ngpt * l, xm = x - ngpt;
        rdn[x] = (Tdif[xm] * rdn[xm] + Rdif[xm] * src[x] + src_dn[xm]) * denom[xm];
        rup[x] = rdn[x] * albedo[x] + src[x];
      }
  } else {
    for (int i = 0; i < ngpt; i++) { albedo[i] = albedo_sfc[i]; src[i] = src_sfc[i]; }
    for (int l = 0; l < nlay; l++)
      for (int i = 0; i < ngpt; i++) {
        size_t x = i + (size_t)ngpt * l, xp = x + ngpt;
        denom[x] = 1.0f / (1.0f - Rdif[x] * albedo[x]);
        albedo[xp] = Rdif[x] + Tdif[x] * Tdif[x] * albedo[x] * denom[x];
        src[xp] = src_up[x] + Tdif[x] * denom[x] * (src[x] + albedo[x] * src_dn[x]);
      }
    for (int i = 0; i < ngpt; i++) {
      size_t x = i + (size_t)ngpt * nlay;
      rup[x] = rdn[x] * albedo[x] + src[x];
    }
    for (int l = nlay - 1; l >= 0; l--)
      for (int i = 0; i < ngpt; i++) {
        size_t x = i + (size_t)ngpt * l, xp = x + ngpt;
        rdn[x] = (Tdif[x] * rdn[xp] + Rdif[x] * src[x] + src_dn[x]) * denom[x];
        rup[x] = rdn[x] * albedo[x] + src[x];
      }
  }
}

/* ---------------------------------------------------------------------------------------------
 * LW two-stream: lw_solver_2stream (rte/kernels/mo_rte_solver_kernels.F90:426-486) with lw_two_stream
 * (:1018-1069, Fu et al. 1997 coefficients, LW_diff_sec = 1.66), lw_source_2str (:1112-1162, Toon et al.
 * linear-in-tau sources), adding (:1526-1637) and sum_broadband_nocol (plain sequential sums).
 * ------------------------------------------------------------------------------------------- */
/* gpt_up/gpt_dn (may be NULL, (ngpt, nlay+1, ncol)): flux_up_gpt / flux_dn_gpt, the adding fluxes per g-point
 * (:443, 481), which the reference always forms (in the caller's arrays when ty_fluxes_flexible asks for them) */
void orc_lw_solver_2stream_gpt(int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux, const float *tau,
                               const float *ssa, const float *gg, const float *lev_source, const float *sfc_emis,
                               const float *sfc_source, float *flux_up, float *flux_dn, float *gpt_up, float *gpt_dn)
{
  const float k_min = 1.e-4f, LW_diff_sec = 1.66f;
#pragma omp parallel
  {
    size_t nl = (size_t)ngpt * nlay, nv = (size_t)ngpt * (nlay + 1);
    float *buf = (float *)malloc(sizeof(float) * (7 * nl + 4 * nv + 2 * ngpt));
    float *Rdif = buf, *Tdif = buf + nl, *src_up = buf + 2 * nl, *src_dn = buf + 3 * nl, *denom = buf + 4 * nl;
    float *gamma1 = buf + 5 * nl, *gamma2 = buf + 6 * nl;
    float *rup = buf + 7 * nl, *rdn = rup + nv, *albedo = rdn + nv, *src = albedo + nv;
    float *src_sfc = src + nv, *alb_sfc = src_sfc + ngpt;
#pragma omp for schedule(static)
    for (int icol = 0; icol < ncol; icol++) {
      const float *t = tau + nl * icol, *w0 = ssa + nl * icol, *g = gg + nl * icol, *lev = lev_source + nv * icol;
      const float *em = sfc_emis + (size_t)ngpt * icol, *ss = sfc_source + (size_t)ngpt * icol;
      int top = top_at_1 ? 0 : nlay;
      for (int i = 0; i < ngpt; i++) rdn[i + (size_t)ngpt * top] = inc_flux[i + (size_t)ngpt * icol];
      for (int j = 0; j < nlay; j++)
        for (int i = 0; i < ngpt; i++) {
          size_t x = i + (size_t)ngpt * j;
          gamma1[x] = LW_diff_sec * (1.0f - 0.5f * w0[x] * (1.0f + g[x]));
          gamma2[x] = LW_diff_sec * 0.5f * w0[x] * (1.0f - g[x]);
          float k = sqrtf(fmaxf((gamma1[x] - gamma2[x]) * (gamma1[x] + gamma2[x]), k_min));
          float emk = expf(-t[x] * k);
          float em2k = emk * emk;
          float RT = 1.0f / (k * (1.0f + em2k) + gamma1[x] * (1.0f - em2k));
          Rdif[x] = RT * gamma2[x] * (1.0f - em2k);
          Tdif[x] = RT * 2.0f * k * emk;
        }
      for (int j = 0; j < nlay; j++) {
        const float *ltop = lev + (size_t)ngpt * (top_at_1 ? j : j + 1);
        const float *lbot = lev + (size_t)ngpt * (top_at_1 ? j + 1 : j);
        for (int i = 0; i < ngpt; i++) {
          size_t x = i + (size_t)ngpt * j;
          if (t[x] > 1.0e-8f) {
            float Z = (lbot[i] - ltop[i]) / (t[x] * (gamma1[x] + gamma2[x]));
            float Zup_top = Z + ltop[i], Zup_bottom = Z + lbot[i];
            float Zdn_top = -Z + ltop[i], Zdn_bottom = -Z + lbot[i];
            src_up[x] = PI_F * (Zup_top - Rdif[x] * Zdn_top - Tdif[x] * Zup_bottom);
            src_dn[x] = PI_F * (Zdn_bottom - Rdif[x] * Zup_bottom - Tdif[x] * Zdn_top);
          } else {
            src_up[x] = 0.0f;
            src_dn[x] = 0.0f;
          }
        }
      }
      for (int i = 0; i < ngpt; i++) {
        src_sfc[i] = PI_F * em[i] * ss[i];
        alb_sfc[i] = 1.0f - em[i];
      }
      adding_col(ngpt, nlay, top_at_1, alb_sfc, Rdif, Tdif, src_dn, src_up, src_sfc, rup, rdn, albedo, src, denom);
      float *fu = flux_up + (size_t)(nlay + 1) * icol, *fd = flux_dn + (size_t)(nlay + 1) * icol;
      for (int l = 0; l <= nlay; l++) {
        float a = 0, b = 0;
        for (int i = 0; i < ngpt; i++) { a += rup[i + (size_t)ngpt * l]; b += rdn[i + (size_t)ngpt * l]; }
        fu[l] = a; fd[l] = b;
      }
      if (gpt_up)
        for (size_t i = 0; i < nv; i++) { gpt_up[nv * icol + i] = rup[i]; gpt_dn[nv * icol + i] = rdn[i]; }
    }
    free(buf);
  }
}

void orc_lw_solver_2stream(int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux, const float *tau,
                           const float *ssa, const float *gg, const float *lev_source, const float *sfc_emis,
                           const float *sfc_source, float *flux_up, float *flux_dn)
{
  orc_lw_solver_2stream_gpt(ngpt, nlay, ncol, top_at_1, inc_flux, tau, ssa, gg, lev_source, sfc_emis, sfc_source,
                            flux_up, flux_dn, NULL, NULL);
}

/* ---------------------------------------------------------------------------------------------
 * SW direct beam without scattering (rte_sw on ty_optical_props_1scl, rte/mo_rte_sw.F90:213-222):
 *   apply_BC(..., inc_flux, mu0, flux_dir) -> the generic resolves to apply_BC_factor
 *     (rte/kernels/mo_rte_solver_kernels.F90:1685-1704): flux_dir(:, top) = inc_flux * mu0;
 *   sw_solver_noscat (:496-532): mu0_inv = 1/mu0; flux_dir(:, l+1) = flux_dir(:, l) * exp(-tau(:, l) * mu0_inv)
 *     walking down from the top; flux_dir_bb = sum(flux_dir, 1) per level (sum_broadband_nocol,
 *     rte/kernels/mo_fluxes_broadband_kernels.F90:40-47: one sequential sum over g).
 * The reference's rte_sw passes fluxes%flux_dn_dir and fluxes%gpt_flux_dn_dir in each other's positions (:220-222;
 * quirk B-10 in DESIGN.md): this follows the kernels' own argument meaning.  sw_solver_noscat also sums the whole
 * spectral array from its first column for every column (:530 passes flux_dir, not flux_dir(:,:,icol); quirk
 * B-11): the broadband sum here is each column's own, which equals the reference's for column 1.  inc_flux (ngpt, ncol), tau (ngpt, nlay,
 * ncol), mu0 (ncol) -> flux_dir (nlay+1, ncol).
 * ------------------------------------------------------------------------------------------- */
void orc_sw_solver_noscat(int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux, const float *tau,
                          const float *mu0, float *flux_dir, float *gpt_flux_dir /* (ngpt, nlay+1, ncol) or NULL */)
{
#pragma omp parallel
  {
    float *f = (float *)malloc(sizeof(float) * ngpt * (nlay + 1));
#pragma omp for schedule(static)
    for (int icol = 0; icol < ncol; icol++) {
      const float mu0_inv = 1.0f / mu0[icol];
      const int top = top_at_1 ? 0 : nlay;
      for (int i = 0; i < ngpt; i++) f[i + (size_t)ngpt * top] = inc_flux[i + (size_t)ngpt * icol] * mu0[icol];
      const float *t = tau + (size_t)ngpt * nlay * icol;
      if (top_at_1) {
        for (int l = 1; l <= nlay; l++)
          for (int i = 0; i < ngpt; i++)
            f[i + (size_t)ngpt * l] = f[i + (size_t)ngpt * (l - 1)] * expf(-t[i + (size_t)ngpt * (l - 1)] * mu0_inv);
      } else {
        for (int l = nlay - 1; l >= 0; l--)
          for (int i = 0; i < ngpt; i++)
            f[i + (size_t)ngpt * l] = f[i + (size_t)ngpt * (l + 1)] * expf(-t[i + (size_t)ngpt * l] * mu0_inv);
      }
      float *o = flux_dir + (size_t)(nlay + 1) * icol;
      for (int l = 0; l <= nlay; l++) {
        float s = 0.0f;
        for (int i = 0; i < ngpt; i++) s += f[i + (size_t)ngpt * l];
        o[l] = s;
      }
      if (gpt_flux_dir) memcpy(gpt_flux_dir + (size_t)ngpt * (nlay + 1) * icol, f, sizeof(float) * ngpt * (nlay + 1));
    }
    free(f);
  }
}

/* ---------------------------------------------------------------------------------------------
 * SW two-stream: rte/kernels/mo_rte_solver_kernels.F90:541-692 (sw_solver_2stream),
 * sw_two_stream_source :1366-1480, adding :1526-1637.  k_min = 1e-4 (sp, :76-82).
 * ------------------------------------------------------------------------------------------- */
/* gpt_up/gpt_dn/gpt_dir (may be NULL, (ngpt, nlay+1, ncol)): save_gpt_flux (:572-588, :660-684) -- the g-point
 * up, TOTAL down (diffuse + direct, rounded once: "adding computes only diffuse flux; flux_dn is total") and direct
 * fluxes, and the broadband down flux summed as s + (dn + dir) instead of (s + dn) + dir. */
void orc_sw_solver_2stream_gpt(int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                               const float *inc_flux_dif, const float *tau, const float *ssa, const float *gg,
                               const float *mu0, const float *sfc_alb_dir, const float *sfc_alb_dif,
                               float *flux_up, float *flux_dn, float *flux_dir, float *gpt_up, float *gpt_dn,
                               float *gpt_dir)
{
  const float k_min = 1.e-4f, eps = FLT_EPSILON;
#pragma omp parallel
  {
    size_t nl = (size_t)ngpt * nlay, nv = (size_t)ngpt * (nlay + 1);
    float *buf = (float *)malloc(sizeof(float) * (5 * nl + 5 * nv + ngpt));
    float *Rdif = buf, *Tdif = buf + nl, *src_up = buf + 2 * nl, *src_dn = buf + 3 * nl, *denom = buf + 4 * nl;
    float *rup = buf + 5 * nl, *rdn = rup + nv, *rdir = rdn + nv, *albedo = rdir + nv, *src = albedo + nv;
    float *src_sfc = src + nv;
#pragma omp for schedule(static)
    for (int icol = 0; icol < ncol; icol++) {
      const float *t = tau + nl * icol, *w0 = ssa + nl * icol, *g = gg + nl * icol;
      float m0 = mu0[icol], mu0_inv = 1.0f / m0;
      int top = top_at_1 ? 0 : nlay;
      for (int i = 0; i < ngpt; i++) {
        rdir[i + (size_t)ngpt * top] = inc_flux[i + (size_t)ngpt * icol] * m0;
        rdn[i + (size_t)ngpt * top] = inc_flux_dif[i + (size_t)ngpt * icol];
      }
      float *dir_trans = NULL;
      for (int j = 0; j < nlay; j++) {
        int ilev = top_at_1 ? j : nlay - 1 - j;
        float *dir_inc = rdir + (size_t)ngpt * (top_at_1 ? ilev : ilev + 1);
        dir_trans = rdir + (size_t)ngpt * (top_at_1 ? ilev + 1 : ilev);
        for (int i = 0; i < ngpt; i++) {
          size_t x = i + (size_t)ngpt * ilev;
          float Tnoscat = expf(-t[x] * mu0_inv);
          float gamma1 = (8.0f - w0[x] * (5.0f + 3.0f * g[x])) * .25f;
          float gamma2 = 3.0f * (w0[x] * (1.0f - g[x])) * .25f;
          float gamma3 = (2.0f - 3.0f * m0 * g[x]) * .25f;
          float gamma4 = 1.0f - gamma3;
          float alpha1 = gamma1 * gamma4 + gamma2 * gamma3;
          float alpha2 = gamma1 * gamma3 + gamma2 * gamma4;
          float k = sqrtf(fmaxf((gamma1 - gamma2) * (gamma1 + gamma2), k_min));
          float emk = expf(-t[x] * k);
          float em2k = emk * emk;
          float k2e = 2.0f * k * emk;
          float RT = 1.0f / (k * (1.0f + em2k) + gamma1 * (1.0f - em2k));
          Rdif[x] = RT * gamma2 * (1.0f - em2k);
          Tdif[x] = RT * 2.0f * k * emk;
          float k_mu = k * m0, k_mu2 = k_mu * k_mu, k_g3 = k * gamma3, k_g4 = k * gamma4;
          float dd = (fabsf(1.0f - k_mu2) >= eps) ? (1.0f - k_mu2) : eps;
          RT = w0[x] * RT / dd;
          float Rdir = RT * ((1.0f - k_mu) * (alpha2 + k_g3) - (1.0f + k_mu) * (alpha2 - k_g3) * em2k -
                             k2e * (gamma3 - alpha2 * m0) * Tnoscat);
          float Tdir = RT * (k2e * (gamma4 + alpha1 * m0) -
                             Tnoscat * ((1.0f + k_mu) * (alpha1 + k_g4) - (1.0f - k_mu) * (alpha1 - k_g4) * em2k));
          Rdir = fmaxf(0.0f, fminf(Rdir, (1.0f - Tnoscat)));
          Tdir = fmaxf(0.0f, fminf(Tdir, (1.0f - Tnoscat - Rdir)));
          src_up[x] = Rdir * dir_inc[i];
          src_dn[x] = Tdir * dir_inc[i];
          dir_trans[i] = Tnoscat * dir_inc[i];
        }
      }
      const float *adir = sfc_alb_dir + (size_t)ngpt * icol, *adif = sfc_alb_dif + (size_t)ngpt * icol;
      for (int i = 0; i < ngpt; i++) src_sfc[i] = dir_trans[i] * adir[i];
      /* adding */
      if (top_at_1) {
        for (int i = 0; i < ngpt; i++) {
          albedo[i + (size_t)ngpt * nlay] = adif[i];
          src[i + (size_t)ngpt * nlay] = src_sfc[i];
        }
        for (int l = nlay - 1; l >= 0; l--)
          for (int i = 0; i < ngpt; i++) {
            size_t x = i + (size_t)ngpt * l, xp = x + ngpt;
            denom[x] = 1.0f / (1.0f - Rdif[x] * albedo[xp]);
            albedo[x] = Rdif[x] + Tdif[x] * Tdif[x] * albedo[xp] * denom[x];
            src[x] = src_up[x] + Tdif[x] * denom[x] * (src[xp] + albedo[xp] * src_dn[x]);
          }
        for (int i = 0; i < ngpt; i++) rup[i] = rdn[i] * albedo[i] + src[i];
        for (int l = 1; l <= nlay; l++)
          for (int i = 0; i < ngpt; i++) {
            size_t x = i + (size_t)ngpt * l, xm = x - ngpt;
            rdn[x] = (Tdif[xm] * rdn[xm] + Rdif[xm] * src[x] + src_dn[xm]) * denom[xm];
            rup[x] = rdn[x] * albedo[x] + src[x];
          }
      } else {
        for (int i = 0; i < ngpt; i++) { albedo[i] = adif[i]; src[i] = src_sfc[i]; }
        for (int l = 0; l < nlay; l++)
          for (int i = 0; i < ngpt; i++) {
            size_t x = i + (size_t)ngpt * l, xp = x + ngpt;
            denom[x] = 1.0f / (1.0f - Rdif[x] * albedo[x]);
            albedo[xp] = Rdif[x] + Tdif[x] * Tdif[x] * albedo[x] * denom[x];
            src[xp] = src_up[x] + Tdif[x] * denom[x] * (src[x] + albedo[x] * src_dn[x]);
          }
        for (int i = 0; i < ngpt; i++) {
          size_t x = i + (size_t)ngpt * nlay;
          rup[x] = rdn[x] * albedo[x] + src[x];
        }
        for (int l = nlay - 1; l >= 0; l--)
          for (int i = 0; i < ngpt; i++) {
            size_t x = i + (size_t)ngpt * l, xp = x + ngpt;
            rdn[x] = (Tdif[x] * rdn[xp] + Rdif[x] * src[x] + src_dn[x]) * denom[x];
            rup[x] = rdn[x] * albedo[x] + src[x];
          }
      }
      float *fu = flux_up + (size_t)(nlay + 1) * icol, *fd = flux_dn + (size_t)(nlay + 1) * icol;
      float *fr = flux_dir + (size_t)(nlay + 1) * icol;
      if (gpt_up) {
        float *gu = gpt_up + nv * icol, *gd = gpt_dn + nv * icol, *gr = gpt_dir + nv * icol;
        for (size_t x = 0; x < nv; x++) { gu[x] = rup[x]; gd[x] = rdn[x] + rdir[x]; gr[x] = rdir[x]; }
      }
      for (int l = 0; l <= nlay; l++) {
        if (ngpt % 4 == 0) {
          float su[4] = {0, 0, 0, 0}, sd[4] = {0, 0, 0, 0}, sr[4] = {0, 0, 0, 0};
          for (int i = 0; i < ngpt; i += 4)
            for (int j = 0; j < 4; j++) {
              size_t x = i + j + (size_t)ngpt * l;
              su[j] = su[j] + rup[x];
              sr[j] = sr[j] + rdir[x];
              if (gpt_up) sd[j] = sd[j] + (rdn[x] + rdir[x]);
              else sd[j] = sd[j] + rdn[x] + rdir[x];
            }
          fu[l] = su[0] + su[1] + su[2] + su[3];
          fd[l] = sd[0] + sd[1] + sd[2] + sd[3];
          fr[l] = sr[0] + sr[1] + sr[2] + sr[3];
        } else {
          float a = 0, b = 0, c = 0;
          for (int i = 0; i < ngpt; i++) {
            size_t x = i + (size_t)ngpt * l;
            c += rdir[x]; a += rup[x]; b += rdn[x] + rdir[x];
          }
          fu[l] = a; fd[l] = b; fr[l] = c;
        }
      }
    }
    free(buf);
  }
}

void orc_sw_solver_2stream(int ngpt, int nlay, int ncol, int top_at_1, const float *inc_flux,
                           const float *inc_flux_dif, const float *tau, const float *ssa, const float *gg,
                           const float *mu0, const float *sfc_alb_dir, const float *sfc_alb_dif,
                           float *flux_up, float *flux_dn, float *flux_dir)
{
  orc_sw_solver_2stream_gpt(ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, tau, ssa, gg, mu0, sfc_alb_dir,
                            sfc_alb_dif, flux_up, flux_dn, flux_dir, NULL, NULL, NULL);
}

/* rte/mo_rte_lw.F90:429-447 (expand): band values -> g-points. band_lims 1-based (2,nbnd). */
void orc_expand(int nband, int ngpt, int ncol, const int *band_lims, const float *arr_in, float *arr_out)
{
  for (int icol = 0; icol < ncol; icol++)
    for (int b = 0; b < nband; b++)
      for (int g = band_lims[2 * b] - 1; g < band_lims[2 * b + 1]; g++)
        arr_out[g + (size_t)ngpt * icol] = arr_in[b + (size_t)nband * icol];
}

/* ---------------------------------------------------------------------------------------------
 * Cloud optics (extensions/cloud_optics/mo_cloud_optics.F90).  Tables are the file's Fortran arrays
 * already sliced to the chosen ice roughness: LUT tab(nsize, nband); Pade c(nband, nsizereg, 0:m+n);
 * size-regime bounds sr[nsizereg+1].  Outputs by band (nband, nlay, ncol).
 * ------------------------------------------------------------------------------------------- */
/* :603-645 (compute_all_from_table) for one (band, layer, column) value */
static void from_table(float lwp, float re, int nsteps, float step, float offset, const float *tt,
                       const float *st, const float *at, int nband, int b, float *t, float *ts, float *tsg)
{
  int index = (int)floorf((re - offset) / step) + 1;
  if (index > nsteps - 1) index = nsteps - 1;
  float fint = (re - offset) / step - (float)(index - 1);
  const float *T = tt + (size_t)nsteps * b, *S = st + (size_t)nsteps * b, *A = at + (size_t)nsteps * b;
  int i = index - 1;
  *t = lwp * (T[i] + fint * (T[i + 1] - T[i]));
  *ts = *t * (S[i] + fint * (S[i + 1] - S[i]));
  *tsg = *ts * (A[i] + fint * (A[i + 1] - A[i]));
}

/* :750-775 (pade_eval_1); c(nbnd, nrads, 0:m+n), irad 1-based */
static float pade_eval(int b, int nbnd, int nrads, int m, int n, int irad, float re, const float *c)
{
#define C_(i) c[b + (size_t)nbnd * ((irad - 1) + (size_t)nrads * (i))]
  float denom = C_(n + m);
  for (int i = n - 1 + m; i >= 1 + m; i--) denom = C_(i) + re * denom;
  denom = 1.0f + re * denom;
  float numer = C_(m);
  for (int i = m - 1; i >= 1; i--) numer = C_(i) + re * numer;
  numer = C_(0) + re * numer;
#undef C_
  return numer / denom;
}

/* :650-714 (compute_all_from_pade) for one value; irad = min(floor((re - b(2))/b(3)) + 2, 3) (quirk:
 * divides by the third bound, valid for exactly three size regimes) */
static int pade_irad(float re, const float *bounds)
{
  int irad = (int)floorf((re - bounds[1]) / bounds[2]) + 2;
  return irad < 3 ? irad : 3;
}

void orc_cloud_optics(int lut, int nband, int nsize_liq, int nsize_ice, float radliq_lwr, float radliq_upr,
                      float radice_lwr, float radice_upr, const float *extliq, const float *ssaliq,
                      const float *asyliq, const float *extice, const float *ssaice, const float *asyice,
                      int nsizereg, const float *p_extliq, const float *p_ssaliq, const float *p_asyliq,
                      const float *p_extice, const float *p_ssaice, const float *p_asyice, const float *sr_extliq,
                      const float *sr_ssaliq, const float *sr_asyliq, const float *sr_extice, const float *sr_ssaice,
                      const float *sr_asyice, int ncol, int nlay, const float *clwp, const float *ciwp,
                      const float *reliq, const float *reice, int nstr, float *tau, float *ssa, float *g)
{
  /* :141-142 step sizes; :354-535 combine */
  const float liq_step = (radliq_upr - radliq_lwr) / (float)(nsize_liq - 1);
  const float ice_step = (radice_upr - radice_lwr) / (float)(nsize_ice - 1);
#pragma omp parallel for schedule(static)
  for (int icol = 0; icol < ncol; icol++)
    for (int ilay = 0; ilay < nlay; ilay++) {
      const size_t s = ilay + (size_t)nlay * icol;
      for (int b = 0; b < nband; b++) {
        float lt = 0, lts = 0, ltsg = 0, it = 0, its = 0, itsg = 0;
        if (clwp[s] > 0.0f) {
          if (lut)
            from_table(clwp[s], reliq[s], nsize_liq, liq_step, radliq_lwr, extliq, ssaliq, asyliq, nband, b, &lt,
                       &lts, &ltsg);
          else {
            lt = clwp[s] * pade_eval(b, nband, nsizereg, 2, 3, pade_irad(reliq[s], sr_extliq), reliq[s], p_extliq);
            float w = pade_eval(b, nband, nsizereg, 2, 2, pade_irad(reliq[s], sr_ssaliq), reliq[s], p_ssaliq);
            lts = lt * (1.0f - fmaxf(0.0f, w));
            ltsg = lts * pade_eval(b, nband, nsizereg, 2, 2, pade_irad(reliq[s], sr_asyliq), reliq[s], p_asyliq);
          }
        }
        if (ciwp[s] > 0.0f) {
          if (lut)
            from_table(ciwp[s], reice[s], nsize_ice, ice_step, radice_lwr, extice, ssaice, asyice, nband, b, &it,
                       &its, &itsg);
          else {
            it = ciwp[s] * pade_eval(b, nband, nsizereg, 2, 3, pade_irad(reice[s], sr_extice), reice[s], p_extice);
            float w = pade_eval(b, nband, nsizereg, 2, 2, pade_irad(reice[s], sr_ssaice), reice[s], p_ssaice);
            its = it * (1.0f - fmaxf(0.0f, w));
            itsg = its * pade_eval(b, nband, nsizereg, 2, 2, pade_irad(reice[s], sr_asyice), reice[s], p_asyice);
          }
        }
        const size_t o = b + (size_t)nband * s;
        if (nstr == 1) {
          tau[o] = (lt - lts) + (it - its);
        } else {
          const float t = lt + it, ts = lts + its;
          g[o] = (ltsg + itsg) / fmaxf(FLT_EPSILON, ts);
          ssa[o] = ts / fmaxf(FLT_EPSILON, t);
          tau[o] = t;
        }
      }
    }
}

/* rte/kernels/mo_optical_props_kernels.F90:358-484 (inc_*_bybnd): io (ngpt,nlay,ncol) incremented by
 * in (nbnd,nlay,ncol).  nstr_io / nstr_in in {1, 2}; eps = 3*tiny(1.0) (:31). */
void orc_increment_bybnd(int ncol, int nlay, int ngpt, int nbnd, const int *band_lims, int nstr_io, float *tau1,
                         float *ssa1, float *g1, int nstr_in, const float *tau2, const float *ssa2, const float *g2)
{
  const float eps = 3.0f * FLT_MIN;
#pragma omp parallel for schedule(static)
  for (int icol = 0; icol < ncol; icol++)
    for (int ilay = 0; ilay < nlay; ilay++)
      for (int b = 0; b < nbnd; b++) {
        const size_t ib = b + (size_t)nbnd * (ilay + (size_t)nlay * icol);
        for (int igpt = band_lims[2 * b] - 1; igpt < band_lims[2 * b + 1]; igpt++) {
          const size_t i = igpt + (size_t)ngpt * (ilay + (size_t)nlay * icol);
          if (nstr_io == 1) {
            tau1[i] = nstr_in == 1 ? tau1[i] + tau2[ib] : tau1[i] + tau2[ib] * (1.0f - ssa2[ib]);
          } else if (nstr_in == 1) {
            const float tau12 = tau1[i] + tau2[ib];
            ssa1[i] = tau1[i] * ssa1[i] / fmaxf(eps, tau12);
            tau1[i] = tau12;
          } else {
            const float tau12 = tau1[i] + tau2[ib];
            const float tauscat12 = tau1[i] * ssa1[i] + tau2[ib] * ssa2[ib];
            g1[i] = (tau1[i] * ssa1[i] * g1[i] + tau2[ib] * ssa2[ib] * g2[ib]) / fmaxf(eps, tauscat12);
            ssa1[i] = tauscat12 / fmaxf(eps, tau12);
            tau1[i] = tau12;
          }
        }
      }
}

/* :41-92 (delta_scale_2str_f_k with for = fwd; delta_scale_2str_k, f = g*g, when fwd == NULL) over n values */
void orc_delta_scale_2str(long n, float *tau, float *ssa, float *g, const float *fwd)
{
  const float eps = 3.0f * FLT_MIN;
#pragma omp parallel for schedule(static)
  for (long i = 0; i < n; i++) {
    const float f = fwd ? fwd[i] : g[i] * g[i], wf = ssa[i] * f;
    tau[i] = (1.0f - wf) * tau[i];
    ssa[i] = (ssa[i] - wf) / fmaxf(eps, 1.0f - wf);
    g[i] = (g[i] - f) / fmaxf(eps, 1.0f - f);
  }
}

/* Heating rates per layer from level fluxes, fluxes/plev (nlay+1, ncol), hr (nlay, ncol).
 * mode 0, K/s: extensions/mo_heating_rates.F90:48-52 with grav, cp_dry of rrtmgp/mo_rrtmgp_constants.F90:50,53.
 * mode 1, K/day: examples/rrtmgp-nn-training/rrtmgp_lw_eval_nn_rfmip.F90:639-651 (cp = 1004). */
void orc_heating_rate(int ncol, int nlay, int mode, const float *up, const float *dn, const float *plev, float *hr)
{
  const float grav = 9.80665f, cp_dry = 1004.64f;
  volatile float day = 24.0f * 3600.0f;
  volatile float t = day * grav;
  const float scaling = -(t / 1004.0f);
  for (long c = 0; c < ncol; c++)
    for (int l = 0; l < nlay; l++) {
      const long k = c * (long)(nlay + 1) + l;
      const float dp = plev[k + 1] - plev[k];
      if (mode == 0) {
        hr[c * (long)nlay + l] = (up[k + 1] - up[k] - dn[k + 1] + dn[k]) * grav / (cp_dry * dp);
      } else {
        const float net1 = dn[k + 1] - up[k + 1], net0 = dn[k] - up[k];
        hr[c * (long)nlay + l] = scaling * (net1 - net0) / dp;
      }
    }
}

int orc_num_threads(void)
{
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void orc_set_num_threads(int n)
{
#ifdef _OPENMP
  omp_set_num_threads(n);
#else
  (void)n;
#endif
}
