"""oracle.py -- TEST INFRASTRUCTURE ONLY: numpy front-end of the CPU oracles.

  * `Oracle`    : the C restatement (oracle/librrtmgpnn_oracle.so, built from rrtmgpnn_oracle.c)
  * `Reference` : the reference's own Fortran compiled by oracle/Makefile.ref
                  (oracle/_ref/librrtmgp_ref.so; only where /root/reference was available to build it)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  The
product (rte-rrtmgp-nn_amd/) never does.  Arrays use numpy C order with reversed Fortran shapes
(Fortran tau(ngpt,nlay,ncol) <-> numpy (ncol,nlay,ngpt)).
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "rte-rrtmgp-nn_amd"))
from rrtmgpnn import data  # noqa: E402

ORACLE_SO = os.path.join(HERE, "librrtmgpnn_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "librrtmgp_ref.so")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
c_int, c_float, c_long, c_vp = ctypes.c_int, ctypes.c_float, ctypes.c_long, ctypes.c_void_p


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a):
    return a.ctypes.data_as(c_vp) if a is not None else None


class Oracle:
    """C restatement of the hot path (rrtmgpnn_oracle.c)."""

    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError("%s missing: run `make -C oracle`" % path)
        L = self.L = ctypes.CDLL(path)
        L.orc_compute_nn_inputs.argtypes = [c_int, c_int, c_int, _f32p, _f32p, ctypes.POINTER(c_vp),
                                            _i32p, _f32p, _f32p, _f32p]
        L.orc_get_col_dry.argtypes = [c_int, c_int, _f32p, _f32p, _f32p]
        L.orc_mlp_forward.argtypes = [c_int, _i32p, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), _i32p, c_long,
                                      _f32p, _f32p]
        L.orc_nn_tau_post.argtypes = [c_int, c_long, _f32p, _f32p, _f32p, _f32p, c_vp]
        L.orc_square.argtypes = [c_long, _f32p]
        L.orc_nn_both_post.argtypes = [c_int, c_long, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.orc_interpolate_tlev.argtypes = [c_int, c_int, _f32p, _f32p, _f32p, _f32p]
        L.orc_planck_source_nn.argtypes = [c_int, c_int, c_int, c_int, c_int, _f32p, _f32p, _f32p, c_int, _i32p,
                                           c_float, c_float, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.orc_lw_solver_noscat_gaussquad.argtypes = [c_int, c_int, c_int, c_int, c_int, _f32p, _f32p, _f32p,
                                                     _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.orc_lw_solver_1rescl_gaussquad.argtypes = [c_int] * 5 + [_f32p] * 12
        L.orc_lw_solver_noscat_ext.argtypes = [c_int] * 5 + [c_vp] * 15
        L.orc_sw_solver_2stream_gpt.argtypes = [c_int] * 4 + [c_vp] * 14
        L.orc_lw_solver_2stream.argtypes = [c_int] * 4 + [_f32p] * 9
        L.orc_lw_solver_2stream_gpt.argtypes = [c_int] * 4 + [_f32p] * 9 + [c_vp] * 2
        L.orc_sw_solver_2stream.argtypes = [c_int, c_int, c_int, c_int, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p,
                                            _f32p, _f32p, _f32p, _f32p, _f32p]
        L.orc_expand.argtypes = [c_int, c_int, c_int, _i32p, _f32p, _f32p]
        L.orc_sw_solver_noscat.argtypes = [c_int] * 4 + [_f32p] * 4 + [c_vp]
        L.orc_cloud_optics.argtypes = ([c_int] * 4 + [c_float] * 4 + [_f32p] * 6 + [c_int] + [_f32p] * 12 +
                                       [c_int, c_int] + [_f32p] * 4 + [c_int] + [_f32p] * 3)
        L.orc_increment_bybnd.argtypes = [c_int] * 4 + [_i32p, c_int, _f32p, _f32p, _f32p, c_int, _f32p, _f32p, _f32p]
        L.orc_delta_scale_2str.argtypes = [c_long, _f32p, _f32p, _f32p, ctypes.c_void_p]
        L.orc_set_num_threads.argtypes = [c_int]
        L.orc_heating_rate.argtypes = [c_int, c_int, c_int, _f32p, _f32p, _f32p, _f32p]
        L.orc_num_threads.restype = c_int

    def heating_rate(self, up, dn, plev, k_day=False):
        """orc_heating_rate: fluxes / plev (ncol, nlay+1) -> (ncol, nlay); K/s (mo_heating_rates) or K/day (eval)."""
        up, dn, plev = f32(up), f32(dn), f32(plev)
        ncol, nlev = up.shape
        out = np.empty((ncol, nlev - 1), np.float32)
        self.L.orc_heating_rate(ncol, nlev - 1, int(bool(k_day)), up, dn, plev, out)
        return out

    def set_threads(self, n):
        self.L.orc_set_num_threads(int(n))

    # -- building blocks ---------------------------------------------------------------------
    def nn_inputs(self, play, tlay, gases, model):
        """gases: dict name -> (ncol,nlay) array or scalar; model: RBIN dict of the first network."""
        from rrtmgpnn import rbin
        names = rbin.unchars(model["input_names"])
        nx = len(names)
        ncol, nlay = play.shape
        keep, ptrs, nds = [], [], []
        for k, n in enumerate(names):
            if k < 2 or n not in gases:
                ptrs.append(None)
                nds.append(2)
                continue
            v = np.asarray(gases[n], np.float32)
            nd = {0: 0, 1: 1}.get(v.ndim, 2)  # before f32(): ascontiguousarray makes a 0-d array 1-d
            v = f32(v)
            keep.append(v)
            ptrs.append(_ptr(v))
            nds.append(nd)
        out = np.zeros((ncol, nlay, nx), np.float32)
        self.L.orc_compute_nn_inputs(ncol, nlay, nx, f32(play), f32(tlay), (c_vp * nx)(*ptrs),
                                     np.array(nds, np.int32), f32(model["input_min"]), f32(model["input_max"]), out)
        return out

    def interpolate_tlev(self, play, plev, tlay):
        """tlev when gas_optics_int gets none (rrtmgp/mo_gas_optics_rrtmgp.F90:317-337): (ncol, nlay+1)."""
        ncol, nlay = play.shape
        out = np.zeros((ncol, nlay + 1), np.float32)
        self.L.orc_interpolate_tlev(ncol, nlay, f32(play), f32(plev), f32(tlay), out)
        return out

    def both_post(self, model, y, col_dry):
        """Single "both" model (mo_gas_optics_kernels.F90:744-772): y (..., 2*ngpt) -> tau, pfrac (..., ngpt)."""
        y = f32(y)
        ngpt = y.shape[-1] // 2
        nb = y.size // (2 * ngpt)
        tau = np.zeros(y.shape[:-1] + (ngpt,), np.float32)
        pf = np.zeros_like(tau)
        self.L.orc_nn_both_post(ngpt, nb, y, f32(model["output_mean"]), f32(model["output_std"]),
                                f32(col_dry).reshape(-1), tau, pf)
        return tau, pf

    def col_dry(self, h2o, plev):
        ncol, nlay = h2o.shape
        out = np.zeros((ncol, nlay), np.float32)
        self.L.orc_get_col_dry(ncol, nlay, f32(h2o), f32(plev), out)
        return out

    def mlp(self, model, x):
        dims = np.asarray(model["dims"], np.int32)
        nl = dims.size - 1
        ws = [f32(model["w%d" % (n + 1)]) for n in range(nl)]
        bs = [f32(model["b%d" % (n + 1)]) for n in range(nl)]
        x = f32(x)
        nb = x.size // dims[0]
        out = np.zeros((nb, dims[-1]), np.float32)
        self.L.orc_mlp_forward(nl, dims, (c_vp * nl)(*[_ptr(w) for w in ws]), (c_vp * nl)(*[_ptr(b) for b in bs]),
                               np.asarray(model["activation"], np.int32), nb, x, out)
        return out

    def tau_post(self, model, y, col_dry, tau_abs_to_tot=None):
        y = f32(y).copy()
        ngpt = y.shape[-1]
        nb = y.size // ngpt
        self.L.orc_nn_tau_post(ngpt, nb, y, f32(model["output_mean"]), f32(model["output_std"]), f32(col_dry).reshape(-1),
                               _ptr(tau_abs_to_tot) if tau_abs_to_tot is not None else None)
        return y

    def planck_source(self, kd, tlay, tlev, tsfc, pfrac, sfc_lay):
        ncol, nlay, ngpt = pfrac.shape
        lay = f32(pfrac).copy()
        lev = np.zeros((ncol, nlay + 1, ngpt), np.float32)
        sfc = np.zeros((ncol, ngpt), np.float32)
        jac = np.zeros((ncol, ngpt), np.float32)
        self.L.orc_planck_source_nn(ncol, nlay, kd["nband"], ngpt, kd["nPlanckTemp"], f32(tlay), f32(tlev), f32(tsfc),
                                    int(sfc_lay), np.ascontiguousarray(kd["band_lims_gpt"], np.int32),
                                    float(kd["temp_ref_min"][0]), float(kd["totplnk_delta"]), f32(kd["totplnk"]),
                                    sfc, jac, lay, lev)
        return lay, lev, sfc, jac

    def lw_solver(self, tau, lay, lev, emis_gpt, sfc_src, top_at_1=True, nmus=1, inc_flux=None, ssa=None, g=None,
                  lw_Ds=None, gpt=False):
        """lw_solver_noscat_GaussQuad; with ssa/g the rescaled solution (do_rescaling, rte/mo_rte_lw.F90:372-387).
        lw_Ds: rte_lw's column-dependent secants, read as D(igpt, icol) (rte/mo_rte_lw.F90:329-341; any array of
        ngpt*ncol values, taken in memory order).  gpt: also return the g-point outputs (ncol, nlay+1, ngpt) -- with one
        angle the radiances (quirk B-5), with several the fluxes."""
        ncol, nlay, ngpt = tau.shape
        if lw_Ds is not None or gpt:
            Ds, W = gauss(1 if lw_Ds is not None else nmus)
            keep = [f32(Ds), f32(W), None if lw_Ds is None else f32(lw_Ds),
                    f32(inc_flux) if inc_flux is not None else np.zeros((ncol, ngpt), np.float32), f32(tau),
                    None if ssa is None else f32(ssa), None if g is None else f32(g), f32(lay), f32(lev),
                    f32(emis_gpt), f32(sfc_src)]
            out = [np.zeros((ncol, nlay + 1), np.float32) for _ in range(2)]
            gp = [np.zeros((ncol, nlay + 1, ngpt), np.float32) for _ in range(2)] if gpt else [None, None]
            self.L.orc_lw_solver_noscat_ext(ngpt, nlay, ncol, int(top_at_1), 1 if lw_Ds is not None else nmus,
                                            *[_ptr(a) for a in keep + out + gp])
            return (out[0], out[1], gp[0], gp[1]) if gpt else (out[0], out[1])
        Ds, W = gauss(nmus)
        up = np.zeros((ncol, nlay + 1), np.float32)
        dn = np.zeros((ncol, nlay + 1), np.float32)
        inc = f32(inc_flux) if inc_flux is not None else np.zeros((ncol, ngpt), np.float32)
        if ssa is None:
            self.L.orc_lw_solver_noscat_gaussquad(ngpt, nlay, ncol, int(top_at_1), nmus, f32(Ds), f32(W), inc,
                                                  f32(tau), f32(lay), f32(lev), f32(emis_gpt), f32(sfc_src), up, dn)
        else:
            self.L.orc_lw_solver_1rescl_gaussquad(ngpt, nlay, ncol, int(top_at_1), nmus, f32(Ds), f32(W), inc,
                                                  f32(tau), f32(ssa), f32(g), f32(lay), f32(lev), f32(emis_gpt),
                                                  f32(sfc_src), up, dn)
        return up, dn

    def lw_solver_2stream(self, tau, ssa, g, lev, emis_gpt, sfc_src, top_at_1=True, inc_flux=None, gpt=False):
        """lw_solver_2stream (rte/kernels/mo_rte_solver_kernels.F90:426-486); gpt: also the g-point fluxes
        flux_up_gpt / flux_dn_gpt (ncol, nlay+1, ngpt)."""
        ncol, nlay, ngpt = tau.shape
        up = np.zeros((ncol, nlay + 1), np.float32)
        dn = np.zeros((ncol, nlay + 1), np.float32)
        inc = f32(inc_flux) if inc_flux is not None else np.zeros((ncol, ngpt), np.float32)
        gp = [np.zeros((ncol, nlay + 1, ngpt), np.float32) for _ in range(2)] if gpt else [None, None]
        self.L.orc_lw_solver_2stream_gpt(ngpt, nlay, ncol, int(top_at_1), inc, f32(tau), f32(ssa), f32(g), f32(lev),
                                         f32(emis_gpt), f32(sfc_src), up, dn, _ptr(gp[0]), _ptr(gp[1]))
        return (up, dn, gp[0], gp[1]) if gpt else (up, dn)

    def sw_solver(self, tau, ssa, g, mu0, inc_flux, alb_dir_gpt, alb_dif_gpt, top_at_1=True, inc_flux_dif=None,
                  gpt=False):
        """sw_solver_2stream; gpt: also the g-point up / total down / direct fluxes (ncol, nlay+1, ngpt), with the
        broadband down flux summed as the reference does in that mode."""
        ncol, nlay, ngpt = tau.shape
        if gpt:
            keep = [f32(inc_flux), f32(inc_flux_dif) if inc_flux_dif is not None else np.zeros((ncol, ngpt), np.float32),
                    f32(tau), f32(ssa), f32(g), f32(mu0), f32(alb_dir_gpt), f32(alb_dif_gpt)]
            out = [np.zeros((ncol, nlay + 1), np.float32) for _ in range(3)]
            gp = [np.zeros((ncol, nlay + 1, ngpt), np.float32) for _ in range(3)]
            self.L.orc_sw_solver_2stream_gpt(ngpt, nlay, ncol, int(top_at_1), *[_ptr(a) for a in keep + out + gp])
            return tuple(out) + tuple(gp)
        up = np.zeros((ncol, nlay + 1), np.float32)
        dn = np.zeros((ncol, nlay + 1), np.float32)
        dr = np.zeros((ncol, nlay + 1), np.float32)
        dif = f32(inc_flux_dif) if inc_flux_dif is not None else np.zeros((ncol, ngpt), np.float32)
        self.L.orc_sw_solver_2stream(ngpt, nlay, ncol, int(top_at_1), f32(inc_flux), dif, f32(tau), f32(ssa), f32(g),
                                     f32(mu0), f32(alb_dir_gpt), f32(alb_dif_gpt), up, dn, dr)
        return up, dn, dr

    def sw_solver_noscat(self, tau, mu0, inc_flux, top_at_1=True, gpt=False):
        """rte_sw on 1scl properties: apply_BC_factor + sw_solver_noscat (rte/mo_rte_sw.F90:213-222) -> flux_dir
        (and the spectral direct flux (ncol, nlay+1, ngpt) when gpt)."""
        ncol, nlay, ngpt = tau.shape
        dr = np.zeros((ncol, nlay + 1), np.float32)
        g = np.zeros((ncol, nlay + 1, ngpt), np.float32) if gpt else None
        self.L.orc_sw_solver_noscat(ngpt, nlay, ncol, int(top_at_1), f32(inc_flux), f32(tau), f32(mu0), dr, _ptr(g))
        return (dr, g) if gpt else dr

    def cloud_optics(self, co, clwp, ciwp, reliq, reice, nstr=2, lut=True, icergh=1):
        """ty_cloud_optics%cloud_optics (extensions/cloud_optics/mo_cloud_optics.F90:354-535); by band."""
        t = cloud_tables(co, icergh)
        ncol, nlay = clwp.shape
        nb = t["nband"]
        tau, ssa, g = (np.zeros((ncol, nlay, nb), np.float32) for _ in range(3))
        self.L.orc_cloud_optics(int(lut), nb, t["nsize_liq"], t["nsize_ice"], *t["rad"], *t["lut"], t["nsizereg"],
                                *t["pade"], *t["sr"], ncol, nlay, f32(clwp), f32(ciwp), f32(reliq), f32(reice),
                                nstr, tau, ssa, g)
        return (tau,) if nstr == 1 else (tau, ssa, g)

    def increment_bybnd(self, band_lims_gpt, io, inc):
        """ty_optical_props_arry%increment by band (rte/mo_optical_props.F90:882-1023); io/inc = (tau,) or
        (tau, ssa, g) tuples, io g-point resolved, inc by band.  Returns new io arrays."""
        io = [f32(a).copy() for a in io]
        ncol, nlay, ngpt = io[0].shape
        nb = inc[0].shape[-1]
        z = np.zeros(1, np.float32)
        self.L.orc_increment_bybnd(ncol, nlay, ngpt, nb, np.ascontiguousarray(band_lims_gpt, np.int32), len(io) if len(io) == 1 else 2,
                                   io[0], io[1] if len(io) > 1 else z, io[2] if len(io) > 1 else z,
                                   1 if len(inc) == 1 else 2, f32(inc[0]), f32(inc[1]) if len(inc) > 1 else z,
                                   f32(inc[2]) if len(inc) > 1 else z)
        return tuple(io)

    def delta_scale(self, tau, ssa, g, fwd=None):
        """delta_scale_2str (rte/kernels/mo_optical_props_kernels.F90:41-92): f = fwd, or g**2 when None."""
        tau, ssa, g = f32(tau).copy(), f32(ssa).copy(), f32(g).copy()
        fw = None if fwd is None else f32(fwd)
        self.L.orc_delta_scale_2str(tau.size, tau, ssa, g, None if fw is None else fw.ctypes.data)
        return tau, ssa, g

    # -- class-level pipelines (gas_optics + rte) -------------------------------------------
    def lw_gas_optics(self, prob, models, kd, col_dry=None, tlev=True):
        """gas_optics_int NN branch (rrtmgp/mo_gas_optics_rrtmgp.F90:239-428). models: [abs, pfrac], or [both]
        (the single-model branch, mo_gas_optics_kernels.F90:744-772).  col_dry: the optional argument (quirk B-3
        fixed: honoured); tlev=False: interpolated from the layers (:317-337) instead of prob["tlev"]."""
        x = self.nn_inputs(prob["play"], prob["tlay"], prob["gases"], models[0])
        cd = self.col_dry(prob["gases"]["h2o"], prob["plev"]) if col_dry is None else f32(col_dry)
        ncol, nlay = prob["play"].shape
        xf = x.reshape(-1, x.shape[-1])
        if len(models) == 1:
            tau, pf = self.both_post(models[0], self.mlp(models[0], xf), cd)
            tau, pf = tau.reshape(ncol, nlay, -1), pf.reshape(ncol, nlay, -1)
        else:
            tau = self.tau_post(models[0], self.mlp(models[0], xf), cd).reshape(ncol, nlay, -1)
            pf = self.mlp(models[1], xf)
            pf = (pf * pf).astype(np.float32).reshape(ncol, nlay, -1)
        sfc_lay = 1 if prob["play"][0, 0] > prob["play"][0, nlay - 1] else nlay
        tl = prob["tlev"] if tlev is True else self.interpolate_tlev(prob["play"], prob["plev"], prob["tlay"])
        lay, lev, sfc, jac = self.planck_source(kd, prob["tlay"], tl, prob["tsfc"], pf, sfc_lay)
        return {"tau": tau, "lay_source": lay, "lev_source": lev, "sfc_source": sfc, "sfc_source_Jac": jac,
                "pfrac": pf, "nn_inputs": x, "col_dry": cd, "tlev": tl}

    def sw_gas_optics(self, prob, models):
        """gas_optics_ext NN branch (:433-602), 2str: tau, ssa, g (= 0)."""
        x = self.nn_inputs(prob["play"], prob["tlay"], prob["gases"], models[0])
        cd = self.col_dry(prob["gases"]["h2o"], prob["plev"])
        ncol, nlay = prob["play"].shape
        xf = x.reshape(-1, x.shape[-1])
        tau = self.tau_post(models[0], self.mlp(models[0], xf), cd)
        ssa = self.tau_post(models[1], self.mlp(models[1], xf), cd, tau_abs_to_tot=tau)
        return {"tau": tau.reshape(ncol, nlay, -1), "ssa": ssa.reshape(ncol, nlay, -1),
                "g": np.zeros((ncol, nlay, tau.shape[-1]), np.float32), "nn_inputs": x, "col_dry": cd}

    def clear_sky_lw(self, prob, models, kd, nmus=1):
        go = self.lw_gas_optics(prob, models, kd)
        ngpt = go["tau"].shape[-1]
        emis = np.repeat(f32(prob["sfc_emis"])[:, None], ngpt, axis=1)
        up, dn = self.lw_solver(go["tau"], go["lay_source"], go["lev_source"], emis, go["sfc_source"],
                                prob["top_at_1"], nmus)
        return up, dn, go

    def all_sky_lw(self, prob, models, kd, co, clouds, nmus=1, icergh=2, lut=True):
        """examples/all-sky/rrtmgp_allsky.F90:366-404 with NN gas optics: cloud_optics (1scl, by band) ->
        gas_optics -> clouds%increment(atmos) -> rte_lw.  clouds = (lwp, iwp, rel, rei), each (ncol, nlay)."""
        go = self.lw_gas_optics(prob, models, kd)
        cld = self.cloud_optics(co, *clouds, nstr=1, lut=lut, icergh=icergh)
        (tau,) = self.increment_bybnd(kd["band_lims_gpt"], (go["tau"],), cld)
        ngpt = tau.shape[-1]
        emis = np.repeat(f32(prob["sfc_emis"])[:, None], ngpt, axis=1)
        up, dn = self.lw_solver(tau, go["lay_source"], go["lev_source"], emis, go["sfc_source"], prob["top_at_1"], nmus)
        return up, dn, dict(go, tau=tau, clouds=cld)

    def all_sky_sw(self, prob, models, kd_sw, co, clouds, icergh=2, lut=True):
        """rrtmgp_allsky.F90:405-446: cloud_optics (2str) -> gas_optics -> clouds%delta_scale() ->
        clouds%increment(atmos) -> rte_sw."""
        go = self.sw_gas_optics(prob, models)
        cld = self.delta_scale(*self.cloud_optics(co, *clouds, nstr=2, lut=lut, icergh=icergh))
        tau, ssa, g = self.increment_bybnd(kd_sw["band_lims_gpt"], (go["tau"], go["ssa"], go["g"]), cld)
        ngpt = tau.shape[-1]
        toa = data.toa_flux(prob, kd_sw)
        alb = np.repeat(f32(prob["sfc_alb"])[:, None], ngpt, axis=1)
        up, dn, dr = self.sw_solver(tau, ssa, g, prob["mu0"], toa, alb, alb, prob["top_at_1"])
        m = ~prob["usecol"]
        up[m] = 0.0
        dn[m] = 0.0
        return up, dn, dr, dict(go, tau=tau, ssa=ssa, g=g, clouds=cld)

    def clear_sky_sw(self, prob, models, kd_sw):
        go = self.sw_gas_optics(prob, models)
        ngpt = go["tau"].shape[-1]
        toa = data.toa_flux(prob, kd_sw)
        alb = np.repeat(f32(prob["sfc_alb"])[:, None], ngpt, axis=1)
        up, dn, dr = self.sw_solver(go["tau"], go["ssa"], go["g"], prob["mu0"], toa, alb, alb, prob["top_at_1"])
        m = ~prob["usecol"]
        up[m] = 0.0
        dn[m] = 0.0
        return up, dn, dr, go


def cloud_tables(co, icergh=1):
    """Flat argument tuple of a cloud-optics RBIN dict (data.load_cloud_optics) for the C/Fortran entry points:
    LUT and Pade tables in the file's Fortran layout, the ice tables sliced at roughness icergh (1-based)."""
    nband = co["bnd_limits_wavenumber"].shape[0]
    r = icergh - 1
    lut = (f32(co["lut_extliq"]), f32(co["lut_ssaliq"]), f32(co["lut_asyliq"]),
           f32(co["lut_extice"][r]), f32(co["lut_ssaice"][r]), f32(co["lut_asyice"][r]))
    pade = (f32(co["pade_extliq"]), f32(co["pade_ssaliq"]), f32(co["pade_asyliq"]),
            f32(co["pade_extice"][r]), f32(co["pade_ssaice"][r]), f32(co["pade_asyice"][r]))
    sr = tuple(f32(co["pade_sizreg_" + k]) for k in ("extliq", "ssaliq", "asyliq", "extice", "ssaice", "asyice"))
    return {"nband": nband, "nsize_liq": co["lut_extliq"].shape[1], "nsize_ice": co["lut_extice"].shape[2],
            "nrgh": co["lut_extice"].shape[0], "nsizereg": co["pade_extliq"].shape[1],
            "rad": tuple(float(co[k][0]) for k in ("radliq_lwr", "radliq_upr", "radice_lwr", "radice_upr")),
            "lut": lut, "pade": pade, "sr": sr}


def gauss(nmus):
    """Gauss_Ds / gauss_wts of rte/mo_rte_lw.F90:113-125 (first-order quadrature, column nmus)."""
    Ds = {1: [1.66], 2: [1.18350343, 2.81649655], 3: [1.09719858, 1.69338507, 4.70941630],
          4: [1.06056257, 1.38282560, 2.40148179, 7.15513024]}[nmus]
    W = {1: [0.5], 2: [0.3180413817, 0.1819586183], 3: [0.2009319137, 0.2292411064, 0.0698269799],
         4: [0.1355069134, 0.2034645680, 0.1298475476, 0.0311809710]}[nmus]
    return np.array(Ds, np.float32), np.array(W, np.float32)


class Reference:
    """The reference's own Fortran (rte_lw, rte_sw, network_type%output_sgemm_flat + MKL sgemm)."""

    def __init__(self, path=REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError("%s missing: build with `make -f oracle/Makefile.ref` (needs /root/reference)" % path)
        os.environ.setdefault("MKL_THREADING_LAYER", "SEQUENTIAL")
        L = self.L = ctypes.CDLL(path)
        L.ref_rte_lw.argtypes = [c_int, c_int, c_int, c_int, _i32p, _f32p, c_int, c_int, _f32p, _f32p, _f32p, _f32p,
                                 _f32p, _f32p, _f32p, _f32p]
        L.ref_rte_lw.restype = c_int
        L.ref_rte_lw_2str.argtypes = [c_int, c_int, c_int, c_int, _i32p, _f32p, c_int, c_int, c_int] + [_f32p] * 10
        L.ref_rte_lw_2str.restype = c_int
        L.ref_rte_sw.argtypes = [c_int, c_int, c_int, c_int, _i32p, _f32p, c_int, _f32p, _f32p, _f32p, _f32p,
                                 _f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.ref_rte_sw.restype = c_int
        L.ref_mlp.argtypes = [c_int, _i32p, _i32p, _f32p, _f32p, c_int, _f32p, _f32p]
        L.ref_mlp.restype = c_int
        L.ref_last_error.argtypes = [ctypes.c_char_p, c_int]
        L.ref_cloud_optics.argtypes = ([c_int, c_int, _f32p, c_int, c_int, c_int] + [c_float] * 4 + [_f32p] * 6 +
                                       [c_int, c_int, c_int] + [_f32p] * 12 + [c_int, c_int, c_int] + [_f32p] * 4 +
                                       [c_int] + [_f32p] * 3)
        L.ref_cloud_optics.restype = c_int
        L.ref_increment_bybnd.argtypes = [c_int] * 4 + [_i32p, _f32p, c_int, _f32p, _f32p, _f32p, c_int, _f32p, _f32p,
                                                        _f32p]
        L.ref_increment_bybnd.restype = c_int
        L.ref_delta_scale.argtypes = [c_int, c_int, c_int, _f32p, _f32p, _f32p, _f32p, c_int, _f32p]
        L.ref_delta_scale.restype = c_int
        L.ref_sw_noscat.argtypes = [c_int] * 4 + [_f32p] * 5
        L.ref_sw_noscat.restype = c_int
        L.ref_rte_lw_gpt.argtypes = [c_int, c_int, c_int, c_int, _i32p, _f32p, c_int, c_int, c_int] + [_f32p] * 11
        L.ref_rte_lw_gpt.restype = c_int
        L.ref_rte_sw_gpt.argtypes = [c_int, c_int, c_int, c_int, _i32p, _f32p, c_int] + [_f32p] * 13
        L.ref_rte_sw_gpt.restype = c_int
        L.ref_rte_lw_2str_gpt.argtypes = [c_int, c_int, c_int, c_int, _i32p, _f32p, c_int, c_int, c_int] + [_f32p] * 12
        L.ref_rte_lw_2str_gpt.restype = c_int

    def sw_noscat(self, tau, mu0, inc_flux, top_at_1=True):
        """The reference's apply_BC (-> apply_BC_factor) + sw_solver_noscat kernels: broadband and spectral direct
        flux (the broadband one is column 1's for every column, quirk B-11)."""
        ncol, nlay, ngpt = tau.shape
        dr = np.zeros((ncol, nlay + 1), np.float32)
        g = np.zeros((ncol, nlay + 1, ngpt), np.float32)
        self._check(self.L.ref_sw_noscat(ncol, nlay, ngpt, int(top_at_1), f32(inc_flux), f32(tau), f32(mu0), dr, g))
        return dr, g

    def _check(self, rc):
        if rc != 0:
            buf = ctypes.create_string_buffer(256)
            self.L.ref_last_error(buf, 256)
            raise RuntimeError("reference failed: %s" % buf.value.decode())

    def rte_lw_2str(self, kd, tau, ssa, g, lay, lev, sfc_src, sfc_jac, sfc_emis_band, top_at_1=True, nmus=1,
                    use_2stream=False):
        ncol, nlay, ngpt = tau.shape
        up = np.zeros((ncol, nlay + 1), np.float32)
        dn = np.zeros((ncol, nlay + 1), np.float32)
        self._check(self.L.ref_rte_lw_2str(ncol, nlay, kd["nband"], ngpt,
                                           np.ascontiguousarray(kd["band_lims_gpt"], np.int32), f32(kd["band_lims_wvn"]),
                                           int(top_at_1), nmus, int(use_2stream), f32(tau), f32(ssa), f32(g), f32(lay),
                                           f32(lev), f32(sfc_src), f32(sfc_jac), f32(sfc_emis_band), up, dn))
        return up, dn

    def rte_lw_2str_gpt(self, kd, tau, ssa, g, lay, lev, sfc_src, sfc_jac, sfc_emis_band, top_at_1=True, nmus=1,
                        use_2stream=False):
        """rte_lw_2str with ty_fluxes_flexible g-point outputs (ncol, nlay+1, ngpt)."""
        ncol, nlay, ngpt = tau.shape
        out = [np.zeros((ncol, nlay + 1), np.float32) for _ in range(2)]
        gp = [np.zeros((ncol, nlay + 1, ngpt), np.float32) for _ in range(2)]
        self._check(self.L.ref_rte_lw_2str_gpt(ncol, nlay, kd["nband"], ngpt,
                                               np.ascontiguousarray(kd["band_lims_gpt"], np.int32),
                                               f32(kd["band_lims_wvn"]), int(top_at_1), nmus, int(use_2stream),
                                               f32(tau), f32(ssa), f32(g), f32(lay), f32(lev), f32(sfc_src),
                                               f32(sfc_jac), f32(sfc_emis_band), *out, *gp))
        return out[0], out[1], gp[0], gp[1]

    def rte_lw(self, kd, tau, lay, lev, sfc_src, sfc_jac, sfc_emis_band, top_at_1=True, nmus=1):
        ncol, nlay, ngpt = tau.shape
        up = np.zeros((ncol, nlay + 1), np.float32)
        dn = np.zeros((ncol, nlay + 1), np.float32)
        self._check(self.L.ref_rte_lw(ncol, nlay, kd["nband"], ngpt, np.ascontiguousarray(kd["band_lims_gpt"], np.int32),
                                      f32(kd["band_lims_wvn"]), int(top_at_1), nmus, f32(tau), f32(lay), f32(lev),
                                      f32(sfc_src), f32(sfc_jac), f32(sfc_emis_band), up, dn))
        return up, dn

    def rte_lw_gpt(self, kd, tau, lay, lev, sfc_src, sfc_jac, sfc_emis_band, top_at_1=True, nmus=1, lw_Ds=None):
        """rte_lw with ty_fluxes_flexible g-point outputs (ncol, nlay+1, ngpt) and optionally lw_Ds (ngpt*ncol values
        in memory order; rte_lw sees them with the extents it checks, (ncol, ngpt))."""
        ncol, nlay, ngpt = tau.shape
        out = [np.zeros((ncol, nlay + 1), np.float32) for _ in range(2)]
        gp = [np.zeros((ncol, nlay + 1, ngpt), np.float32) for _ in range(2)]
        ds = f32(lw_Ds).ravel() if lw_Ds is not None else np.ones(ngpt * ncol, np.float32)
        self._check(self.L.ref_rte_lw_gpt(ncol, nlay, kd["nband"], ngpt, np.ascontiguousarray(kd["band_lims_gpt"], np.int32),
                                          f32(kd["band_lims_wvn"]), int(top_at_1), nmus, int(lw_Ds is not None), ds,
                                          f32(tau), f32(lay), f32(lev), f32(sfc_src), f32(sfc_jac), f32(sfc_emis_band),
                                          *out, *gp))
        return out[0], out[1], gp[0], gp[1]

    def rte_sw_gpt(self, kd, tau, ssa, g, mu0, inc_flux, alb_dir_gpt, alb_dif_gpt, top_at_1=True):
        """rte_sw with ty_fluxes_flexible g-point up / down (total) / direct outputs (ncol, nlay+1, ngpt)."""
        ncol, nlay, ngpt = tau.shape
        out = [np.zeros((ncol, nlay + 1), np.float32) for _ in range(3)]
        gp = [np.zeros((ncol, nlay + 1, ngpt), np.float32) for _ in range(3)]
        self._check(self.L.ref_rte_sw_gpt(ncol, nlay, kd["nband"], ngpt, np.ascontiguousarray(kd["band_lims_gpt"], np.int32),
                                          f32(kd["band_lims_wvn"]), int(top_at_1), f32(tau), f32(ssa), f32(g), f32(mu0),
                                          f32(inc_flux), f32(alb_dir_gpt), f32(alb_dif_gpt), *out, *gp))
        return tuple(out) + tuple(gp)

    def rte_sw(self, kd, tau, ssa, g, mu0, inc_flux, alb_dir_gpt, alb_dif_gpt, top_at_1=True):
        ncol, nlay, ngpt = tau.shape
        up = np.zeros((ncol, nlay + 1), np.float32)
        dn = np.zeros((ncol, nlay + 1), np.float32)
        dr = np.zeros((ncol, nlay + 1), np.float32)
        self._check(self.L.ref_rte_sw(ncol, nlay, kd["nband"], ngpt, np.ascontiguousarray(kd["band_lims_gpt"], np.int32),
                                      f32(kd["band_lims_wvn"]), int(top_at_1), f32(tau), f32(ssa), f32(g), f32(mu0),
                                      f32(inc_flux), f32(alb_dir_gpt), f32(alb_dif_gpt), up, dn, dr))
        return up, dn, dr

    def mlp(self, model, x):
        dims = np.asarray(model["dims"], np.int32)
        nl = dims.size - 1
        w_all = np.concatenate([f32(model["w%d" % (n + 1)]).ravel() for n in range(nl)])
        b_all = np.concatenate([f32(model["b%d" % (n + 1)]).ravel() for n in range(nl)])
        x = f32(x)
        nb = x.size // dims[0]
        out = np.zeros((nb, dims[-1]), np.float32)
        self._check(self.L.ref_mlp(nl, dims, np.asarray(model["activation"], np.int32), w_all, b_all, nb, x, out))
        return out

    def cloud_optics(self, co, clwp, ciwp, reliq, reice, nstr=2, lut=True, icergh=1):
        """The reference's ty_cloud_optics (load_lut / load_pade, set_ice_roughness, cloud_optics)."""
        t = cloud_tables(co, 1)
        nb = t["nband"]
        ncol, nlay = clwp.shape
        full = lambda k: f32(co[k])  # noqa: E731  (all roughness types; the reference slices itself)
        tau, ssa, g = (np.zeros((ncol, nlay, nb), np.float32) for _ in range(3))
        ncx, ncs = co["pade_extliq"].shape[0], co["pade_ssaliq"].shape[0]
        self._check(self.L.ref_cloud_optics(
            int(lut), nb, f32(co["bnd_limits_wavenumber"]), t["nsize_liq"], t["nsize_ice"], t["nrgh"], *t["rad"],
            full("lut_extliq"), full("lut_ssaliq"), full("lut_asyliq"), full("lut_extice"), full("lut_ssaice"),
            full("lut_asyice"), t["nsizereg"], ncx, ncs, full("pade_extliq"), full("pade_ssaliq"),
            full("pade_asyliq"), full("pade_extice"), full("pade_ssaice"), full("pade_asyice"), *t["sr"], icergh,
            ncol, nlay, f32(clwp), f32(ciwp), f32(reliq), f32(reice), nstr, tau, ssa, g))
        return (tau,) if nstr == 1 else (tau, ssa, g)

    def increment_bybnd(self, kd, io, inc):
        io = [f32(a).copy() for a in io]
        ncol, nlay, ngpt = io[0].shape
        z = np.zeros(io[0].shape, np.float32)
        zi = np.zeros(inc[0].shape, np.float32)
        self._check(self.L.ref_increment_bybnd(ncol, nlay, kd["nband"], ngpt, np.ascontiguousarray(kd["band_lims_gpt"], np.int32),
                                               f32(kd["band_lims_wvn"]), 1 if len(io) == 1 else 2, io[0],
                                               io[1] if len(io) > 1 else z, io[2] if len(io) > 1 else z,
                                               1 if len(inc) == 1 else 2, f32(inc[0]),
                                               f32(inc[1]) if len(inc) > 1 else zi, f32(inc[2]) if len(inc) > 1 else zi))
        return tuple(io)

    def delta_scale(self, kd, tau, ssa, g, fwd=None):
        tau, ssa, g = f32(tau).copy(), f32(ssa).copy(), f32(g).copy()
        ncol, nlay, nb = tau.shape
        fw = np.zeros_like(tau) if fwd is None else f32(fwd)
        self._check(self.L.ref_delta_scale(ncol, nlay, nb, f32(kd["band_lims_wvn"]), tau, ssa, g, int(fwd is not None),
                                           fw))
        return tau, ssa, g
