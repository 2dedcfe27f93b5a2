"""Device-resident clear-sky LW+SW step: the hot path of BASELINE.json's metric.

One `ClearSkyStep` owns every input and output of one column block in HBM and replays
    gas_optics_int (NN)  ->  rte_lw (no-scattering)      [LW, g256]
    gas_optics_ext (NN)  ->  rte_sw (two-stream)         [SW, g224]
with the same kernels as the class-level API (api.py), but with all ctypes arguments prepared once
so the host cost per step is just the launches (or one hipGraph replay).

fused=True (default) keeps intermediates that the flux computation does not need out of HBM: the
Planck sources are formed inside the LW solver from the Planck fraction
(rrtmgpnn_lw_solver_noscat_planck: same products, same bits, compute_Planck_source_nn's arrays never
stored), and the SW asymmetry parameter -- identically zero in the NN path -- is passed as NULL
instead of being written and re-read.  fused=False issues exactly the class layer's call sequence.

What one step computes is exactly the drivers' per-block work
(examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:399-441, rrtmgp_rfmip_sw.F90:374-451):
compute_nn_inputs, get_col_dry, both NN models per stream with post-processing, the Planck sources,
the band->g emissivity expansion, the SW boundary conditions (gas_optics_ext's incident flux
renormalised to each column's TSI, the per-g-point surface albedo and mu0 = cos(sza), formed from the
block's TSI, albedo and zenith angle, rrtmgp_rfmip_sw.F90:403-434: in the fused step inside the SW
solver, rrtmgpnn_sw_solver_2stream_rfmip; unfused rrtmgpnn_sw_boundary_rfmip), both solvers and the
broadband reductions.  The step's inputs are the driver's per-column state; the only
data prepared once are the model's (network weights, the Planck table, solar_source after set_tsi).
The unfused step computes col_dry once and shares it between LW and SW (same h2o and plev).

clouds=(lwp, iwp, rel, rei) makes it the all-sky step of examples/all-sky/rrtmgp_allsky.F90:366-446
(config C4) with NN gas optics: cloud optics by band (LUT by default, ice roughness 2 as in the example,
:219), added to the LW absorption optical depth by band (1scl increment), and for SW delta-scaled and
added as a two-stream increment; the SW solver then sees a non-zero asymmetry parameter.
"""

import numpy as np
import torch

from . import _lib, data, shard
from ._lib import check, float_array, int_array, ptr_array
from .api import GAUSS_DS, GAUSS_WTS, Context


# calls of the SW chain (issued on the second stream when overlapping)
SW_CHAIN = {"sw_boundary", "nn_inputs_sw", "predict_nn_sw", "cloud_optics_sw", "delta_scale_sw", "increment_sw",
            "sw_solver"}


# issue order of the fused step (stable sort; names not listed keep their place at the end)
FUSED_ORDER = ["sw_boundary", "get_col_dry", "expand_emis", "nn_inputs_lw", "cloud_optics_lw", "predict_nn_lw", "lw_solver",
               "nn_inputs_sw", "cloud_optics_sw", "delta_scale_sw", "predict_nn_sw", "sw_solver"]


def issue_order(calls, fused, lw_after=""):
    """The step's issue order of `calls` ((name, fn, args) tuples): fused steps sort by FUSED_ORDER (stable; names
    not listed keep their place at the end); lw_after (an SW-chain call) moves the SW-chain calls up to and including
    it ahead of the rest, so the LW chain can be gated on it.  Each chain keeps its own relative order (a chain is
    issued on one stream, in this order)."""
    calls = list(calls)
    if fused:
        order = {n: i for i, n in enumerate(FUSED_ORDER)}
        calls.sort(key=lambda c: order.get(c[0], len(order)))
    if lw_after:
        names = [n for n, _, _ in calls]
        if lw_after not in names or lw_after not in SW_CHAIN or "get_col_dry" in names:
            raise ValueError("lw_after: %r is not a call of this fused step's SW chain" % lw_after)
        cut = names.index(lw_after)
        head = [c for i, c in enumerate(calls) if c[0] in SW_CHAIN and i <= cut]
        calls = head + [c for c in calls if c not in head]
    return calls


def _t(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=dev)


class ClearSkyStep:
    def __init__(self, prob, device=0, nmus=1, ctx=None, lw_models=("lw_abs", "lw_pfrac"),
                 sw_models=("sw_abs", "sw_ray"), fused=True, clouds=None, icergh=2, cloud_lut=True, overlap=True,
                 sw=True, lw_after=None, sw_after=None, sw_priority=0, lw_net_cus=None, sw_net_cus=0):
        # sw=False: the LW half alone (config C2, rrtmgp_rfmip_lw.F90): gas optics LW + Planck + rte_lw
        # lw_after: the SW-chain call the LW chain starts after on two streams (None: the default gate in _finish;
        # "": the chains start together)
        self.dev = torch.device("cuda", device)
        self.allsky = clouds is not None
        self.fused = fused
        self._own_ctx = ctx is None  # a caller's context keeps its settings (the LW network's CU cap below)
        # Streams: non-blocking HIP streams this step alone holds for its lifetime (_lib.stream_acquire), released by
        # close() after its graph and contexts -- never torch's pooled streams, which torch hands out round-robin to
        # every caller, nor the legacy null stream.  Captures run on these same streams and replays launch on the LW
        # one (the round-5 host segfault).
        self._streams, self._closed, self.graph, self.ctx2 = [], False, None, None
        self.ctx = ctx or Context(device, self._new_stream())
        L = self.L = _lib.lib()
        self.kd_lw, self.kd_sw = data.load_kdist("lw"), data.load_kdist("sw")
        self.ncol, self.nlay = ncol, nlay = prob["ncol"], prob["nlay"]
        self.top_at_1 = int(bool(prob["top_at_1"]))
        dev = self.dev

        def net(name):
            h = _lib.c_vp()
            check(L.rrtmgpnn_network_load(self.ctx.h, data.path(name).encode(), h), "network_load " + name)
            return h

        self.lw_nets = [net(n) for n in lw_models]
        self.sw_nets = [net(n) for n in sw_models]
        self.lw_names = data.rbin.unchars(data.load_model(lw_models[0])["input_names"])
        self.sw_names = data.rbin.unchars(data.load_model(sw_models[0])["input_names"])
        self.nx_lw, self.nx_sw = len(self.lw_names), len(self.sw_names)
        self.ng_lw, self.ng_sw = self.kd_lw["ngpt"], self.kd_sw["ngpt"]
        self.nb_lw = self.kd_lw["nband"]

        # ---- inputs (HBM resident) ----
        self._gas_names = list(prob["gases"])
        ins = self._inputs(prob, clouds)
        self.play, self.plev, self.tlay, self.tlev, self.tsfc = ins[:5]
        self.gases = dict(zip(self._gas_names, ins[5:5 + len(self._gas_names)]))
        self.sfc_emis, self.sza, self.tsi, self.sfc_alb = ins[5 + len(self._gas_names):9 + len(self._gas_names)]
        self.totplnk = _t(self.kd_lw["totplnk"], dev)
        # gas_optics_ext's toa_src per g-point: solar_source after set_tsi(1361) (rrtmgp_rfmip_sw.F90:317)
        self.solar_source = _t(data.set_tsi(self.kd_sw["solar_source"], 1361.0), dev)
        self.sfc_lay = 1 if prob["play"][0, 0] > prob["play"][0, nlay - 1] else nlay

        # ---- intermediates / outputs ----
        f = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        self.col_dry = f(ncol, nlay)
        self.x_lw, self.x_sw = f(ncol, nlay, self.nx_lw), f(ncol, nlay, self.nx_sw)
        self.tau_lw, self.lay_src = f(ncol, nlay, self.ng_lw), f(ncol, nlay, self.ng_lw)
        self.emis_gpt = f(ncol, self.ng_lw)
        self.sw = sw
        if sw:
            self.tau_sw, self.ssa_sw = f(ncol, nlay, self.ng_sw), f(ncol, nlay, self.ng_sw)
            # the SW boundary conditions, formed every step (unfused: rrtmgpnn_sw_boundary_rfmip; fused: in the SW
            # solver, which uses these only as scratch when its kernel does not form them itself)
            self.toa, self.alb, self.mu0 = f(ncol, self.ng_sw), f(ncol, self.ng_sw), f(ncol)
        if not fused:  # arrays the fused step never materialises
            self.lev_src = f(ncol, nlay + 1, self.ng_lw)
            self.sfc_src, self.sfc_jac = f(ncol, self.ng_lw), f(ncol, self.ng_lw)
        if not fused and sw:
            self.g_sw = f(ncol, nlay, self.ng_sw)
        if self.allsky:
            self.nb_sw = self.kd_sw["nband"]
            self.lwp, self.iwp, self.rel, self.rei = ins[-4:]
            self.cld_tau_lw = f(ncol, nlay, self.nb_lw)
            self.cld_tau_sw, self.cld_ssa_sw, self.cld_g_sw = (f(ncol, nlay, self.nb_sw) for _ in range(3))
            self.cloud_lw, self.cloud_sw = (self._cloud_optics(w, cloud_lut, icergh) for w in ("lw", "sw"))
        self.lw_up, self.lw_dn = f(ncol, nlay + 1), f(ncol, nlay + 1)
        self.sw_up, self.sw_dn, self.sw_dir = f(ncol, nlay + 1), f(ncol, nlay + 1), f(ncol, nlay + 1)
        if not sw:
            for t in (self.sw_up, self.sw_dn, self.sw_dir):
                t.zero_()

        # ---- prepared ctypes argument lists ----
        def gas_args(names):
            ptrs, nds = [], []
            for k, n in enumerate(names):
                t = self.gases.get(n) if k >= 2 else None
                ptrs.append(t.data_ptr() if t is not None else None)
                nds.append(2)
            return ptr_array(ptrs), int_array(nds)

        p = lambda t: t.data_ptr()  # noqa: E731
        self._g_lw, self._nd_lw = gas_args(self.lw_names)
        self._g_sw, self._nd_sw = gas_args(self.sw_names)
        self._nets_lw = ptr_array([h.value for h in self.lw_nets])
        self._nets_sw = ptr_array([h.value for h in self.sw_nets])
        self._lims_lw = int_array(self.kd_lw["band_lims_gpt"].ravel())
        self._Ds, self._W = float_array(GAUSS_DS[nmus]), float_array(GAUSS_WTS[nmus])
        self.nmus = nmus
        c = self.ctx.h
        if fused:
            # compute_nn_inputs + get_col_dry + predict_nn_lw in one kernel (rrtmgpnn_gas_optics_lw_nn): the network
            # inputs and column amounts are formed in-kernel and never stored (same bits as the three calls)
            self.calls = [
                ("predict_nn_lw", L.rrtmgpnn_gas_optics_lw_nn,
                 (c, ncol, nlay, self.ng_lw, self.nx_lw, p(self.play), p(self.tlay), p(self.plev), p(self.gases["h2o"]),
                  self._g_lw, self._nd_lw, self._nets_lw, len(self.lw_nets), p(self.tau_lw), p(self.lay_src))),
            ]
        else:
            self.calls = [
                ("get_col_dry", L.rrtmgpnn_get_col_dry,
                 (c, ncol, nlay, p(self.gases["h2o"]), p(self.plev), p(self.col_dry))),
                ("nn_inputs_lw", L.rrtmgpnn_compute_nn_inputs,
                 (c, ncol, nlay, self.nx_lw, p(self.play), p(self.tlay), self._g_lw, self._nd_lw, self.lw_nets[0],
                  p(self.x_lw))),
                ("predict_nn_lw", L.rrtmgpnn_predict_nn_lw,
                 (c, ncol, nlay, self.ng_lw, self.nx_lw, p(self.x_lw), p(self.col_dry), self._nets_lw,
                  len(self.lw_nets), p(self.tau_lw), p(self.lay_src))),
            ]
        if fused:
            # compute_Planck_source_nn fused into the LW solver (sources formed in-kernel from pfrac); all-sky:
            # the cloud increment by band is added as tau is read (rrtmgpnn_lw_solver_noscat_planck_inc)
            tail = (p(self.tau_lw),) + ((p(self.cld_tau_lw),) if self.allsky else ()) + (
                p(self.lay_src), self.nb_lw, self.kd_lw["nPlanckTemp"], p(self.tlay), p(self.tlev), p(self.tsfc),
                self.sfc_lay, self._lims_lw, float(self.kd_lw["temp_ref_min"][0]), float(self.kd_lw["totplnk_delta"]),
                p(self.totplnk), 1, p(self.sfc_emis), p(self.lw_up), p(self.lw_dn))
            # the surface emissivity goes in by band (as rte_lw takes it) and is expanded in-kernel
            lw_calls = [
                ("lw_solver", L.rrtmgpnn_lw_solver_noscat_planck_inc if self.allsky else L.rrtmgpnn_lw_solver_noscat_planck,
                 (c, self.ng_lw, nlay, ncol, self.top_at_1, nmus, self._Ds, self._W, None) + tail),
            ]
        else:
            lw_calls = [
                ("planck_source", L.rrtmgpnn_compute_planck_source_nn,
                 (c, ncol, nlay, self.nb_lw, self.ng_lw, self.kd_lw["nPlanckTemp"], p(self.tlay), p(self.tlev),
                  p(self.tsfc), self.sfc_lay, self._lims_lw, float(self.kd_lw["temp_ref_min"][0]),
                  float(self.kd_lw["totplnk_delta"]), p(self.totplnk), p(self.sfc_src), p(self.sfc_jac),
                  p(self.lay_src), p(self.lev_src))),
                ("expand_emis", L.rrtmgpnn_expand_band_to_gpt,
                 (c, self.nb_lw, self.ng_lw, ncol, self._lims_lw, p(self.sfc_emis), p(self.emis_gpt))),
                ("lw_solver", L.rrtmgpnn_lw_solver_noscat,
                 (c, self.ng_lw, nlay, ncol, self.top_at_1, nmus, self._Ds, self._W, None, p(self.tau_lw),
                  p(self.lay_src), p(self.lev_src), p(self.emis_gpt), p(self.sfc_src), p(self.lw_up), p(self.lw_dn))),
            ]
        if self.allsky:  # clouds%increment(atmos) before rte_lw (rrtmgp_allsky.F90:383-395)
            self._lims_sw = int_array(self.kd_sw["band_lims_gpt"].ravel())
            self.calls += [
                ("cloud_optics_lw", L.rrtmgpnn_cloud_optics_compute,
                 (c, self.cloud_lw, ncol, nlay, p(self.lwp), p(self.iwp), p(self.rel), p(self.rei),
                  p(self.cld_tau_lw), None, None)),
            ]
            if not fused:
                self.calls += [
                    ("increment_lw", L.rrtmgpnn_increment_bybnd,
                     (c, ncol, nlay, self.ng_lw, self.nb_lw, self._lims_lw, p(self.tau_lw), None, None,
                      p(self.cld_tau_lw), None, None)),
                ]
        self.calls += lw_calls
        if not sw:
            self.calls = [c for c in self.calls if c[0] != "cloud_optics_sw"]
            self._finish(False)
            return
        # the driver's SW boundary conditions.  Fused: formed in the SW solver's prologue
        # (rrtmgpnn_sw_solver_2stream_rfmip).  Round 6 before that: a kernel at the head of the SW chain (7.7 us at C3);
        # on the LW stream beside the SW network, with the SW solver waiting for it, the C3 step measured 0.497 ms against
        # 0.43 (the extra edge into the SW solver let the LW network take the CUs first; profiles/r06/README.md).
        # Unfused (the class layer's calls): the kernel after get_col_dry, the call the SW stream forks after
        if not fused:
            self.calls.insert(1, ("sw_boundary", L.rrtmgpnn_sw_boundary_rfmip,
                                  (c, self.ng_sw, ncol, p(self.solar_source), p(self.tsi), p(self.sfc_alb),
                                   p(self.sza), p(self.toa), p(self.alb), p(self.mu0))))
        # g == NULL: the NN path's asymmetry parameter is identically zero (quirk B-6); the SW kernels take
        # that as a literal 0 instead of writing and re-reading a zero array (same fluxes, bit for bit)
        g_sw = None if fused else p(self.g_sw)
        if fused:
            self.calls += [
                ("predict_nn_sw", L.rrtmgpnn_gas_optics_sw_nn,
                 (c, ncol, nlay, self.ng_sw, self.nx_sw, p(self.play), p(self.tlay), p(self.plev), p(self.gases["h2o"]),
                  self._g_sw, self._nd_sw, self._nets_sw, p(self.tau_sw), p(self.ssa_sw), g_sw)),
            ]
        else:
            self.calls += [
                ("nn_inputs_sw", L.rrtmgpnn_compute_nn_inputs,
                 (c, ncol, nlay, self.nx_sw, p(self.play), p(self.tlay), self._g_sw, self._nd_sw, self.sw_nets[0],
                  p(self.x_sw))),
                ("predict_nn_sw", L.rrtmgpnn_predict_nn_sw,
                 (c, ncol, nlay, self.ng_sw, self.nx_sw, p(self.x_sw), p(self.col_dry), self._nets_sw, p(self.tau_sw),
                  p(self.ssa_sw), g_sw)),
            ]
        if self.allsky:  # clouds%delta_scale(); clouds%increment(atmos) before rte_sw (rrtmgp_allsky.F90:420-433)
            self.calls += [
                ("cloud_optics_sw", L.rrtmgpnn_cloud_optics_compute,
                 (c, self.cloud_sw, ncol, nlay, p(self.lwp), p(self.iwp), p(self.rel), p(self.rei),
                  p(self.cld_tau_sw), p(self.cld_ssa_sw), p(self.cld_g_sw))),
                ("delta_scale_sw", L.rrtmgpnn_delta_scale_2str,
                 (c, ncol * nlay * self.nb_sw, p(self.cld_tau_sw), p(self.cld_ssa_sw), p(self.cld_g_sw), None)),
            ]
            if not fused:
                self.calls += [
                    ("increment_sw", L.rrtmgpnn_increment_bybnd,
                     (c, ncol, nlay, self.ng_sw, self.nb_sw, self._lims_sw, p(self.tau_sw), p(self.ssa_sw), g_sw,
                      p(self.cld_tau_sw), p(self.cld_ssa_sw), p(self.cld_g_sw))),
                ]
        if fused:
            # the boundary conditions and (all sky) clouds%increment(atmos) fused into the solver
            # (rrtmgpnn_sw_solver_2stream_rfmip; same bits as sw_boundary_rfmip + sw_solver_2stream[_inc])
            bnd = (self.nb_sw, self._lims_sw, p(self.cld_tau_sw), p(self.cld_ssa_sw), p(self.cld_g_sw)) \
                if self.allsky else (0, None, None, None, None)
            self.calls += [
                ("sw_solver", L.rrtmgpnn_sw_solver_2stream_rfmip,
                 (c, self.ng_sw, nlay, ncol, self.top_at_1, p(self.solar_source), p(self.tsi), p(self.sfc_alb),
                  p(self.sza), p(self.tau_sw), p(self.ssa_sw), None) + bnd
                 + (p(self.toa), p(self.alb), p(self.mu0), p(self.sw_up), p(self.sw_dn), p(self.sw_dir))),
            ]
        else:
            self.calls += [
                ("sw_solver", L.rrtmgpnn_sw_solver_2stream,
                 (c, self.ng_sw, nlay, ncol, self.top_at_1, p(self.toa), None, p(self.tau_sw), p(self.ssa_sw),
                  g_sw, p(self.mu0), p(self.alb), p(self.alb), p(self.sw_up), p(self.sw_dn), p(self.sw_dir))),
            ]
        self.sw_priority = sw_priority
        self._finish(overlap, lw_after, sw_after, lw_net_cus, sw_net_cus)

    def _finish(self, overlap, lw_after=None, sw_after=None, lw_net_cus=None, sw_net_cus=0):
        # fused: the small kernels that do not depend on a network's output go first in their chain, ahead of the big
        # ones: issued after the LW network (class-layer order), expand_emis waited ~75 us at C3 for CUs the SW solver
        # held while the LW solver, which needs it, could not start
        self.calls = issue_order(self.calls, self.fused)
        # overlap: the SW chain runs on a second context/stream, forked after col_dry (which both streams read; the
        # fused step, whose chains form col_dry each in their network kernel, forks at its start)
        # and joined at the end of the step -- the VALU-bound SW solver shares the CUs with the MFMA-bound LW
        # network and the LW solver instead of running after them
        self.overlap = overlap
        # The LW chain may start once a call of the SW chain has finished (issued first, the SW network then has the
        # chip to itself), and the SW solver may wait for a call of the LW chain (sw_after).  Default: the LW chain
        # after the SW network -- the SW chain is the critical path at every size.  Round 4, alternating whole steps on
        # one box: C3 0.435-0.439 ms, against 0.470-0.473 for both networks first and then the two solvers side by
        # side (the SW solver waiting for both networks) and 0.469-0.476 for the chains started together; C4 2.613-2.618
        # against 2.649-2.670 started together (3 pairs), C5 shard 62.96-63.03 against 63.64-63.65 (2 pairs).  Started
        # together at C4, the SW network ran beside the LW network and solver for 775 us (239 alone) and the SW solver
        # started 1.1 ms into the step.
        names = [n for n, _, _ in self.calls]
        gate = ""
        if overlap and self.fused and "predict_nn_sw" in names and "predict_nn_lw" in names:
            gate = "predict_nn_sw"
        if sw_after is None:
            sw_after = ""
        self.lw_after = (gate if lw_after is None else lw_after) if overlap else ""
        if self.lw_after:
            self.calls = issue_order(self.calls, self.fused, self.lw_after)
            self._gate = torch.cuda.Event()
        # lw_net_cus: the LW network's blocks on at most that many CUs (rrtmgpnn_context_set_mlp_max_cus; 0: all).
        # Default with the LW chain gated on the SW network and an SW solver grid that fits in one round of resident
        # waves (ncol * ngpt_sw / 128 waves of 64 lanes, 2 g-points per lane, against 16 per CU; C3): 3/8 of the CUs.
        # Each LW network block holds most of a CU's LDS (108 KB), so on the full chip it kept the SW solver, launched
        # beside it, off every CU for its first 75 us at C3; confined, it leaves the SW solver the other CUs from the
        # start.  Round 4, C3 whole steps (3 alternating rounds, one box): 0.4350-0.4368 ms on 160 CUs, 0.4374-0.4379
        # on 192, 0.4417-0.4434 on 224, 0.4456-0.4462 on all 256.  Round 6, on the kernels with their prologue loads in
        # flight (4 alternating rounds, profiles/r06/lwcap*_c3.txt): 96 CUs 1.1 % faster than 160 (every round), 128
        # 0.6-1.1 %, 64 and 144 equal.  With more columns (C4) the cap costs 2 % (the SW solver is throughput-bound
        # there; 2.705-2.726 on 192 against 2.651-2.664 ms); C5 equal.
        # A caller's context is left as it is unless lw_net_cus is given.  The caps are overlap measures: without a
        # second stream both networks run on self.ctx, so a cap would confine the SW network too -- refused.
        explicit = lw_net_cus is not None
        if not overlap and (lw_net_cus or sw_net_cus):
            raise ValueError("lw_net_cus / sw_net_cus cap the networks of overlapped chains; overlap is off")
        if lw_net_cus is None:
            lw_net_cus = 0
            cus = torch.cuda.get_device_properties(self.dev).multi_processor_count
            if self._own_ctx and self.overlap and self.lw_after and self.ncol * self.ng_sw <= 2048 * cus:
                lw_net_cus = 3 * cus // 8
        if self._own_ctx or explicit:
            self.ctx.set_mlp_max_cus(int(lw_net_cus))
        # the cap in force on the LW context (a caller's context may carry its own), which bench.py's serialised stage
        # timings lift and restore
        self.lw_net_cus = self.ctx.mlp_max_cus()
        # sw_after: an LW-chain call the SW solver waits for (the two networks first, then the two solvers side by side)
        self.sw_after = sw_after if overlap else ""
        if self.sw_after:
            names = [n for n, _, _ in self.calls]
            if self.sw_after not in names or self.sw_after in SW_CHAIN or "sw_solver" not in names:
                raise ValueError("sw_after: %r is not a call of this fused step's LW chain" % self.sw_after)
            names = [n for n, _, _ in self.calls]
            if names.index(self.sw_after) > names.index("sw_solver"):
                raise ValueError("sw_after: %r is issued after the SW solver" % self.sw_after)
            # the event is recorded on the LW stream right after that call is issued, and the SW stream waits for it
            # right before the SW solver -- the SW network, issued in between, does not wait
            self._gate2 = torch.cuda.Event()
        self.ctx2 = None
        if overlap:
            self.ctx2 = Context(self.dev.index, self._sw_stream())
            # sw_net_cus: the SW network's blocks on at most that many CUs (0: all; an A/B knob, not a default)
            self.sw_net_cus = int(sw_net_cus or 0)
            if self.sw_net_cus:
                check(self.L.rrtmgpnn_context_set_mlp_max_cus(self.ctx2.h, self.sw_net_cus), "context_set_mlp_max_cus")
            self.calls = [(n, f, ((self.ctx2.h,) + tuple(a[1:])) if n in SW_CHAIN else a) for n, f, a in self.calls]
            self._fork, self._join = torch.cuda.Event(), torch.cuda.Event()
        self.graph = None

    def _new_stream(self, priority=0):
        """A stream held by this step alone until close() (_lib.stream_acquire)."""
        h = _lib.stream_acquire(self.dev.index, priority)
        self._streams.append((h, priority))
        return torch.cuda.ExternalStream(h, device=self.dev)

    def _sw_stream(self):
        # default priority: a high-priority SW stream (critical path) was measured 25 % slower at C3 -- it takes every
        # CU first and the chains stop overlapping (tools/ab_prio.sh)
        # sw_priority < 0: a higher-priority stream (the two-solvers-side-by-side schedule, so the SW solver's blocks are
        # dispatched ahead of the LW solver's when both are ready)
        return self._new_stream(getattr(self, "sw_priority", 0))

    def stream_for(self, name):
        """The torch stream a call of `self.calls` is issued on."""
        return self.ctx2.stream if (self.overlap and name in SW_CHAIN) else self.ctx.stream

    def _cloud_optics(self, which, lut, icergh):
        h = _lib.c_vp()
        check(self.L.rrtmgpnn_cloud_optics_load(self.ctx.h, data.cloud_optics_path(which).encode(), int(bool(lut)), h),
              "cloud_optics_load " + which)
        check(self.L.rrtmgpnn_cloud_optics_set_ice_roughness(h, int(icergh)), "set_ice_roughness")
        return h

    def close(self):
        """Release the step's device state in dependency order: finish its work, destroy its hipGraph, then its
        contexts (workspaces, buffer pools) and cloud-optics objects, then hand its streams back.  Left to garbage collection the
        order is the attribute dict's (the contexts before the graph whose nodes address their workspaces).  Idempotent;
        the step is unusable afterwards."""
        if getattr(self, "_closed", True):
            return
        self._closed = True
        torch.cuda.synchronize(self.dev)
        g, self.graph = getattr(self, "graph", None), None
        for x in (g,) + tuple(getattr(self, "chain_graphs", ())):
            if x is not None:
                x.reset()
        self.chain_graphs = ()
        for k in ("cloud_lw", "cloud_sw"):
            h = getattr(self, k, None)
            if h:
                self.L.rrtmgpnn_cloud_optics_destroy(h)
                setattr(self, k, None)
        if getattr(self, "ctx2", None) is not None:
            self.ctx2.close()
        if self._own_ctx:
            self.ctx.close()
        streams, self._streams = self._streams, []
        for h, prio in streams:
            _lib.stream_release(h, self.dev.index, prio)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _enter(self):
        """Order the step after the caller's current stream (the step runs on its own streams); returns the caller's
        stream when it differs from the step's, for _leave."""
        cur = torch.cuda.current_stream(self.dev)
        if cur.cuda_stream == self.ctx.stream.cuda_stream:
            return None
        self.ctx.stream.wait_stream(cur)
        return cur

    def _leave(self, cur):
        if cur is not None:
            cur.wait_stream(self.ctx.stream)

    def step(self, timing=None):
        """Issue one step, ordered after the caller's current stream's work and before its later work.  timing: a dict
        name -> list; each launch is then bracketed by timing events recorded on the stream it runs on (the step's own
        concurrency is unchanged) and (start, end) is appended."""
        cur = self._enter()
        self._issue(timing)
        self._leave(cur)

    def _issue(self, timing=None):
        fork_after = "get_col_dry" if any(n == "get_col_dry" for n, _, _ in self.calls) else None
        if self.overlap and fork_after is None:  # fused step: the chains share no kernel; fork at the start
            self._fork.record(self.ctx.stream)
            self.ctx2.stream.wait_event(self._fork)
        for name, fn, args in self.calls:
            if self.sw_after and name == "sw_solver":
                self.ctx2.stream.wait_event(self._gate2)
            if timing is not None:
                s = self.stream_for(name)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
            rc = fn(*args)
            if rc:
                check(rc, name)
            if timing is not None:
                e1.record(s)
                timing.setdefault(name, []).append((e0, e1))
            if self.overlap and name == fork_after:
                self._fork.record(self.ctx.stream)
                self.ctx2.stream.wait_event(self._fork)
            if self.overlap and name == self.lw_after:
                self._gate.record(self.ctx2.stream)
                self.ctx.stream.wait_event(self._gate)
            if self.sw_after and name == self.sw_after:
                self._gate2.record(self.ctx.stream)
        if self.overlap:
            self._join.record(self.ctx2.stream)
            self.ctx.stream.wait_event(self._join)

    def capture(self):
        """Capture one step into a hipGraph (torch.cuda.CUDAGraph); replay with `replay()`.  The capture runs on the
        step's own streams (a caller's context, which may sit on the legacy null stream, is moved to a capture stream
        the step owns for the duration), with events of its own: no stream or event of the graph is shared with
        another graph or with eager steps."""
        self.step()  # warm-up: kernel attributes + workspace allocation happen outside capture
        torch.cuda.synchronize(self.dev)
        if self.graph is not None:
            self.graph.reset()
            self.graph = None
        self._fork, self._join = torch.cuda.Event(), torch.cuda.Event()
        if self.lw_after:
            self._gate = torch.cuda.Event()
        if self.sw_after:
            self._gate2 = torch.cuda.Event()
        g = torch.cuda.CUDAGraph()
        old = None
        if not self._own_ctx:
            if getattr(self, "_cap_stream", None) is None:
                self._cap_stream = self._new_stream()
            old = self.ctx.stream
            self.ctx.use_stream(self._cap_stream)
        s = self.ctx.stream
        try:
            with torch.cuda.graph(g, stream=s):
                self._issue()
        finally:
            if old is not None:
                self.ctx.use_stream(old)
        self.graph = g
        return g

    def capture_chains(self):
        """A stream of blocks (run_blocks): the SW chain (network, solver with the boundary conditions) and the LW chain
        (network, solver) captured as two hipGraphs, each on its own context's stream and alone -- no gate or join
        between them."""
        if not (self.overlap and self.sw):
            raise ValueError("capture_chains: a step with its LW and SW chains on two streams")
        self.step()  # warm-up outside capture
        torch.cuda.synchronize(self.dev)
        graphs = []
        for chain, ctx in ((lambda n: n in SW_CHAIN, self.ctx2), (lambda n: n not in SW_CHAIN, self.ctx)):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=ctx.stream):
                for name, fn, args in self.calls:
                    if chain(name):
                        rc = fn(*args)
                        if rc:
                            check(rc, name)
            graphs.append(g)
        self.chain_graphs = tuple(graphs)

    def run_blocks(self, k):
        """k blocks streamed through the step: each chain replays k times in its own stream's order, and block b+1's
        SW chain starts as soon as block b's SW solver is done -- beside block b's LW chain -- instead of after
        block b's join.  (A stream of distinct blocks needs each block's inputs and outputs in storage of its own;
        this one re-runs the step's block, whose results are the same every time.)  Ordered after the caller's
        current stream's work and before its later work."""
        g_sw, g_lw = self.chain_graphs
        cur = torch.cuda.current_stream(self.dev)
        for s in (self.ctx2.stream, self.ctx.stream):
            if s.cuda_stream != cur.cuda_stream:
                s.wait_stream(cur)
        for _ in range(k):
            with torch.cuda.stream(self.ctx2.stream):
                g_sw.replay()
            with torch.cuda.stream(self.ctx.stream):
                g_lw.replay()
        for s in (self.ctx2.stream, self.ctx.stream):
            if s.cuda_stream != cur.cuda_stream:
                cur.wait_stream(s)

    def replay(self):
        """Launch the captured step on the step's stream, ordered after the caller's current stream's work and before
        its later work."""
        cur = self._enter()
        with torch.cuda.stream(self.ctx.stream):
            self.graph.replay()
        self._leave(cur)

    def _inputs(self, prob, clouds=None):
        """Device input tensors of a host problem, in io_tensors() order: the state, the gases, the surface emissivity
        by band, and the driver's per-column SW state -- solar zenith angle, TSI, surface albedo (rrtmgp_rfmip_sw.F90:
        244-259) -- (+ the cloud fields)."""
        dev = self.dev
        ins = [_t(prob[k], dev) for k in ("play", "plev", "tlay", "tlev", "tsfc")]
        ins += [_t(prob["gases"][k], dev) for k in self._gas_names]
        ins += [_t(np.repeat(prob["sfc_emis"][:, None], self.nb_lw, axis=1), dev),  # (ncol, nband)
                _t(prob["sza"], dev), _t(prob["tsi"], dev), _t(prob["sfc_alb"], dev)]
        if clouds is not None:
            ins += [_t(a, dev) for a in clouds]
        return ins

    def inputs_for(self, prob, clouds=None):
        """io_tensors()-ordered device inputs of another block of the same shape (bench.py's chunked shard: copied
        into this step's inputs before each replay)."""
        if prob["ncol"] != self.ncol or prob["nlay"] != self.nlay or list(prob["gases"]) != self._gas_names:
            raise ValueError("inputs_for: block shape differs from the step's")
        return self._inputs(prob, clouds if self.allsky else None)

    def io_tensors(self):
        """(inputs, outputs): the device tensors a host-resident caller would upload / download per step."""
        ins = [self.play, self.plev, self.tlay, self.tlev, self.tsfc, *self.gases.values(), self.sfc_emis, self.sza,
               self.tsi, self.sfc_alb]
        if self.allsky:
            ins += [self.lwp, self.iwp, self.rel, self.rei]
        return ins, [self.lw_up, self.lw_dn, self.sw_up, self.sw_dn, self.sw_dir]

    def fluxes(self):
        """Host copies of the broadband fluxes, with SW zeroed where sza >= 90 is applied by the caller."""
        return {k: getattr(self, k).cpu().numpy() for k in ("lw_up", "lw_dn", "sw_up", "sw_dn", "sw_dir")}


class ChunkedRank:
    """A rank's column range [lo, hi) streamed through one step in chunks (bench.py --global: a C5 rank holds more
    columns than one step's block).  Every chunk's inputs stay resident in HBM; `run()` copies each chunk's inputs
    into the step's input tensors (device to device, on the step's stream), replays the step (its hipGraph when
    captured) and copies its fluxes into the rank's flux slab `flux` (lw_up, lw_dn, sw_up, sw_dn, sw_dir; (hi - lo,
    nlay + 1) each).  A short last chunk runs through a second step of its own shape.

    problem(c0, c1) -> (prob, clouds): columns [c0, c1) of the global problem.  make_step(prob, clouds) -> a
    ClearSkyStep of that block's shape."""

    def __init__(self, lo, hi, chunk, problem, make_step, use_graph=True):
        self.lo, self.hi = lo, hi
        self.chunks = shard.chunk_ranges(lo, hi, chunk)
        self.steps, self._run_of, self.chunk_ins, self._step_of = [], [], [], []
        for k, (c0, c1) in enumerate(self.chunks):
            prob, clouds = problem(c0, c1)
            if k == 0:
                self.first = (prob, clouds)  # the first chunk's host problem (bench.py's CPU baseline samples it)
            st = next((s for s in self.steps if s.ncol == c1 - c0), None)
            if st is None:
                st = make_step(prob, clouds)
                self.steps.append(st)
                ins, _ = st.io_tensors()
                self.chunk_ins.append([t.clone() for t in ins] if len(self.chunks) > 1 else None)
                if use_graph:
                    st.capture()
            else:
                self.chunk_ins.append(st.inputs_for(prob, clouds))
            self._step_of.append(st)
        self.step = self.steps[0]
        dev = self.step.dev
        outs = self.step.io_tensors()[1]
        self.single = len(self.chunks) == 1
        self.flux = list(outs) if self.single else [
            torch.empty((hi - lo,) + tuple(o.shape[1:]), dtype=o.dtype, device=dev) for o in outs]
        self.use_graph = use_graph

    def run(self):
        """One pass over the rank's columns, ordered after the caller's current stream's work and before its later
        work (the chunks run on their steps' own streams; no ordering is needed between the two steps' chunks: their
        buffers and slab rows are disjoint)."""
        if self.single:
            st = self.step
            st.replay() if self.use_graph else st.step()
            return
        cur = torch.cuda.current_stream(self.step.dev)
        used = []
        for (c0, c1), st, src in zip(self.chunks, self._step_of, self.chunk_ins):
            ins, outs = st.io_tensors()
            s = st.ctx.stream
            if st not in used:
                used.append(st)
                if s.cuda_stream != cur.cuda_stream:
                    s.wait_stream(cur)
            with torch.cuda.stream(s):
                for d, x in zip(ins, src):
                    d.copy_(x, non_blocking=True)
                st.replay() if self.use_graph else st.step()
                for r, o in zip(self.flux, outs):
                    r[c0 - self.lo:c1 - self.lo].copy_(o, non_blocking=True)
        for st in used:
            if st.ctx.stream.cuda_stream != cur.cuda_stream:
                cur.wait_stream(st.ctx.stream)

    def close(self):
        """Release every step (ClearSkyStep.close: graph, contexts, streams, in that order)."""
        for st in self.steps:
            st.close()
