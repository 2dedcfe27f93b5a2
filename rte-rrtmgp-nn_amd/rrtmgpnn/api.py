"""Host-side mirror of the reference's class layer, on torch device tensors, over the C ABI.

Names, argument meaning and error behaviour follow the reference:
  rrtmgp_network_type            neural/mod_network_rrtmgp.F90:34-122       -> RrtmgpNetwork
  ty_gas_concs                   rrtmgp/mo_gas_concentrations.F90:50-444    -> GasConcs
  ty_optical_props_1scl/2str     rte/mo_optical_props.F90:62-210           -> OpticalProps1scl/2str
  ty_source_func_lw              rte/mo_source_functions.F90:26-136        -> SourceFuncLW
  ty_fluxes_broadband            rte/mo_fluxes.F90:46-67                   -> FluxesBroadband
  ty_gas_optics_rrtmgp%gas_optics  rrtmgp/mo_gas_optics_rrtmgp.F90:239-602 -> GasOpticsRRTMGP.gas_optics
  rte_lw                         rte/mo_rte_lw.F90:60-424                  -> rte_lw
  rte_sw                         rte/mo_rte_sw.F90:48-266                  -> rte_sw
  ty_cloud_optics                extensions/cloud_optics/mo_cloud_optics.F90 -> CloudOptics
  ty_optical_props_arry%increment / %delta_scale  rte/mo_optical_props.F90:882-1023, 565-604
  rte_config_checks              rte/mo_rte_rrtmgp_config.F90:45-61        -> rte_config_checks
Class-level functions RETURN an error message ('' on success), never raise for user errors, like the
reference's `character(len=128) error_msg`; `stop_on_err` turns one into an exception.

Layout: torch tensors in C order with the Fortran shape reversed (reference tau(ngpt,nlay,ncol) is
tensor (ncol, nlay, ngpt) here): the bytes are identical, so the kernels see the reference layout.
All compute runs in HIP kernels of librrtmgpnn.so; there is no torch/CPU compute path.
"""
import ctypes

import numpy as np
import torch

from . import _lib, data, rbin
from ._lib import check, float_array, int_array, ptr_array

_CTX = {}
# mo_rte_rrtmgp_config: value checks off by default, as in the reference (:23-24); extents are always checked
check_values = False


def rte_config_checks(logical):
    """rte_config_checks (rte/mo_rte_rrtmgp_config.F90:56-61)."""
    global check_values
    check_values = bool(logical)


class Context:
    """A rrtmgpnn_context bound to a device and a HIP stream (default: torch's current stream)."""

    def __init__(self, device=0, stream=None):
        L = _lib.lib()
        self.device = int(device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self.stream = s
        h = _lib.c_vp()
        check(L.rrtmgpnn_context_create(self.device, s.cuda_stream, h), "context_create")
        self.h = h

    def use_stream(self, stream):
        check(_lib.lib().rrtmgpnn_context_set_stream(self.h, stream.cuda_stream), "context_set_stream")
        self.stream = stream

    def synchronize(self):
        check(_lib.lib().rrtmgpnn_context_synchronize(self.h), "context_synchronize")

    def unpin_workspace(self):
        """After destroying every hipGraph captured on this context: let its workspace grow again."""
        check(_lib.lib().rrtmgpnn_context_unpin_workspace(self.h), "context_unpin_workspace")

    def set_sw_kernel(self, mode):
        """0: SW two-stream kernel by ngpt (two g-points per lane when even; default); 1 / 2: one / two (bit-identical)."""
        check(_lib.lib().rrtmgpnn_context_set_sw_kernel(self.h, int(mode)), "context_set_sw_kernel")

    def set_mlp_max_cus(self, cus):
        """The gas-optics networks launched on this context on at most `cus` CUs (0: all; bit-identical)."""
        check(_lib.lib().rrtmgpnn_context_set_mlp_max_cus(self.h, int(cus)), "context_set_mlp_max_cus")

    def mlp_max_cus(self):
        """The network CU cap in force on this context (0: every CU)."""
        v = ctypes.c_int(0)
        check(_lib.lib().rrtmgpnn_context_get_mlp_max_cus(self.h, ctypes.byref(v)), "context_get_mlp_max_cus")
        return v.value

    def set_mlp_kernel(self, mode):
        """0: the gas-optics networks on 32x32x2 MFMA tiles where instantiated (default); 1: 16x16x4 (bit-identical)."""
        check(_lib.lib().rrtmgpnn_context_set_mlp_kernel(self.h, int(mode)), "context_set_mlp_kernel")

    def close(self):
        """Destroy the context now (its workspace and buffer pool); the handle is unusable afterwards."""
        h, self.h = getattr(self, "h", None), None
        if h:
            _lib.lib().rrtmgpnn_context_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def set_mlp_kernel_default(mode):
    """The gas-optics networks' MFMA tiling of every context not set itself: 0 32x32x2 where instantiated (the default),
    1 16x16x4 (bit-identical outputs; tests force each)."""
    check(_lib.lib().rrtmgpnn_context_set_mlp_kernel(None, int(mode)), "context_set_mlp_kernel")


def set_sw_kernel_default(mode):
    """The SW two-stream kernel of every context not set itself: 0 by ngpt (the default), 1 / 2 one /
    two g-points per lane (bit-identical fluxes; tests force each)."""
    check(_lib.lib().rrtmgpnn_context_set_sw_kernel(None, int(mode)), "context_set_sw_kernel")


def context(device=None):
    """Per-device default context on torch's current stream."""
    if device is None:
        device = torch.cuda.current_device()
    dev = int(device)
    c = _CTX.get(dev)
    cur = torch.cuda.current_stream(dev)
    if c is None:
        c = _CTX[dev] = Context(dev, cur)
    elif c.stream.cuda_stream != cur.cuda_stream:
        c.use_stream(cur)
    return c


def _p(t):
    return t.data_ptr() if t is not None else None


def _f32dev(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.float32).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float32), device=device)


def stop_on_err(msg):
    if msg:
        raise RuntimeError(msg)


# ---------------------------------------------------------------------------------------------
class RrtmgpNetwork:
    """rrtmgp_network_type: an MLP plus its input/output scaling (neural/mod_network_rrtmgp.F90:34-53)."""

    def __init__(self, device=None):
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.h = None

    def load_netcdf(self, filename):
        """neural/mod_network_rrtmgp.F90:58-122.  `filename` is the reference's netCDF model file (read natively,
        csrc/datafile.cpp) or its RBIN conversion."""
        from . import ncio
        with ncio.DataFile(filename) as f:
            if "nn_dimsize" in f:  # the netCDF model: nn_dim_input, nn_dimsize, nn_activation_char, ...
                self.dims = [int(f.read("nn_input_coeffs_min").size)] + [int(v) for v in f.read("nn_dimsize")]
                acts = ["linear", "softsign", "relu", "sigmoid", "hard_sigmoid", "tanh", "gaussian"]
                self.activation = [acts.index(a) for a in f.strings("nn_activation_char")]
                self.input_names = f.strings("nn_inputs_char") if "nn_inputs_char" in f else [""] * self.dims[0]
                self.coeffs_input_min = f.read("nn_input_coeffs_min", np.float32)
                self.coeffs_input_max = f.read("nn_input_coeffs_max", np.float32)
                has_out = "nn_output_coeffs_mean" in f
                self.coeffs_output_mean = f.read("nn_output_coeffs_mean", np.float32) if has_out else None
                self.coeffs_output_std = f.read("nn_output_coeffs_std", np.float32) if has_out else None
                m = {"dims": np.array(self.dims, np.int32), "activation": np.array(self.activation, np.int32),
                     "input_names": rbin.chars(self.input_names), "input_min": self.coeffs_input_min,
                     "input_max": self.coeffs_input_max}
                for n in range(1, len(self.dims)):
                    m["w%d" % n] = f.read("nn_weights_%d" % n, np.float32)
                    m["b%d" % n] = f.read("nn_bias_%d" % n, np.float32)
                if has_out:
                    m["output_mean"], m["output_std"] = self.coeffs_output_mean, self.coeffs_output_std
            else:
                m = {v: f.read(v) for v in f.vars}
                self.dims = [int(v) for v in m["dims"]]
                self.activation = [int(v) for v in m["activation"]]
                self.input_names = rbin.unchars(m["input_names"]) if "input_names" in m else [""] * self.dims[0]
                self.coeffs_input_min = m["input_min"]
                self.coeffs_input_max = m["input_max"]
                self.coeffs_output_mean = m.get("output_mean")
                self.coeffs_output_std = m.get("output_std")
        self.model = m
        ctx = context(self.device)
        h = _lib.c_vp()
        check(_lib.lib().rrtmgpnn_network_load(ctx.h, str(filename).encode(), h), "network_load(%s)" % filename)
        self.h = h
        return self

    load = load_netcdf

    @property
    def nlayers(self):
        return len(self.dims) - 1

    def output_sgemm_flat(self, x):
        """network_type%output_sgemm_flat (neural/mod_network.F90:273): x (nbatch, nx) -> (nbatch, ny)."""
        x = _f32dev(x, "cuda:%d" % self.device)
        nb = x.numel() // self.dims[0]
        out = torch.empty((nb, self.dims[-1]), dtype=torch.float32, device=x.device)
        check(_lib.lib().rrtmgpnn_network_forward(context(self.device).h, self.h, nb, _p(x), _p(out)), "network_forward")
        return out

    def __del__(self):
        try:
            if self.h:
                _lib.lib().rrtmgpnn_network_destroy(self.h)
        except Exception:
            pass


# ---------------------------------------------------------------------------------------------
class GasConcs:
    """ty_gas_concs: per-gas scalar / (nlay) / (ncol,nlay) volume mixing ratios (device tensors)."""

    def init(self, gas_names):
        self.gas_name = [g.strip().lower() for g in gas_names]
        if len(set(self.gas_name)) != len(self.gas_name):
            return "ty_gas_concs%init(): duplicate gas names"
        self.concs = {}
        return ""

    def set_vmr(self, gas, w, device=None):
        gas = gas.strip().lower()
        if gas not in self.gas_name:
            return "ty_gas_concs%set_vmr(): trying to set " + gas + " but name not present"
        if isinstance(w, (float, int, np.floating)):
            if w < 0 or w > 1:
                return "ty_gas_concs%set_vmr(): concentrations should be >= 0, <= 1"
            self.concs[gas] = torch.tensor([float(w)], dtype=torch.float32,
                                           device=device or "cuda:%d" % torch.cuda.current_device())
            return ""
        t = _f32dev(w, device or "cuda:%d" % torch.cuda.current_device())
        if t.numel() and (bool((t < 0).any()) or bool((t > 1).any())):
            return "ty_gas_concs%set_vmr(): concentrations should be >= 0, <= 1"
        self.concs[gas] = t
        return ""

    def get_gas_names(self):
        return list(self.gas_name)

    def ndims(self, gas):
        t = self.concs[gas]
        return 0 if t.numel() == 1 and t.dim() <= 1 else t.dim()


# ---------------------------------------------------------------------------------------------
class OpticalProps:
    """ty_optical_props: spectral discretisation (band limits in wavenumber and g-point)."""

    def init(self, band_lims_wvn, band_lims_gpt=None, name=""):
        wv = np.asarray(band_lims_wvn, np.float32).reshape(-1, 2)
        if band_lims_gpt is None:
            band_lims_gpt = np.stack([np.arange(1, wv.shape[0] + 1)] * 2, axis=1)
        gp = np.asarray(band_lims_gpt, np.int32).reshape(-1, 2)
        if (wv < 0).any():
            return "optical_props%init(): band_lims_wvn has values <  0., respectively"
        if gp.min() < 1:
            return "optical_props%init(): band_lims_gpt has values < 1"
        self.band_lims_wvn, self.band_lims_gpt, self.name = wv, gp, name
        return ""

    def init_from(self, other):
        return self.init(other.band_lims_wvn, other.band_lims_gpt, getattr(other, "name", ""))

    def get_nband(self):
        return int(self.band_lims_gpt.shape[0])

    def get_ngpt(self):
        return int(self.band_lims_gpt[:, 1].max())

    def get_band_lims_gpoint(self):
        return self.band_lims_gpt.copy()

    def get_band_lims_wavenumber(self):
        return self.band_lims_wvn.copy()

    def get_gpoint_bands(self):
        b = np.zeros(self.get_ngpt(), np.int32)
        for i, (lo, hi) in enumerate(self.band_lims_gpt):
            b[lo - 1:hi] = i + 1
        return b

    def bands_are_equal(self, that):
        """rte/mo_optical_props.F90:1204-1214: same nband and limits within 5 spacings."""
        if self.get_nband() != that.get_nband() or self.get_nband() <= 0:
            return False
        a, b = self.band_lims_wvn, that.band_lims_wvn
        return bool((np.abs(a - b) < np.float32(5) * np.spacing(a)).all())

    def gpoints_are_equal(self, that):
        """rte/mo_optical_props.F90:1220-1229."""
        return self.bands_are_equal(that) and self.get_ngpt() == that.get_ngpt() and \
            bool((self.get_gpoint_bands() == that.get_gpoint_bands()).all())

    def is_initialized(self):
        return getattr(self, "band_lims_gpt", None) is not None


class _OpticalPropsArry(OpticalProps):
    ssa = g = None

    def get_ncol(self):
        return int(self.tau.shape[0])

    def get_nlay(self):
        return int(self.tau.shape[1])

    def increment(self, op_io):
        """op_in%increment(op_io) (rte/mo_optical_props.F90:882-1023): add self's optical properties to op_io,
        at the same g-point resolution or, when self is defined by band, by band into op_io's g-points."""
        if not self.bands_are_equal(op_io):
            return "ty_optical_props%increment: optical properties objects have different band structures"
        ncol, nlay, ngpt = op_io.get_ncol(), op_io.get_nlay(), op_io.get_ngpt()
        if self.get_ncol() != ncol or self.get_nlay() != nlay:
            return "ty_optical_props%increment: optical properties objects have different extents"
        io2, in2 = isinstance(op_io, OpticalProps2str), isinstance(self, OpticalProps2str)
        ctx = context(op_io.tau.device.index)
        L = _lib.lib()
        args = (_p(op_io.tau), _p(op_io.ssa) if io2 else None, _p(op_io.g) if io2 else None,
                _p(self.tau), _p(self.ssa) if in2 else None, _p(self.g) if in2 else None)
        if self.gpoints_are_equal(op_io):
            check(L.rrtmgpnn_increment(ctx.h, ncol, nlay, ngpt, *args), "increment")
            return ""
        # Values defined by band have ngpt() = nband() (:955-958)
        if self.get_ngpt() != op_io.get_nband():
            return "ty_optical_props%increment: optical properties objects have incompatible g-point structures"
        check(L.rrtmgpnn_increment_bybnd(ctx.h, ncol, nlay, ngpt, op_io.get_nband(),
                                         int_array(op_io.band_lims_gpt.ravel()), *args), "increment_bybnd")
        return ""


class OpticalProps1scl(_OpticalPropsArry):
    def alloc_1scl(self, ncol, nlay, spec=None, device=None):
        if spec is not None:
            e = self.init_from(spec)
            if e:
                return e
        if ncol <= 0 or nlay <= 0:
            return "optical_props%alloc: must provide positive extents for ncol, nlay"
        dev = device or "cuda:%d" % torch.cuda.current_device()
        self.tau = torch.zeros((ncol, nlay, self.get_ngpt()), dtype=torch.float32, device=dev)
        return ""

    def delta_scale(self, for_=None):
        """delta_scale_1scl (rte/mo_optical_props.F90:565-574): nothing to do for absorption optical depth."""
        return ""


class OpticalProps2str(_OpticalPropsArry):
    def alloc_2str(self, ncol, nlay, spec=None, device=None):
        if spec is not None:
            e = self.init_from(spec)
            if e:
                return e
        if ncol <= 0 or nlay <= 0:
            return "optical_props%alloc: must provide positive extents for ncol, nlay"
        dev = device or "cuda:%d" % torch.cuda.current_device()
        shape = (ncol, nlay, self.get_ngpt())
        self.tau = torch.zeros(shape, dtype=torch.float32, device=dev)
        self.ssa = torch.zeros(shape, dtype=torch.float32, device=dev)
        self.g = torch.zeros(shape, dtype=torch.float32, device=dev)
        return ""

    def validate(self):
        """validate_2stream (rte/mo_optical_props.F90:635-671)."""
        if self.tau.shape != self.ssa.shape or self.tau.shape != self.g.shape:
            return "validate: arrays not sized consistently"
        e = ""
        if bool((self.tau < 0).any()):
            e = "validate: tau values out of range"
        if bool(((self.ssa < 0) | (self.ssa > 1.0001)).any()):
            e = "validate: ssa values out of range"
        if bool(((self.g < -1) | (self.g > 1)).any()):
            e = "validate: g values out of range"
        return e

    def delta_scale(self, for_=None):
        """delta_scale_2str (rte/mo_optical_props.F90:576-604); forward fraction g**2 unless `for_` is given."""
        ctx = context(self.tau.device.index)
        fw = None
        if for_ is not None:
            fw = _f32dev(for_, self.tau.device)
            if tuple(fw.shape) != tuple(self.tau.shape):
                return "delta_scale: dimension of 'for' don't match optical properties arrays"
            if bool((fw < 0).any()) or bool((fw > 1).any()):
                return "delta_scale: values of 'for' out of bounds [0,1]"
        check(_lib.lib().rrtmgpnn_delta_scale_2str(ctx.h, self.tau.numel(), _p(self.tau), _p(self.ssa), _p(self.g),
                                                   _p(fw)), "delta_scale_2str")
        return ""


class SourceFuncLW(OpticalProps):
    def alloc(self, ncol, nlay, spec=None, device=None):
        if spec is not None:
            e = self.init_from(spec)
            if e:
                return e
        if ncol <= 0 or nlay <= 0:
            return "source_func_lw%alloc: must provide positive extents for ncol, nlay"
        dev = device or "cuda:%d" % torch.cuda.current_device()
        ng = self.get_ngpt()
        self.lay_source = torch.zeros((ncol, nlay, ng), dtype=torch.float32, device=dev)
        self.lev_source = torch.zeros((ncol, nlay + 1, ng), dtype=torch.float32, device=dev)
        self.sfc_source = torch.zeros((ncol, ng), dtype=torch.float32, device=dev)
        self.sfc_source_Jac = torch.zeros((ncol, ng), dtype=torch.float32, device=dev)
        return ""

    def get_ncol(self):
        return int(self.lay_source.shape[0])

    def get_nlay(self):
        return int(self.lay_source.shape[1])


class FluxesBroadband:
    """ty_fluxes_broadband: (ncol, nlay+1) outputs the caller allocates (pointers into caller memory)."""

    def __init__(self, flux_up=None, flux_dn=None, flux_dn_dir=None, flux_net=None):
        self.flux_up, self.flux_dn, self.flux_dn_dir, self.flux_net = flux_up, flux_dn, flux_dn_dir, flux_net

    def are_desired(self):
        return any(x is not None for x in (self.flux_up, self.flux_dn, self.flux_dn_dir, self.flux_net))

    def are_desired_gpt(self):
        return False


class FluxesFlexible(FluxesBroadband):
    """ty_fluxes_flexible (rte/mo_fluxes.F90:57-67): the broadband outputs plus g-point fluxes, (ncol, nlay+1, ngpt)
    tensors the caller allocates.  rte_lw fills gpt_flux_up/dn (no-scattering and rescaled solutions: with one angle
    the g-point radiances, quirk B-5, with several the angle-summed fluxes; use_2stream: the adding fluxes), rte_sw
    gpt_flux_up/dn (total)/dn_dir on 2str properties and gpt_flux_dn_dir (the spectral direct beam) on 1scl ones;
    gpt_flux_net is not written (as in the reference)."""

    def __init__(self, flux_up=None, flux_dn=None, flux_dn_dir=None, flux_net=None, gpt_flux_up=None,
                 gpt_flux_dn=None, gpt_flux_dn_dir=None, gpt_flux_net=None):
        super().__init__(flux_up, flux_dn, flux_dn_dir, flux_net)
        self.gpt_flux_up, self.gpt_flux_dn = gpt_flux_up, gpt_flux_dn
        self.gpt_flux_dn_dir, self.gpt_flux_net = gpt_flux_dn_dir, gpt_flux_net

    def are_desired_gpt(self):
        return any(x is not None for x in (self.gpt_flux_up, self.gpt_flux_dn, self.gpt_flux_dn_dir, self.gpt_flux_net))


# ---------------------------------------------------------------------------------------------
class GasOpticsRRTMGP(OpticalProps):
    """ty_gas_optics_rrtmgp, NN branch.  The lookup-table branch needs the k-distribution files that are
    missing from the reference and is not provided."""

    def load(self, which, device=None):
        """Load the (surrogate) k-distribution tables, 'lw' (g256) or 'sw' (g224)."""
        kd = data.load_kdist(which)
        e = self.init(kd["band_lims_wvn"], kd["band_lims_gpt"])
        if e:
            return e
        self.kd = kd
        self.dev = device or "cuda:%d" % torch.cuda.current_device()
        self.press_ref_min = float(kd["press_ref_min"][0])
        self.temp_ref_min = float(kd["temp_ref_min"][0])
        self.temp_ref_max = float(kd["temp_ref_max"][0])
        if which == "lw":
            self.totplnk = torch.as_tensor(kd["totplnk"], device=self.dev)  # (nbnd, nPlanckTemp) = Fortran (nT, nbnd)
            self.totplnk_delta = float(kd["totplnk_delta"])
            self.solar_source = None
        else:
            self.totplnk = None
            self.solar_source = np.asarray(kd["solar_source"], np.float32).copy()
        return ""

    def source_is_internal(self):
        return self.totplnk is not None

    def source_is_external(self):
        return self.solar_source is not None

    def get_press_min(self):
        return self.press_ref_min

    def get_temp_min(self):
        return self.temp_ref_min

    def get_temp_max(self):
        return self.temp_ref_max

    def get_nPlanckTemp(self):
        return int(self.totplnk.shape[1])

    def set_tsi(self, tsi):
        if tsi < 0:
            return "tsi out of range"
        self.solar_source = data.set_tsi(self.solar_source, tsi)
        return ""

    # -- helpers ----
    def _nn_inputs(self, ctx, play, tlay, gas_desc, net):
        ncol, nlay = play.shape
        nx = net.dims[0]
        ptrs, nds, keep = [], [], []
        for k, name in enumerate(net.input_names):
            if k < 2 or name not in gas_desc.concs:
                ptrs.append(None)
                nds.append(2)
                continue
            t = gas_desc.concs[name]
            keep.append(t)
            ptrs.append(t.data_ptr())
            nds.append(gas_desc.ndims(name))
        if net.input_names[2] not in gas_desc.concs or net.input_names[3] not in gas_desc.concs:
            return None, "compute_nn_inputs: gas " + net.input_names[2] + "/" + net.input_names[3] + " not found"
        x = torch.empty((ncol, nlay, nx), dtype=torch.float32, device=play.device)
        check(_lib.lib().rrtmgpnn_compute_nn_inputs(ctx.h, ncol, nlay, nx, _p(play), _p(tlay), ptr_array(ptrs),
                                                    int_array(nds), net.h, _p(x)), "compute_nn_inputs")
        return x, ""

    def gas_optics(self, play, plev, tlay, *args, **kw):
        """LW: gas_optics(play, plev, tlay, tsfc, gas_desc, optical_props, sources, col_dry=, tlev=, neural_nets=)
        SW: gas_optics(play, plev, tlay, gas_desc, optical_props, toa_src, col_dry=, neural_nets=)"""
        if self.source_is_internal():
            return self._gas_optics_int(play, plev, tlay, *args, **kw)
        return self._gas_optics_ext(play, plev, tlay, *args, **kw)

    def _common(self, play, plev, tlay, gas_desc, optical_props, col_dry):
        ncol, nlay = play.shape
        if plev.shape != (ncol, nlay + 1) or tlay.shape != (ncol, nlay):
            return None, "gas_optics(): array plev/tlay has wrong size"
        if optical_props.get_ngpt() != self.get_ngpt() or optical_props.get_ncol() != ncol or \
                optical_props.get_nlay() != nlay:
            return None, "gas_optics(): optical properties inconsistently sized"
        ctx = context(play.device.index)
        if col_dry is None:
            if "h2o" not in gas_desc.concs:
                return None, "gas_optics(): h2o concentration is required"
            col_dry = torch.empty((ncol, nlay), dtype=torch.float32, device=play.device)
            check(_lib.lib().rrtmgpnn_get_col_dry(ctx.h, ncol, nlay, _p(gas_desc.concs["h2o"]), _p(plev), _p(col_dry)),
                  "get_col_dry")
        return (ctx, col_dry), ""

    def _gas_optics_int(self, play, plev, tlay, tsfc, gas_desc, optical_props, sources, col_dry=None, tlev=None,
                        neural_nets=None):
        if neural_nets is None:
            return "gas_optics(): the lookup-table branch is not available (k-distribution files missing); pass neural_nets"
        r, e = self._common(play, plev, tlay, gas_desc, optical_props, col_dry)
        if e:
            return e
        ctx, cd = r
        ncol, nlay = play.shape
        ngpt = self.get_ngpt()
        L = _lib.lib()
        if tlev is None:  # mo_gas_optics_rrtmgp.F90:317-337
            tlev = torch.empty((ncol, nlay + 1), dtype=torch.float32, device=play.device)
            check(L.rrtmgpnn_interpolate_tlev(ctx.h, ncol, nlay, _p(play), _p(plev), _p(tlay), _p(tlev)), "tlev")
        x, e = self._nn_inputs(ctx, play, tlay, gas_desc, neural_nets[0])
        if e:
            return e
        nets = ptr_array([n.h.value for n in neural_nets])
        check(L.rrtmgpnn_predict_nn_lw(ctx.h, ncol, nlay, ngpt, neural_nets[0].dims[0], _p(x), _p(cd), nets,
                                       len(neural_nets), _p(optical_props.tau), _p(sources.lay_source)),
              "predict_nn_lw")
        sfc_lay = 1 if float(play[0, 0]) > float(play[0, nlay - 1]) else nlay  # :402
        check(L.rrtmgpnn_compute_planck_source_nn(
            ctx.h, ncol, nlay, self.get_nband(), ngpt, self.get_nPlanckTemp(), _p(tlay), _p(tlev), _p(tsfc), sfc_lay,
            int_array(self.band_lims_gpt.ravel()), self.temp_ref_min, self.totplnk_delta, _p(self.totplnk),
            _p(sources.sfc_source), _p(sources.sfc_source_Jac), _p(sources.lay_source), _p(sources.lev_source)),
            "compute_planck_source_nn")
        return ""

    def _gas_optics_ext(self, play, plev, tlay, gas_desc, optical_props, toa_src, col_dry=None, neural_nets=None):
        if neural_nets is None:
            return "gas_optics(): the lookup-table branch is not available (k-distribution files missing); pass neural_nets"
        r, e = self._common(play, plev, tlay, gas_desc, optical_props, col_dry)
        if e:
            return e
        ctx, cd = r
        ncol, nlay = play.shape
        ngpt = self.get_ngpt()
        x, e = self._nn_inputs(ctx, play, tlay, gas_desc, neural_nets[0])
        if e:
            return e
        nets = ptr_array([n.h.value for n in neural_nets])
        is2 = isinstance(optical_props, OpticalProps2str)
        check(_lib.lib().rrtmgpnn_predict_nn_sw(
            ctx.h, ncol, nlay, ngpt, neural_nets[0].dims[0], _p(x), _p(cd), nets, _p(optical_props.tau),
            _p(optical_props.ssa) if is2 else None, _p(optical_props.g) if is2 else None), "predict_nn_sw")
        if tuple(toa_src.shape) != (ncol, ngpt):
            return "gas_optics(): array toa_src has wrong size"
        toa_src.copy_(torch.as_tensor(self.solar_source, device=toa_src.device).expand(ncol, ngpt))  # :594-599
        return ""


# ---------------------------------------------------------------------------------------------
class CloudOptics(OpticalProps):
    """ty_cloud_optics (extensions/cloud_optics/mo_cloud_optics.F90): liquid + ice cloud optical properties by
    band from a lookup table or Pade approximants of effective radius.  Tables live on the device."""

    def __init__(self, device=None):
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.h = None

    def _adopt(self, h):
        if self.h:
            _lib.lib().rrtmgpnn_cloud_optics_destroy(self.h)
        self.h = h
        nb, nr = _lib.c_int(), _lib.c_int()
        r = (_lib.c_float * 4)()
        check(_lib.lib().rrtmgpnn_cloud_optics_get(h, nb, nr, r), "cloud_optics_get")
        self.nrghice = nr.value
        self.radii = [float(v) for v in r]
        self.icergh = 1
        return ""

    def load(self, which, use_lut=True):
        """Coefficients of extensions/cloud_optics/rrtmgp-cloud-optics-coeffs-{lw,sw}.nc (RBIN conversion);
        the LUT (load_lut) or Pade (load_pade) method."""
        return self._load_path(data.cloud_optics_path(which), use_lut)

    def _load_path(self, path, use_lut=True):
        """The coefficient file itself (classic netCDF, read natively) or its RBIN conversion."""
        from . import ncio
        with ncio.DataFile(path) as f:
            wvn = f.read("bnd_limits_wavenumber", np.float32)
        e = self.init(wvn, name="RRTMGP cloud optics")
        if e:
            return e
        h = _lib.c_vp()
        check(_lib.lib().rrtmgpnn_cloud_optics_load(context(self.device).h, str(path).encode(), int(bool(use_lut)), h),
              "cloud_optics_load(%s)" % path)
        return self._adopt(h)

    def load_lut(self, band_lims_wvn, radliq_lwr, radliq_upr, radice_lwr, radice_upr, lut_extliq, lut_ssaliq,
                 lut_asyliq, lut_extice, lut_ssaice, lut_asyice):
        """load_lut (:91-173).  Arrays in C order = Fortran shape reversed: liquid (nband, nsize_liq),
        ice (nrghice, nband, nsize_ice)."""
        e = self.init(band_lims_wvn, name="RRTMGP cloud optics")
        if e:
            return e
        liq = [np.ascontiguousarray(a, np.float32) for a in (lut_extliq, lut_ssaliq, lut_asyliq)]
        ice = [np.ascontiguousarray(a, np.float32) for a in (lut_extice, lut_ssaice, lut_asyice)]
        nband = self.get_nband()
        if liq[0].ndim != 2 or liq[0].shape[0] != nband:
            return "cloud_optics%init(): number of bands inconsistent between lookup tables, spectral discretization"
        if ice[0].ndim != 3 or ice[0].shape[1] != nband:
            return "cloud_optics%init(): array lut_extice has the wrong number of bands"
        if any(a.shape != liq[0].shape for a in liq[1:]):
            return "cloud_optics%init(): array lut_ssaliq isn't consistently sized"
        if any(a.shape != ice[0].shape for a in ice[1:]):
            return "cloud_optics%init(): array lut_ssaice  isn't consistently sized"
        h = _lib.c_vp()
        F = lambda a: a.ctypes.data_as(_lib.P(_lib.c_float))  # noqa: E731
        check(_lib.lib().rrtmgpnn_cloud_optics_create_lut(
            context(self.device).h, nband, F(np.ascontiguousarray(self.band_lims_wvn)), liq[0].shape[1],
            ice[0].shape[2], ice[0].shape[0], float(radliq_lwr), float(radliq_upr), float(radice_lwr),
            float(radice_upr), *[F(a) for a in liq + ice], h), "cloud_optics_create_lut")
        return self._adopt(h)

    def load_pade(self, band_lims_wvn, pade_extliq, pade_ssaliq, pade_asyliq, pade_extice, pade_ssaice, pade_asyice,
                  pade_sizreg_extliq, pade_sizreg_ssaliq, pade_sizreg_asyliq, pade_sizreg_extice, pade_sizreg_ssaice,
                  pade_sizreg_asyice):
        """load_pade (:179-301).  Coefficients in C order: liquid (ncoef, nsizereg, nband), ice
        (nrghice, ncoef, nsizereg, nband); size-regime bounds (nsizereg + 1)."""
        e = self.init(band_lims_wvn, name="RRTMGP cloud optics")
        if e:
            return e
        c = [np.ascontiguousarray(a, np.float32) for a in (pade_extliq, pade_ssaliq, pade_asyliq, pade_extice,
                                                            pade_ssaice, pade_asyice)]
        b = [np.ascontiguousarray(a, np.float32) for a in (pade_sizreg_extliq, pade_sizreg_ssaliq, pade_sizreg_asyliq,
                                                            pade_sizreg_extice, pade_sizreg_ssaice, pade_sizreg_asyice)]
        if c[0].ndim != 3 or c[3].ndim != 4:
            return "cloud_optics%init(): array pade_extice isn't consistently sized"
        nsizereg = c[0].shape[1]
        if nsizereg != 3:
            return "cloud optics: code assumes exactly three size regimes for Pade approximants but data is otherwise"
        if c[0].shape[2] != self.get_nband():
            return "cloud_optics%init(): number of bands inconsistent between lookup tables, spectral discretization"
        if any(x.shape != (nsizereg + 1,) for x in b):
            return "cloud_optics%init(): one or more Pade size regime arrays are inconsistently sized"
        h = _lib.c_vp()
        F = lambda a: a.ctypes.data_as(_lib.P(_lib.c_float))  # noqa: E731
        check(_lib.lib().rrtmgpnn_cloud_optics_create_pade(
            context(self.device).h, self.get_nband(), F(np.ascontiguousarray(self.band_lims_wvn)), nsizereg,
            c[0].shape[0], c[1].shape[0], c[3].shape[0], *[F(a) for a in c + b], h), "cloud_optics_create_pade")
        return self._adopt(h)

    def set_ice_roughness(self, icergh):
        """set_ice_roughness (:541-554)."""
        if not self.h:
            return "cloud_optics%set_ice_roughness(): can't set before initialization"
        if icergh < 1 or icergh > self.nrghice:
            return "cloud optics: cloud ice surface roughness flag is out of bounds"
        check(_lib.lib().rrtmgpnn_cloud_optics_set_ice_roughness(self.h, int(icergh)), "set_ice_roughness")
        self.icergh = int(icergh)
        return ""

    def get_num_ice_roughness_types(self):
        return self.nrghice if self.h else 0

    def get_min_radius_liq(self):
        return self.radii[0]

    def get_max_radius_liq(self):
        return self.radii[1]

    def get_min_radius_ice(self):
        return self.radii[2]

    def get_max_radius_ice(self):
        return self.radii[3]

    def cloud_optics(self, clwp, ciwp, reliq, reice, optical_props):
        """cloud_optics (:354-535): (ncol, nlay) water paths [g/m2] and effective radii [microns] -> optical
        properties by band; absorption optical depth for 1scl, tau/ssa/g for 2str."""
        if not self.h:
            return "cloud optics: no data has been initialized"
        ncol, nlay = clwp.shape
        for name, a in (("ciwp", ciwp), ("reliq", reliq), ("reice", reice)):
            if tuple(a.shape) != (ncol, nlay):
                return "cloud optics: %s has wrong extents" % name
        if optical_props.get_ncol() != ncol or optical_props.get_nlay() != nlay:
            return "cloud optics: optical_props have wrong extents"
        e = ""
        if not self.bands_are_equal(optical_props):
            e = "cloud optics: optical properties don't have the same band structure"
        if optical_props.get_nband() != optical_props.get_ngpt():
            e = "cloud optics: optical properties must be requested by band not g-points"
        if e:
            return e
        dev = optical_props.tau.device
        lwp, iwp, rl, ri = (_f32dev(a, dev) for a in (clwp, ciwp, reliq, reice))
        if check_values:  # :436-444
            liq, ice = lwp > 0, iwp > 0
            if bool(((rl < self.radii[0]) | (rl > self.radii[1]))[liq].any()):
                e = "cloud optics: liquid effective radius is out of bounds"
            if bool(((ri < self.radii[2]) | (ri > self.radii[3]))[ice].any()):
                e = "cloud optics: ice effective radius is out of bounds"
            if e:
                return e
        is2 = isinstance(optical_props, OpticalProps2str)
        check(_lib.lib().rrtmgpnn_cloud_optics_compute(
            context(dev.index).h, self.h, ncol, nlay, _p(lwp), _p(iwp), _p(rl), _p(ri), _p(optical_props.tau),
            _p(optical_props.ssa) if is2 else None, _p(optical_props.g) if is2 else None), "cloud_optics")
        return ""

    def __del__(self):
        try:
            if self.h:
                _lib.lib().rrtmgpnn_cloud_optics_destroy(self.h)
        except Exception:
            pass


# ---------------------------------------------------------------------------------------------
GAUSS_DS = {1: [1.66], 2: [1.18350343, 2.81649655], 3: [1.09719858, 1.69338507, 4.70941630],
            4: [1.06056257, 1.38282560, 2.40148179, 7.15513024]}
GAUSS_WTS = {1: [0.5], 2: [0.3180413817, 0.1819586183], 3: [0.2009319137, 0.2292411064, 0.0698269799],
             4: [0.1355069134, 0.2034645680, 0.1298475476, 0.0311809710]}


def rte_lw(optical_props, top_at_1, sources, sfc_emis, fluxes, inc_flux=None, n_gauss_angles=None,
           use_2stream=False, lw_Ds=None, flux_up_Jac=None, flux_dn_Jac=None):
    """rte/mo_rte_lw.F90:60-424.  sfc_emis (ncol, nband)."""
    if not fluxes.are_desired():
        return "rte_lw: no space allocated for fluxes"
    nmu = 1 if n_gauss_angles is None else int(n_gauss_angles)
    if nmu > 4:
        return "rte_lw: asking for too many quadrature points for no-scattering calculation"
    if nmu < 1:
        return "rte_lw: have to ask for at least one quadrature point for no-scattering calculation"
    is2 = isinstance(optical_props, OpticalProps2str)
    if not is2 and not isinstance(optical_props, OpticalProps1scl):
        return "lw_solver(...ty_optical_props_nstr...) not yet implemented"
    if not is2 and use_2stream:
        return "rte_lw: can't use two-stream methods with only absorption optical depth"
    if is2:
        # The reference's 2str checks (:248-253) each overwrite error_msg, so the last failing one is returned.  The
        # Jacobian check tests flux_up_Jac twice (`present(flux_up_Jac) .or. present(flux_up_Jac)`), so a lone
        # flux_dn_Jac passes, as there.
        e = ""
        if lw_Ds is not None:
            e = "rte_lw: lw_Ds not valid input for _2str class"
        if use_2stream and nmu != 1:
            e = "rte_lw: using_2stream=true incompatible with specifying n_gauss_angles"
        if use_2stream and flux_up_Jac is not None:
            e = "rte_lw: can't provide Jacobian of fluxes w.r.t surface temperature with 2-stream"
        if e:
            return e
    # flux_up_Jac / flux_dn_Jac are otherwise accepted and left untouched: compute_Jac is a .false. parameter
    # (rte/mo_rte_rrtmgp_config.F90:28), so the reference neither checks their extents (:160-163) nor writes them.
    ncol, nlay, ngpt = optical_props.tau.shape
    if lw_Ds is not None:  # (:239-246); Fortran extents (ncol, ngpt) = this tensor layout's (ngpt, ncol)
        if tuple(lw_Ds.shape) != (ngpt, ncol):
            return "rte_lw: lw_Ds inconsistently sized"
        if bool((torch.as_tensor(lw_Ds) < 1.0).any()):
            return "rte_lw: one or more values of lw_Ds < 1."
        if nmu != 1:
            return "rte_lw: providing lw_Ds incompatible with specifying n_gauss_angles"
    gpt = fluxes.are_desired_gpt()
    if gpt:
        for a in (fluxes.gpt_flux_up, fluxes.gpt_flux_dn):
            if a is not None and tuple(a.shape) != (ncol, nlay + 1, ngpt):
                return "rte_lw: g-point flux arrays inconsistently sized"
    nband = optical_props.get_nband()
    if tuple(sfc_emis.shape) != (ncol, nband):
        return "rte_lw: sfc_emis inconsistently sized"
    if inc_flux is not None and tuple(inc_flux.shape) != (ncol, ngpt):
        return "rte_lw: inc_flux inconsistently sized"
    ctx = context(optical_props.tau.device.index)
    L = _lib.lib()
    emis = _f32dev(sfc_emis, optical_props.tau.device)
    emis_gpt = torch.empty((ncol, ngpt), dtype=torch.float32, device=emis.device)
    check(L.rrtmgpnn_expand_band_to_gpt(ctx.h, nband, ngpt, ncol, int_array(optical_props.band_lims_gpt.ravel()),
                                        _p(emis), _p(emis_gpt)), "expand")
    up = fluxes.flux_up if fluxes.flux_up is not None else torch.empty((ncol, nlay + 1), device=emis.device)
    dn = fluxes.flux_dn if fluxes.flux_dn is not None else torch.empty((ncol, nlay + 1), device=emis.device)
    op = optical_props
    # ty_fluxes_flexible g-point outputs (:275-288): the caller's arrays, scratch for the one not asked for
    gu = gd = None
    if gpt:
        gu = fluxes.gpt_flux_up if fluxes.gpt_flux_up is not None else \
            torch.empty((ncol, nlay + 1, ngpt), device=emis.device)
        gd = fluxes.gpt_flux_dn if fluxes.gpt_flux_dn is not None else \
            torch.empty((ncol, nlay + 1, ngpt), device=emis.device)
    if is2 and use_2stream:  # lw_solver_2stream (rte/mo_rte_lw.F90:357-371); validate() runs unconditionally
        e = op.validate()
        if e:
            return e
        common = (ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), _p(inc_flux), _p(op.tau), _p(op.ssa), _p(op.g),
                  _p(sources.lev_source), _p(emis_gpt), _p(sources.sfc_source), _p(up), _p(dn))
        if gpt:
            check(L.rrtmgpnn_lw_solver_2stream_gpt(*common, _p(gu), _p(gd)), "lw_solver_2stream_gpt")
        else:
            check(L.rrtmgpnn_lw_solver_2stream(*common), "lw_solver_2stream")
    elif is2:  # rescaled no-scattering solution (:372-387)
        if check_values:
            e = op.validate()
            if e:
                return e
        common = (ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), nmu, float_array(GAUSS_DS[nmu]),
                  float_array(GAUSS_WTS[nmu]), _p(inc_flux), _p(op.tau), _p(op.ssa), _p(op.g), _p(sources.lay_source),
                  _p(sources.lev_source), _p(emis_gpt), _p(sources.sfc_source), _p(up), _p(dn))
        if gpt:
            check(L.rrtmgpnn_lw_solver_1rescl_gpt(*common, _p(gu), _p(gd)), "lw_solver_1rescl_gpt")
        else:
            check(L.rrtmgpnn_lw_solver_1rescl(*common), "lw_solver_1rescl")
    elif gpt or lw_Ds is not None:  # ty_fluxes_flexible g-point outputs / column-dependent secants (:329-341)
        ds = _f32dev(lw_Ds, emis.device) if lw_Ds is not None else None
        check(L.rrtmgpnn_lw_solver_noscat_gpt(ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), nmu,
                                              float_array(GAUSS_DS[nmu]), float_array(GAUSS_WTS[nmu]), _p(ds),
                                              _p(inc_flux), _p(op.tau), _p(sources.lay_source),
                                              _p(sources.lev_source), _p(emis_gpt), _p(sources.sfc_source), _p(up),
                                              _p(dn), _p(gu), _p(gd)), "lw_solver_noscat_gpt")
    else:
        check(L.rrtmgpnn_lw_solver_noscat(ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), nmu,
                                          float_array(GAUSS_DS[nmu]), float_array(GAUSS_WTS[nmu]), _p(inc_flux),
                                          _p(op.tau), _p(sources.lay_source), _p(sources.lev_source),
                                          _p(emis_gpt), _p(sources.sfc_source), _p(up), _p(dn)), "lw_solver_noscat")
    if fluxes.flux_net is not None:
        torch.sub(dn, up, out=fluxes.flux_net)
    return ""


def rte_sw(atmos, top_at_1, mu0, inc_flux, sfc_alb_dir_gpt, sfc_alb_dif_gpt, fluxes, inc_flux_dif=None):
    """rte/mo_rte_sw.F90:48-266 (fork: albedos per g-point (ncol, ngpt)).  1scl: the direct beam (sw_solver_noscat);
    2str: sw_solver_2stream."""
    if not fluxes.are_desired():
        return "rte_sw: no space allocated for fluxes"
    if not isinstance(atmos, (OpticalProps1scl, OpticalProps2str)):
        return "sw_solver(...ty_optical_props_nstr...) not yet implemented"
    ncol, nlay, ngpt = atmos.tau.shape
    if tuple(mu0.shape) != (ncol,):
        return "rte_sw: mu0 inconsistently sized"
    if tuple(inc_flux.shape) != (ncol, ngpt):
        return "rte_sw: inc_flux inconsistently sized"
    if tuple(sfc_alb_dir_gpt.shape) != (ncol, ngpt):
        return "rte_sw: sfc_alb_dir inconsistently sized"
    if tuple(sfc_alb_dif_gpt.shape) != (ncol, ngpt):
        return "rte_sw: sfc_alb_dif inconsistently sized"
    if inc_flux_dif is not None and tuple(inc_flux_dif.shape) != (ncol, ngpt):
        return "rte_sw: inc_flux_dif inconsistently sized"
    ctx = context(atmos.tau.device.index)
    dev = atmos.tau.device
    if isinstance(atmos, OpticalProps1scl):
        # direct beam only (:213-222): apply_BC_factor + sw_solver_noscat; as in the reference only the direct flux
        # is written (flux_up / flux_dn / flux_net are left as they are)
        if fluxes.flux_dn_dir is None:
            return "rte_sw: the no-scattering solution needs flux_dn_dir"
        gdir = getattr(fluxes, "gpt_flux_dn_dir", None)
        if gdir is not None:  # the spectral beam into the caller's gpt_flux_dn_dir (:155-163, 218-222)
            if tuple(gdir.shape) != (ncol, nlay + 1, ngpt):
                return "rte_sw: g-point flux arrays inconsistently sized"
            check(_lib.lib().rrtmgpnn_sw_solver_noscat_gpt(ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), _p(inc_flux),
                                                           _p(atmos.tau), _p(mu0), _p(fluxes.flux_dn_dir), _p(gdir)),
                  "sw_solver_noscat_gpt")
        else:
            check(_lib.lib().rrtmgpnn_sw_solver_noscat(ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), _p(inc_flux),
                                                       _p(atmos.tau), _p(mu0), _p(fluxes.flux_dn_dir)),
                  "sw_solver_noscat")
        return ""
    up = fluxes.flux_up if fluxes.flux_up is not None else torch.empty((ncol, nlay + 1), device=dev)
    dn = fluxes.flux_dn if fluxes.flux_dn is not None else torch.empty((ncol, nlay + 1), device=dev)
    dr = fluxes.flux_dn_dir if fluxes.flux_dn_dir is not None else torch.empty((ncol, nlay + 1), device=dev)
    if fluxes.are_desired_gpt():  # save_gpt_flux (rte/mo_rte_sw.F90:155-173, 228-234): up, total down, direct
        g3 = []
        for a in (fluxes.gpt_flux_up, fluxes.gpt_flux_dn, fluxes.gpt_flux_dn_dir):
            if a is not None and tuple(a.shape) != (ncol, nlay + 1, ngpt):
                return "rte_sw: g-point flux arrays inconsistently sized"
            g3.append(a if a is not None else torch.empty((ncol, nlay + 1, ngpt), device=dev))
        check(_lib.lib().rrtmgpnn_sw_solver_2stream_gpt(ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), _p(inc_flux),
                                                        _p(inc_flux_dif), _p(atmos.tau), _p(atmos.ssa), _p(atmos.g),
                                                        _p(mu0), _p(sfc_alb_dir_gpt), _p(sfc_alb_dif_gpt), _p(up),
                                                        _p(dn), _p(dr), *[_p(a) for a in g3]), "sw_solver_2stream_gpt")
    else:
        check(_lib.lib().rrtmgpnn_sw_solver_2stream(ctx.h, ngpt, nlay, ncol, int(bool(top_at_1)), _p(inc_flux),
                                                    _p(inc_flux_dif), _p(atmos.tau), _p(atmos.ssa), _p(atmos.g),
                                                    _p(mu0), _p(sfc_alb_dir_gpt), _p(sfc_alb_dif_gpt), _p(up),
                                                    _p(dn), _p(dr)), "sw_solver_2stream")
    if fluxes.flux_net is not None:
        torch.sub(dn, up, out=fluxes.flux_net)
    return ""


def _heating_rate(fn, name, flux_up, flux_dn, plev, heating_rate):
    ncol, nlev = flux_up.shape
    nlay = nlev - 1
    if tuple(flux_dn.shape) != (ncol, nlev):
        return name + ": flux_dn array inconsistently sized."
    if tuple(plev.shape) != (ncol, nlev):
        return name + ": plev array inconsistently sized."
    if tuple(heating_rate.shape) != (ncol, nlay):
        return name + ": heating_rate array inconsistently sized."
    ctx = context(flux_up.device.index)
    check(fn(ctx.h, ncol, nlay, _p(flux_up), _p(flux_dn), _p(plev), _p(heating_rate)), name)
    return ""


def compute_heating_rate(flux_up, flux_dn, plev, heating_rate):
    """compute_heating_rate (extensions/mo_heating_rates.F90:26-53), K/s, grav / cp_dry from mo_rrtmgp_constants.
    Arrays in this fork's layout: fluxes and plev (ncol, nlay+1), heating_rate (ncol, nlay) device tensors."""
    return _heating_rate(_lib.lib().rrtmgpnn_compute_heating_rate, "heating_rate", flux_up, flux_dn, plev,
                         heating_rate)


def calc_heating_rate(flux_up, flux_dn, plev, hr_k_day):
    """calc_heating_rate (examples/rrtmgp-nn-training/rrtmgp_lw_eval_nn_rfmip.F90:624-653), K/day with cp = 1004,
    as the NN evaluation programs report it.  Same layouts as compute_heating_rate."""
    return _heating_rate(_lib.lib().rrtmgpnn_calc_heating_rate_k_day, "calc_heating_rate", flux_up, flux_dn, plev,
                         hr_k_day)
