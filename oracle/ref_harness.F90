! ref_harness.F90 -- TEST INFRASTRUCTURE ONLY (never shipped, never linked by the product).
!
! bind(C) entry points around the REFERENCE's own compiled Fortran, so the tests can
! pin the C restatement (oracle/rrtmgpnn_oracle.c) against the reference itself.
! Built by oracle/Makefile.ref from the sources where they lie under /root/reference;
! output goes to oracle/_ref/ only.  Exposes:
!   ref_rte_lw   -> rte_lw (rte/mo_rte_lw.F90:60) on ty_optical_props_1scl + ty_source_func_lw
!   ref_rte_sw   -> rte_sw (rte/mo_rte_sw.F90:48) on ty_optical_props_2str
!   ref_sw_noscat -> the kernels of rte_sw's 1scl branch (rte/mo_rte_sw.F90:213-222): apply_BC (the generic resolves
!                    to apply_BC_factor, rte/kernels/mo_rte_solver_kernels.F90:1685-1704) and sw_solver_noscat
!                    (:496-532), called with the kernels' own argument meaning (rte_sw swaps the spectral and the
!                    broadband direct-flux arrays at :220-222, quirk B-10, so rte_sw itself is not called)
!   ref_mlp      -> network_type%output_sgemm_flat (neural/mod_network.F90:273) with MKL sgemm
!   ref_cloud_optics -> ty_cloud_optics%load (LUT or Pade) + set_ice_roughness + cloud_optics
!                       (extensions/cloud_optics/mo_cloud_optics.F90) into 1scl or 2str by band
!   ref_increment_bybnd / ref_delta_scale -> ty_optical_props_arry%increment, %delta_scale
!                       (rte/mo_optical_props.F90:882-1023, :576-604)
! The NN modules that need netcdf (mod_network_rrtmgp, mo_gas_optics_rrtmgp,
! mo_gas_optics_kernels) are not built: netcdf-fortran is absent and we do not stub it.
module ref_harness
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,         only: wp, wl
  use mo_rte_solver_kernels, only: apply_BC, sw_solver_noscat
  use mo_optical_props,    only: ty_optical_props_1scl, ty_optical_props_2str
  use mo_source_functions, only: ty_source_func_lw
  use mo_fluxes,           only: ty_fluxes_flexible
  use mo_rte_lw,           only: rte_lw
  use mo_rte_sw,           only: rte_sw
  use mod_network,         only: network_type
  use mo_cloud_optics,     only: ty_cloud_optics
  implicit none
  character(len=128), save :: last_msg = ''
contains

  integer(c_int) function ref_rte_lw(ncol, nlay, nband, ngpt, band_lims_gpt, band_lims_wvn, top_at_1, nmus, &
                                     tau, lay_src, lev_src, sfc_src, sfc_src_jac, sfc_emis, &
                                     flux_up, flux_dn) bind(C, name="ref_rte_lw")
    integer(c_int), value :: ncol, nlay, nband, ngpt, top_at_1, nmus
    integer(c_int), intent(in) :: band_lims_gpt(2, nband)
    real(c_float),  intent(in) :: band_lims_wvn(2, nband)
    real(c_float),  intent(in) :: tau(ngpt, nlay, ncol), lay_src(ngpt, nlay, ncol), lev_src(ngpt, nlay+1, ncol)
    real(c_float),  intent(in) :: sfc_src(ngpt, ncol), sfc_src_jac(ngpt, ncol), sfc_emis(nband, ncol)
    real(c_float),  intent(out), target :: flux_up(nlay+1, ncol), flux_dn(nlay+1, ncol)

    type(ty_optical_props_1scl) :: op
    type(ty_source_func_lw)     :: src
    type(ty_fluxes_flexible)    :: fl
    real(wp), allocatable, target :: gup(:,:,:), gdn(:,:,:)
    character(len=128) :: err

    ref_rte_lw = 1
    err = op%alloc_1scl(ncol, nlay, band_lims_wvn, band_lims_gpt)
    if (err /= '') then; last_msg = err; return; end if
    err = src%alloc(ncol, nlay, op)
    if (err /= '') then; last_msg = err; return; end if
    op%tau = tau
    src%lay_source = lay_src
    src%lev_source = lev_src
    src%sfc_source = sfc_src
    src%sfc_source_Jac = sfc_src_jac
    fl%flux_up => flux_up
    fl%flux_dn => flux_dn
    if (nmus > 1) then
      ! n_gauss_angles > 1 needs g-point flux storage (lw_solver_noscat_GaussQuad :383-412)
      allocate(gup(ngpt, nlay+1, ncol), gdn(ngpt, nlay+1, ncol))
      fl%gpt_flux_up => gup
      fl%gpt_flux_dn => gdn
    end if
    err = rte_lw(op, top_at_1 /= 0, src, sfc_emis, fl, n_gauss_angles=int(nmus), use_2stream=.false.)
    if (err /= '') then; last_msg = err; return; end if
    ref_rte_lw = 0
  end function ref_rte_lw

  ! rte_lw on two-stream optical properties: the rescaled no-scattering solution (use_2stream = 0,
  ! rte/mo_rte_lw.F90:372-387) or lw_solver_2stream (use_2stream = 1, :357-371).
  integer(c_int) function ref_rte_lw_2str(ncol, nlay, nband, ngpt, band_lims_gpt, band_lims_wvn, top_at_1, nmus, &
                                          use_2stream, tau, ssa, g, lay_src, lev_src, sfc_src, sfc_src_jac, &
                                          sfc_emis, flux_up, flux_dn) bind(C, name="ref_rte_lw_2str")
    integer(c_int), value :: ncol, nlay, nband, ngpt, top_at_1, nmus, use_2stream
    integer(c_int), intent(in) :: band_lims_gpt(2, nband)
    real(c_float),  intent(in) :: band_lims_wvn(2, nband)
    real(c_float),  intent(in) :: tau(ngpt, nlay, ncol), ssa(ngpt, nlay, ncol), g(ngpt, nlay, ncol)
    real(c_float),  intent(in) :: lay_src(ngpt, nlay, ncol), lev_src(ngpt, nlay+1, ncol)
    real(c_float),  intent(in) :: sfc_src(ngpt, ncol), sfc_src_jac(ngpt, ncol), sfc_emis(nband, ncol)
    real(c_float),  intent(out), target :: flux_up(nlay+1, ncol), flux_dn(nlay+1, ncol)

    type(ty_optical_props_2str) :: op
    type(ty_source_func_lw)     :: src
    type(ty_fluxes_flexible)    :: fl
    real(wp), allocatable, target :: gup(:,:,:), gdn(:,:,:)
    character(len=128) :: err

    ref_rte_lw_2str = 1
    err = op%alloc_2str(ncol, nlay, band_lims_wvn, band_lims_gpt)
    if (err /= '') then; last_msg = err; return; end if
    err = src%alloc(ncol, nlay, op)
    if (err /= '') then; last_msg = err; return; end if
    op%tau = tau
    op%ssa = ssa
    op%g = g
    src%lay_source = lay_src
    src%lev_source = lev_src
    src%sfc_source = sfc_src
    src%sfc_source_Jac = sfc_src_jac
    fl%flux_up => flux_up
    fl%flux_dn => flux_dn
    if (nmus > 1 .or. use_2stream /= 0) then
      ! GaussQuad with several angles and lw_solver_2stream write g-point fluxes
      allocate(gup(ngpt, nlay+1, ncol), gdn(ngpt, nlay+1, ncol))
      fl%gpt_flux_up => gup
      fl%gpt_flux_dn => gdn
    end if
    err = rte_lw(op, top_at_1 /= 0, src, sfc_emis, fl, n_gauss_angles=int(nmus), use_2stream=use_2stream /= 0)
    if (err /= '') then; last_msg = err; return; end if
    ref_rte_lw_2str = 0
  end function ref_rte_lw_2str

  ! ref_rte_lw_2str with the caller's g-point outputs associated (ty_fluxes_flexible gpt_flux_up/dn): the rescaled
  ! solution's radiances (one angle) or angle-summed fluxes, or lw_solver_2stream's adding fluxes.
  integer(c_int) function ref_rte_lw_2str_gpt(ncol, nlay, nband, ngpt, band_lims_gpt, band_lims_wvn, top_at_1, nmus, &
                                              use_2stream, tau, ssa, g, lay_src, lev_src, sfc_src, sfc_src_jac, &
                                              sfc_emis, flux_up, flux_dn, gpt_up, gpt_dn) bind(C, name="ref_rte_lw_2str_gpt")
    integer(c_int), value :: ncol, nlay, nband, ngpt, top_at_1, nmus, use_2stream
    integer(c_int), intent(in) :: band_lims_gpt(2, nband)
    real(c_float),  intent(in) :: band_lims_wvn(2, nband)
    real(c_float),  intent(in) :: tau(ngpt, nlay, ncol), ssa(ngpt, nlay, ncol), g(ngpt, nlay, ncol)
    real(c_float),  intent(in) :: lay_src(ngpt, nlay, ncol), lev_src(ngpt, nlay+1, ncol)
    real(c_float),  intent(in) :: sfc_src(ngpt, ncol), sfc_src_jac(ngpt, ncol), sfc_emis(nband, ncol)
    real(c_float),  intent(out), target :: flux_up(nlay+1, ncol), flux_dn(nlay+1, ncol)
    real(c_float),  intent(out), target :: gpt_up(ngpt, nlay+1, ncol), gpt_dn(ngpt, nlay+1, ncol)

    type(ty_optical_props_2str) :: op
    type(ty_source_func_lw)     :: src
    type(ty_fluxes_flexible)    :: fl
    character(len=128) :: err

    ref_rte_lw_2str_gpt = 1
    err = op%alloc_2str(ncol, nlay, band_lims_wvn, band_lims_gpt)
    if (err /= '') then; last_msg = err; return; end if
    err = src%alloc(ncol, nlay, op)
    if (err /= '') then; last_msg = err; return; end if
    op%tau = tau
    op%ssa = ssa
    op%g = g
    src%lay_source = lay_src
    src%lev_source = lev_src
    src%sfc_source = sfc_src
    src%sfc_source_Jac = sfc_src_jac
    fl%flux_up => flux_up
    fl%flux_dn => flux_dn
    fl%gpt_flux_up => gpt_up
    fl%gpt_flux_dn => gpt_dn
    err = rte_lw(op, top_at_1 /= 0, src, sfc_emis, fl, n_gauss_angles=int(nmus), use_2stream=use_2stream /= 0)
    if (err /= '') then; last_msg = err; return; end if
    ref_rte_lw_2str_gpt = 0
  end function ref_rte_lw_2str_gpt

  integer(c_int) function ref_rte_sw(ncol, nlay, nband, ngpt, band_lims_gpt, band_lims_wvn, top_at_1, &
                                     tau, ssa, g, mu0, inc_flux, sfc_alb_dir, sfc_alb_dif, &
                                     flux_up, flux_dn, flux_dir) bind(C, name="ref_rte_sw")
    integer(c_int), value :: ncol, nlay, nband, ngpt, top_at_1
    integer(c_int), intent(in) :: band_lims_gpt(2, nband)
    real(c_float),  intent(in) :: band_lims_wvn(2, nband)
    real(c_float),  intent(in) :: tau(ngpt, nlay, ncol), ssa(ngpt, nlay, ncol), g(ngpt, nlay, ncol)
    real(c_float),  intent(in) :: mu0(ncol), inc_flux(ngpt, ncol), sfc_alb_dir(ngpt, ncol), sfc_alb_dif(ngpt, ncol)
    real(c_float),  intent(out), target :: flux_up(nlay+1, ncol), flux_dn(nlay+1, ncol), flux_dir(nlay+1, ncol)

    type(ty_optical_props_2str) :: op
    type(ty_fluxes_flexible)    :: fl
    character(len=128) :: err

    ref_rte_sw = 1
    err = op%alloc_2str(ncol, nlay, band_lims_wvn, band_lims_gpt)
    if (err /= '') then; last_msg = err; return; end if
    op%tau = tau
    op%ssa = ssa
    op%g   = g
    fl%flux_up     => flux_up
    fl%flux_dn     => flux_dn
    fl%flux_dn_dir => flux_dir
    err = rte_sw(op, top_at_1 /= 0, mu0, inc_flux, sfc_alb_dir, sfc_alb_dif, fl)
    if (err /= '') then; last_msg = err; return; end if
    ref_rte_sw = 0
  end function ref_rte_sw

  ! rte_lw on 1scl properties with g-point outputs (ty_fluxes_flexible gpt_flux_up/dn associated) and, when use_ds /= 0,
  ! the column-dependent secants lw_Ds (rte/mo_rte_lw.F90:239-246, 329-341): the extents rte_lw checks, (ncol, ngpt).
  integer(c_int) function ref_rte_lw_gpt(ncol, nlay, nband, ngpt, band_lims_gpt, band_lims_wvn, top_at_1, nmus, &
                                         use_ds, lw_ds, tau, lay_src, lev_src, sfc_src, sfc_src_jac, sfc_emis, &
                                         flux_up, flux_dn, gpt_up, gpt_dn) bind(C, name="ref_rte_lw_gpt")
    integer(c_int), value :: ncol, nlay, nband, ngpt, top_at_1, nmus, use_ds
    integer(c_int), intent(in) :: band_lims_gpt(2, nband)
    real(c_float),  intent(in) :: band_lims_wvn(2, nband), lw_ds(ncol, ngpt)
    real(c_float),  intent(in) :: tau(ngpt, nlay, ncol), lay_src(ngpt, nlay, ncol), lev_src(ngpt, nlay+1, ncol)
    real(c_float),  intent(in) :: sfc_src(ngpt, ncol), sfc_src_jac(ngpt, ncol), sfc_emis(nband, ncol)
    real(c_float),  intent(out), target :: flux_up(nlay+1, ncol), flux_dn(nlay+1, ncol)
    real(c_float),  intent(out), target :: gpt_up(ngpt, nlay+1, ncol), gpt_dn(ngpt, nlay+1, ncol)

    type(ty_optical_props_1scl) :: op
    type(ty_source_func_lw)     :: src
    type(ty_fluxes_flexible)    :: fl
    character(len=128) :: err

    ref_rte_lw_gpt = 1
    err = op%alloc_1scl(ncol, nlay, band_lims_wvn, band_lims_gpt)
    if (err /= '') then; last_msg = err; return; end if
    err = src%alloc(ncol, nlay, op)
    if (err /= '') then; last_msg = err; return; end if
    op%tau = tau
    src%lay_source = lay_src
    src%lev_source = lev_src
    src%sfc_source = sfc_src
    src%sfc_source_Jac = sfc_src_jac
    fl%flux_up => flux_up
    fl%flux_dn => flux_dn
    fl%gpt_flux_up => gpt_up
    fl%gpt_flux_dn => gpt_dn
    if (use_ds /= 0) then
      err = rte_lw(op, top_at_1 /= 0, src, sfc_emis, fl, lw_Ds=lw_ds)
    else
      err = rte_lw(op, top_at_1 /= 0, src, sfc_emis, fl, n_gauss_angles=int(nmus), use_2stream=.false.)
    end if
    if (err /= '') then; last_msg = err; return; end if
    ref_rte_lw_gpt = 0
  end function ref_rte_lw_gpt

  ! rte_sw on 2str properties with g-point outputs (save_gpt_flux, rte/mo_rte_sw.F90:155-173, 228-234)
  integer(c_int) function ref_rte_sw_gpt(ncol, nlay, nband, ngpt, band_lims_gpt, band_lims_wvn, top_at_1, &
                                         tau, ssa, g, mu0, inc_flux, sfc_alb_dir, sfc_alb_dif, &
                                         flux_up, flux_dn, flux_dir, gpt_up, gpt_dn, gpt_dir) bind(C, name="ref_rte_sw_gpt")
    integer(c_int), value :: ncol, nlay, nband, ngpt, top_at_1
    integer(c_int), intent(in) :: band_lims_gpt(2, nband)
    real(c_float),  intent(in) :: band_lims_wvn(2, nband)
    real(c_float),  intent(in) :: tau(ngpt, nlay, ncol), ssa(ngpt, nlay, ncol), g(ngpt, nlay, ncol)
    real(c_float),  intent(in) :: mu0(ncol), inc_flux(ngpt, ncol), sfc_alb_dir(ngpt, ncol), sfc_alb_dif(ngpt, ncol)
    real(c_float),  intent(out), target :: flux_up(nlay+1, ncol), flux_dn(nlay+1, ncol), flux_dir(nlay+1, ncol)
    real(c_float),  intent(out), target :: gpt_up(ngpt, nlay+1, ncol), gpt_dn(ngpt, nlay+1, ncol), &
                                           gpt_dir(ngpt, nlay+1, ncol)

    type(ty_optical_props_2str) :: op
    type(ty_fluxes_flexible)    :: fl
    character(len=128) :: err

    ref_rte_sw_gpt = 1
    err = op%alloc_2str(ncol, nlay, band_lims_wvn, band_lims_gpt)
    if (err /= '') then; last_msg = err; return; end if
    op%tau = tau
    op%ssa = ssa
    op%g   = g
    fl%flux_up         => flux_up
    fl%flux_dn         => flux_dn
    fl%flux_dn_dir     => flux_dir
    fl%gpt_flux_up     => gpt_up
    fl%gpt_flux_dn     => gpt_dn
    fl%gpt_flux_dn_dir => gpt_dir
    err = rte_sw(op, top_at_1 /= 0, mu0, inc_flux, sfc_alb_dir, sfc_alb_dif, fl)
    if (err /= '') then; last_msg = err; return; end if
    ref_rte_sw_gpt = 0
  end function ref_rte_sw_gpt

  ! MLP chain of the reference: h = act(W^T x + b) via MKL sgemm (neural/mod_network.F90:273-354).
  ! w_all: concatenation of each layer's weights stored (n_in, n_out) C-order = w_transposed(n_out,n_in).
  integer(c_int) function ref_mlp(nlayers, dims, acts, w_all, b_all, nbatch, x, out) bind(C, name="ref_mlp")
    integer(c_int), value :: nlayers, nbatch
    integer(c_int), intent(in) :: dims(nlayers+1), acts(nlayers)
    real(c_float),  intent(in) :: w_all(*), b_all(*)
    real(c_float),  intent(in) :: x(dims(1), nbatch)
    real(c_float),  intent(out) :: out(dims(nlayers+1), nbatch)
    type(network_type) :: net
    integer :: n, ow, ob, nin, nout, j0, nb
    integer, parameter :: chunk = 1024   ! output_sgemm_flat keeps (neurons, nbatch) automatic arrays on the stack
    character(len=16), dimension(0:6) :: names = [character(len=16) :: 'linear', 'softsign', 'relu', 'sigmoid', &
                                                  'hard_sigmoid', 'tanh', 'gaussian']

    call net%init(dims)
    ow = 0; ob = 0
    do n = 1, nlayers
      nin = dims(n); nout = dims(n+1)
      net%layers(n)%w_transposed = reshape(w_all(ow+1:ow+nin*nout), [nout, nin])
      net%layers(n)%w = transpose(net%layers(n)%w_transposed)
      net%layers(n)%b = b_all(ob+1:ob+nout)
      call net%layers(n)%set_activation(trim(names(acts(n))))
      ow = ow + nin*nout; ob = ob + nout
    end do
    do j0 = 1, nbatch, chunk
      nb = min(chunk, nbatch - j0 + 1)
      call net%output_sgemm_flat(dims(1), dims(nlayers+1), nb, x(:, j0:j0+nb-1), out(:, j0:j0+nb-1))
    end do
    ref_mlp = 0
  end function ref_mlp

  integer(c_int) function ref_sw_noscat(ncol, nlay, ngpt, top_at_1, inc_flux, tau, mu0, flux_dir, gpt_flux_dir) &
      bind(C, name="ref_sw_noscat")
    integer(c_int), value :: ncol, nlay, ngpt, top_at_1
    real(c_float),  intent(in) :: inc_flux(ngpt, ncol), tau(ngpt, nlay, ncol), mu0(ncol)
    real(c_float),  intent(out) :: flux_dir(nlay+1, ncol), gpt_flux_dir(ngpt, nlay+1, ncol)
    call apply_BC(ngpt, nlay, ncol, logical(top_at_1 /= 0, wl), inc_flux, mu0, gpt_flux_dir)
    call sw_solver_noscat(ngpt, nlay, ncol, logical(top_at_1 /= 0, wl), tau, mu0, gpt_flux_dir, flux_dir)
    ref_sw_noscat = 0
  end function ref_sw_noscat

  subroutine ref_last_error(buf, n) bind(C, name="ref_last_error")
    integer(c_int), value :: n
    character(kind=c_char), intent(out) :: buf(n)
    integer :: i
    do i = 1, n
      buf(i) = c_null_char
    end do
    do i = 1, min(n-1, len_trim(last_msg))
      buf(i) = last_msg(i:i)
    end do
  end subroutine ref_last_error
  ! cloud_optics: LUT (lut != 0) or Pade coefficient arrays in the file's (Fortran) layout.
  ! nstr = 1 -> ty_optical_props_1scl (absorption tau), 2 -> 2str (tau, ssa, g); outputs (nband, nlay, ncol).
  integer(c_int) function ref_cloud_optics(lut, nband, band_lims_wvn, nsize_liq, nsize_ice, nrgh, &
      radliq_lwr, radliq_upr, radice_lwr, radice_upr, extliq, ssaliq, asyliq, extice, ssaice, asyice, &
      nsizereg, ncoef_ext, ncoef_ssa, p_extliq, p_ssaliq, p_asyliq, p_extice, p_ssaice, p_asyice, &
      sr_extliq, sr_ssaliq, sr_asyliq, sr_extice, sr_ssaice, sr_asyice, icergh, &
      ncol, nlay, clwp, ciwp, reliq, reice, nstr, tau, ssa, g) bind(C, name="ref_cloud_optics")
    integer(c_int), value :: lut, nband, nsize_liq, nsize_ice, nrgh, nsizereg, ncoef_ext, ncoef_ssa, icergh
    integer(c_int), value :: ncol, nlay, nstr
    real(c_float),  value :: radliq_lwr, radliq_upr, radice_lwr, radice_upr
    real(c_float),  intent(in) :: band_lims_wvn(2, nband)
    real(c_float),  intent(in) :: extliq(nsize_liq, nband), ssaliq(nsize_liq, nband), asyliq(nsize_liq, nband)
    real(c_float),  intent(in) :: extice(nsize_ice, nband, nrgh), ssaice(nsize_ice, nband, nrgh), &
                                  asyice(nsize_ice, nband, nrgh)
    real(c_float),  intent(in) :: p_extliq(nband, nsizereg, ncoef_ext), p_ssaliq(nband, nsizereg, ncoef_ssa), &
                                  p_asyliq(nband, nsizereg, ncoef_ssa)
    real(c_float),  intent(in) :: p_extice(nband, nsizereg, ncoef_ext, nrgh), p_ssaice(nband, nsizereg, ncoef_ssa, nrgh), &
                                  p_asyice(nband, nsizereg, ncoef_ssa, nrgh)
    real(c_float),  intent(in) :: sr_extliq(nsizereg+1), sr_ssaliq(nsizereg+1), sr_asyliq(nsizereg+1), &
                                  sr_extice(nsizereg+1), sr_ssaice(nsizereg+1), sr_asyice(nsizereg+1)
    real(c_float),  intent(in) :: clwp(nlay, ncol), ciwp(nlay, ncol), reliq(nlay, ncol), reice(nlay, ncol)
    real(c_float),  intent(out) :: tau(nband, nlay, ncol), ssa(nband, nlay, ncol), g(nband, nlay, ncol)

    type(ty_cloud_optics) :: co
    type(ty_optical_props_1scl) :: o1
    type(ty_optical_props_2str) :: o2
    character(len=128) :: err

    ref_cloud_optics = 1
    if (lut /= 0) then
      err = co%load(band_lims_wvn, radliq_lwr, radliq_upr, 0._wp, radice_lwr, radice_upr, 0._wp, &
                    extliq, ssaliq, asyliq, extice, ssaice, asyice)
    else
      err = co%load(band_lims_wvn, p_extliq, p_ssaliq, p_asyliq, p_extice, p_ssaice, p_asyice, &
                    sr_extliq, sr_ssaliq, sr_asyliq, sr_extice, sr_ssaice, sr_asyice)
    end if
    if (err /= '') then; last_msg = err; return; end if
    err = co%set_ice_roughness(int(icergh))
    if (err /= '') then; last_msg = err; return; end if
    if (nstr == 1) then
      err = o1%alloc_1scl(ncol, nlay, band_lims_wvn)
      if (err /= '') then; last_msg = err; return; end if
      err = co%cloud_optics(clwp, ciwp, reliq, reice, o1)
      if (err /= '') then; last_msg = err; return; end if
      tau = o1%tau
      ssa = 0._wp
      g = 0._wp
    else
      err = o2%alloc_2str(ncol, nlay, band_lims_wvn)
      if (err /= '') then; last_msg = err; return; end if
      err = co%cloud_optics(clwp, ciwp, reliq, reice, o2)
      if (err /= '') then; last_msg = err; return; end if
      tau = o2%tau
      ssa = o2%ssa
      g = o2%g
    end if
    ref_cloud_optics = 0
  end function ref_cloud_optics

  ! op_io (ngpt g-points, nstr_io) %increment'ed by op_in given by band (nband, nstr_in); in place.
  integer(c_int) function ref_increment_bybnd(ncol, nlay, nband, ngpt, band_lims_gpt, band_lims_wvn, nstr_io, &
      tau_io, ssa_io, g_io, nstr_in, tau_in, ssa_in, g_in) bind(C, name="ref_increment_bybnd")
    integer(c_int), value :: ncol, nlay, nband, ngpt, nstr_io, nstr_in
    integer(c_int), intent(in) :: band_lims_gpt(2, nband)
    real(c_float),  intent(in) :: band_lims_wvn(2, nband)
    real(c_float),  intent(inout) :: tau_io(ngpt, nlay, ncol), ssa_io(ngpt, nlay, ncol), g_io(ngpt, nlay, ncol)
    real(c_float),  intent(in) :: tau_in(nband, nlay, ncol), ssa_in(nband, nlay, ncol), g_in(nband, nlay, ncol)
    type(ty_optical_props_1scl) :: a1, b1
    type(ty_optical_props_2str) :: a2, b2
    character(len=128) :: err

    ref_increment_bybnd = 1
    err = ''
    if (nstr_in == 1) then
      err = b1%alloc_1scl(ncol, nlay, band_lims_wvn)
      b1%tau = tau_in
    else
      err = b2%alloc_2str(ncol, nlay, band_lims_wvn)
      b2%tau = tau_in; b2%ssa = ssa_in; b2%g = g_in
    end if
    if (err /= '') then; last_msg = err; return; end if
    if (nstr_io == 1) then
      err = a1%alloc_1scl(ncol, nlay, band_lims_wvn, band_lims_gpt)
      a1%tau = tau_io
      if (nstr_in == 1) then
        err = b1%increment(a1)
      else
        err = b2%increment(a1)
      end if
      tau_io = a1%tau
    else
      err = a2%alloc_2str(ncol, nlay, band_lims_wvn, band_lims_gpt)
      a2%tau = tau_io; a2%ssa = ssa_io; a2%g = g_io
      if (nstr_in == 1) then
        err = b1%increment(a2)
      else
        err = b2%increment(a2)
      end if
      tau_io = a2%tau; ssa_io = a2%ssa; g_io = a2%g
    end if
    if (err /= '') then; last_msg = err; return; end if
    ref_increment_bybnd = 0
  end function ref_increment_bybnd

  ! ty_optical_props_2str%delta_scale([for]) on (n, nlay, ncol) arrays, in place; has_for = 0: f = g**2.
  integer(c_int) function ref_delta_scale(ncol, nlay, nband, band_lims_wvn, tau, ssa, g, has_for, for) &
      bind(C, name="ref_delta_scale")
    integer(c_int), value :: ncol, nlay, nband, has_for
    real(c_float),  intent(in) :: band_lims_wvn(2, nband), for(nband, nlay, ncol)
    real(c_float),  intent(inout) :: tau(nband, nlay, ncol), ssa(nband, nlay, ncol), g(nband, nlay, ncol)
    type(ty_optical_props_2str) :: a
    character(len=128) :: err
    ref_delta_scale = 1
    err = a%alloc_2str(ncol, nlay, band_lims_wvn)
    if (err /= '') then; last_msg = err; return; end if
    a%tau = tau; a%ssa = ssa; a%g = g
    if (has_for /= 0) then
      err = a%delta_scale(for)
    else
      err = a%delta_scale()
    end if
    if (err /= '') then; last_msg = err; return; end if
    tau = a%tau; ssa = a%ssa; g = a%g
    ref_delta_scale = 0
  end function ref_delta_scale

end module ref_harness
