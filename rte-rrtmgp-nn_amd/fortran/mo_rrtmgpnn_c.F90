! mo_rrtmgpnn_c.F90 -- ISO_C_BINDING interfaces to include/rrtmgpnn.h (the C ABI of librrtmgpnn.so)
! plus the small device-memory helpers the Fortran class layer uses.  The Fortran modules in this
! directory keep the reference's module and type names (mo_rte_lw, mo_rte_sw, mo_gas_optics_rrtmgp,
! mod_network_rrtmgp, ...) so the reference's drivers compile against them unchanged; every
! computation runs in the HIP kernels behind this interface.
module mo_rrtmgpnn_c
  use, intrinsic :: iso_c_binding
  implicit none
  private
  public :: rrtmgpnn_ctx, rrtmgpnn_check, rrtmgpnn_error_message, dev_alloc, dev_free, h2d, d2h, &
            rrtmgpnn_set_context, dev_upload, dev_download, dev_upload_int
  public :: c_rrtmgpnn_compute_heating_rate
  public :: c_rrtmgpnn_network_load, c_rrtmgpnn_compute_nn_inputs, c_rrtmgpnn_get_col_dry, &
            c_rrtmgpnn_interpolate_tlev, c_rrtmgpnn_predict_nn_lw, c_rrtmgpnn_predict_nn_sw, &
            c_rrtmgpnn_compute_planck_source_nn, c_rrtmgpnn_lw_solver_noscat, c_rrtmgpnn_sw_solver_2stream, &
            c_rrtmgpnn_expand_band_to_gpt, c_rrtmgpnn_context_synchronize, c_rrtmgpnn_network_destroy
  public :: c_rrtmgpnn_cloud_optics_create_lut, c_rrtmgpnn_cloud_optics_create_pade, &
            c_rrtmgpnn_cloud_optics_set_ice_roughness, c_rrtmgpnn_cloud_optics_load, c_rrtmgpnn_cloud_optics_get, &
            c_rrtmgpnn_cloud_optics_destroy, c_rrtmgpnn_cloud_optics_compute, c_rrtmgpnn_increment_bybnd, &
            c_rrtmgpnn_increment, c_rrtmgpnn_delta_scale_2str, c_rrtmgpnn_lw_solver_1rescl, &
            c_rrtmgpnn_lw_solver_2stream

  type(c_ptr), save :: ctx_ = c_null_ptr
  !$omp threadprivate(ctx_)

  interface
    integer(c_int) function c_rrtmgpnn_context_create(device, stream, ctx) bind(C, name="rrtmgpnn_context_create")
      import :: c_int, c_ptr
      integer(c_int), value :: device
      type(c_ptr), value :: stream
      type(c_ptr), intent(out) :: ctx
    end function
    integer(c_int) function c_rrtmgpnn_context_synchronize(ctx) bind(C, name="rrtmgpnn_context_synchronize")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx
    end function
    type(c_ptr) function c_rrtmgpnn_last_error() bind(C, name="rrtmgpnn_last_error")
      import :: c_ptr
    end function
    integer(c_int) function c_rrtmgpnn_malloc(ctx, bytes, dptr) bind(C, name="rrtmgpnn_malloc")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx
      integer(c_long_long), value :: bytes
      type(c_ptr), intent(out) :: dptr
    end function
    integer(c_int) function c_rrtmgpnn_free(ctx, dptr) bind(C, name="rrtmgpnn_free")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, dptr
    end function
    integer(c_int) function c_rrtmgpnn_memcpy_h2d(ctx, dst, src, bytes) bind(C, name="rrtmgpnn_memcpy_h2d")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, dst, src
      integer(c_long_long), value :: bytes
    end function
    integer(c_int) function c_rrtmgpnn_memcpy_d2h(ctx, dst, src, bytes) bind(C, name="rrtmgpnn_memcpy_d2h")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, dst, src
      integer(c_long_long), value :: bytes
    end function
    integer(c_int) function c_rrtmgpnn_network_load(ctx, path, net) bind(C, name="rrtmgpnn_network_load")
      import :: c_int, c_ptr, c_char
      type(c_ptr), value :: ctx
      character(kind=c_char), dimension(*), intent(in) :: path
      type(c_ptr), intent(out) :: net
    end function
    integer(c_int) function c_rrtmgpnn_network_destroy(net) bind(C, name="rrtmgpnn_network_destroy")
      import :: c_int, c_ptr
      type(c_ptr), value :: net
    end function
    integer(c_int) function c_rrtmgpnn_compute_nn_inputs(ctx, ncol, nlay, ninputs, play, tlay, gas_conc, gas_ndims, &
                                                         net, nn_inputs) bind(C, name="rrtmgpnn_compute_nn_inputs")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, play, tlay, net, nn_inputs
      integer(c_int), value :: ncol, nlay, ninputs
      type(c_ptr), dimension(*), intent(in) :: gas_conc
      integer(c_int), dimension(*), intent(in) :: gas_ndims
    end function
    integer(c_int) function c_rrtmgpnn_get_col_dry(ctx, ncol, nlay, vmr_h2o, plev, col_dry) &
        bind(C, name="rrtmgpnn_get_col_dry")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, vmr_h2o, plev, col_dry
      integer(c_int), value :: ncol, nlay
    end function
    integer(c_int) function c_rrtmgpnn_interpolate_tlev(ctx, ncol, nlay, play, plev, tlay, tlev) &
        bind(C, name="rrtmgpnn_interpolate_tlev")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, play, plev, tlay, tlev
      integer(c_int), value :: ncol, nlay
    end function
    integer(c_int) function c_rrtmgpnn_predict_nn_lw(ctx, ncol, nlay, ngpt, ninputs, nn_inputs, col_dry, nets, nnets, &
                                                     tau, pfrac) bind(C, name="rrtmgpnn_predict_nn_lw")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, nn_inputs, col_dry, tau, pfrac
      integer(c_int), value :: ncol, nlay, ngpt, ninputs, nnets
      type(c_ptr), dimension(*), intent(in) :: nets
    end function
    integer(c_int) function c_rrtmgpnn_predict_nn_sw(ctx, ncol, nlay, ngpt, ninputs, nn_inputs, col_dry, nets, &
                                                     tau, ssa, g) bind(C, name="rrtmgpnn_predict_nn_sw")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, nn_inputs, col_dry, tau, ssa, g
      integer(c_int), value :: ncol, nlay, ngpt, ninputs
      type(c_ptr), dimension(*), intent(in) :: nets
    end function
    integer(c_int) function c_rrtmgpnn_compute_planck_source_nn(ctx, ncol, nlay, nbnd, ngpt, nPlanckTemp, tlay, tlev, &
        tsfc, sfc_lay, band_lims_gpt, temp_ref_min, totplnk_delta, totplnk, sfc_source, sfc_source_Jac, pfrac, &
        lev_source) bind(C, name="rrtmgpnn_compute_planck_source_nn")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx, tlay, tlev, tsfc, totplnk, sfc_source, sfc_source_Jac, pfrac, lev_source
      integer(c_int), value :: ncol, nlay, nbnd, ngpt, nPlanckTemp, sfc_lay
      integer(c_int), dimension(*), intent(in) :: band_lims_gpt
      real(c_float), value :: temp_ref_min, totplnk_delta
    end function
    integer(c_int) function c_rrtmgpnn_lw_solver_noscat(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, inc_flux, &
        tau, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn) bind(C, name="rrtmgpnn_lw_solver_noscat")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx, inc_flux, tau, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1, nmus
      real(c_float), dimension(*), intent(in) :: Ds, weights
    end function
    integer(c_int) function c_rrtmgpnn_lw_solver_1rescl(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, &
        inc_flux, tau, ssa, g, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn) &
        bind(C, name="rrtmgpnn_lw_solver_1rescl")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx, inc_flux, tau, ssa, g, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, &
                            flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1, nmus
      real(c_float), dimension(*), intent(in) :: Ds, weights
    end function
    integer(c_int) function c_rrtmgpnn_lw_solver_2stream(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, ssa, g, &
        lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn) bind(C, name="rrtmgpnn_lw_solver_2stream")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, inc_flux, tau, ssa, g, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1
    end function
    integer(c_int) function c_rrtmgpnn_sw_solver_2stream(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, &
        tau, ssa, g, mu0, sfc_alb_dir_gpt, sfc_alb_dif_gpt, flux_up, flux_dn, flux_dir) &
        bind(C, name="rrtmgpnn_sw_solver_2stream")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, inc_flux, inc_flux_dif, tau, ssa, g, mu0, sfc_alb_dir_gpt, sfc_alb_dif_gpt, &
                            flux_up, flux_dn, flux_dir
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1
    end function
    integer(c_int) function c_rrtmgpnn_expand_band_to_gpt(ctx, nband, ngpt, ncol, band_lims_gpt, arr_in, arr_out) &
        bind(C, name="rrtmgpnn_expand_band_to_gpt")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, arr_in, arr_out
      integer(c_int), value :: nband, ngpt, ncol
      integer(c_int), dimension(*), intent(in) :: band_lims_gpt
    end function
    integer(c_int) function c_rrtmgpnn_compute_heating_rate(ctx, ncol, nlay, flux_up, flux_dn, plev, heating_rate) &
        bind(C, name="rrtmgpnn_compute_heating_rate")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, flux_up, flux_dn, plev, heating_rate
      integer(c_int), value :: ncol, nlay
    end function
    ! ---- all-sky: cloud optics, increment, delta scaling ----
    integer(c_int) function c_rrtmgpnn_cloud_optics_create_lut(ctx, nband, band_lims_wvn, nsize_liq, nsize_ice, &
        nrghice, radliq_lwr, radliq_upr, radice_lwr, radice_upr, lut_extliq, lut_ssaliq, lut_asyliq, lut_extice, &
        lut_ssaice, lut_asyice, co) bind(C, name="rrtmgpnn_cloud_optics_create_lut")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx
      integer(c_int), value :: nband, nsize_liq, nsize_ice, nrghice
      real(c_float), value :: radliq_lwr, radliq_upr, radice_lwr, radice_upr
      real(c_float), dimension(*), intent(in) :: band_lims_wvn, lut_extliq, lut_ssaliq, lut_asyliq, lut_extice, &
                                                 lut_ssaice, lut_asyice
      type(c_ptr), intent(out) :: co
    end function
    integer(c_int) function c_rrtmgpnn_cloud_optics_create_pade(ctx, nband, band_lims_wvn, nsizereg, ncoef_ext, &
        ncoef_ssa, nrghice, pade_extliq, pade_ssaliq, pade_asyliq, pade_extice, pade_ssaice, pade_asyice, &
        sizreg_extliq, sizreg_ssaliq, sizreg_asyliq, sizreg_extice, sizreg_ssaice, sizreg_asyice, co) &
        bind(C, name="rrtmgpnn_cloud_optics_create_pade")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx
      integer(c_int), value :: nband, nsizereg, ncoef_ext, ncoef_ssa, nrghice
      real(c_float), dimension(*), intent(in) :: band_lims_wvn, pade_extliq, pade_ssaliq, pade_asyliq, &
                                                 pade_extice, pade_ssaice, pade_asyice, sizreg_extliq, &
                                                 sizreg_ssaliq, sizreg_asyliq, sizreg_extice, sizreg_ssaice, &
                                                 sizreg_asyice
      type(c_ptr), intent(out) :: co
    end function
    integer(c_int) function c_rrtmgpnn_cloud_optics_load(ctx, path, use_lut, co) bind(C, name="rrtmgpnn_cloud_optics_load")
      import :: c_int, c_ptr, c_char
      type(c_ptr), value :: ctx
      character(kind=c_char), dimension(*), intent(in) :: path
      integer(c_int), value :: use_lut
      type(c_ptr), intent(out) :: co
    end function
    integer(c_int) function c_rrtmgpnn_cloud_optics_set_ice_roughness(co, icergh) &
        bind(C, name="rrtmgpnn_cloud_optics_set_ice_roughness")
      import :: c_int, c_ptr
      type(c_ptr), value :: co
      integer(c_int), value :: icergh
    end function
    integer(c_int) function c_rrtmgpnn_cloud_optics_get(co, nband, nrghice, radii) bind(C, name="rrtmgpnn_cloud_optics_get")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: co
      integer(c_int), intent(out) :: nband, nrghice
      real(c_float), dimension(4), intent(out) :: radii
    end function
    integer(c_int) function c_rrtmgpnn_cloud_optics_destroy(co) bind(C, name="rrtmgpnn_cloud_optics_destroy")
      import :: c_int, c_ptr
      type(c_ptr), value :: co
    end function
    integer(c_int) function c_rrtmgpnn_cloud_optics_compute(ctx, co, ncol, nlay, clwp, ciwp, reliq, reice, tau, ssa, g) &
        bind(C, name="rrtmgpnn_cloud_optics_compute")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, co, clwp, ciwp, reliq, reice, tau, ssa, g
      integer(c_int), value :: ncol, nlay
    end function
    integer(c_int) function c_rrtmgpnn_increment_bybnd(ctx, ncol, nlay, ngpt, nband, band_lims_gpt, tau_io, ssa_io, &
        g_io, tau_in, ssa_in, g_in) bind(C, name="rrtmgpnn_increment_bybnd")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, tau_io, ssa_io, g_io, tau_in, ssa_in, g_in
      integer(c_int), value :: ncol, nlay, ngpt, nband
      integer(c_int), dimension(*), intent(in) :: band_lims_gpt
    end function
    integer(c_int) function c_rrtmgpnn_increment(ctx, ncol, nlay, ngpt, tau_io, ssa_io, g_io, tau_in, ssa_in, g_in) &
        bind(C, name="rrtmgpnn_increment")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, tau_io, ssa_io, g_io, tau_in, ssa_in, g_in
      integer(c_int), value :: ncol, nlay, ngpt
    end function
    integer(c_int) function c_rrtmgpnn_delta_scale_2str(ctx, n, tau, ssa, g, fwd) bind(C, name="rrtmgpnn_delta_scale_2str")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, tau, ssa, g, fwd
      integer(c_long_long), value :: n
    end function
    integer(c_size_t) function c_strlen(s) bind(C, name="strlen")
      import :: c_size_t, c_ptr
      type(c_ptr), value :: s
    end function
  end interface

contains

  ! The calling thread's context (created on device 0, legacy default stream, on first use).
  function rrtmgpnn_ctx() result(ctx)
    type(c_ptr) :: ctx
    integer(c_int) :: rc
    if (.not. c_associated(ctx_)) then
      rc = c_rrtmgpnn_context_create(0_c_int, c_null_ptr, ctx_)
      if (rc /= 0) then
        write(*, '(a)') "rrtmgpnn: " // trim(rrtmgpnn_error_message())
        error stop 1
      end if
    end if
    ctx = ctx_
  end function rrtmgpnn_ctx

  ! Use an existing context (e.g. one per OpenMP thread / GPU) for this thread's calls.
  subroutine rrtmgpnn_set_context(ctx)
    type(c_ptr), intent(in) :: ctx
    ctx_ = ctx
  end subroutine rrtmgpnn_set_context

  function rrtmgpnn_error_message() result(msg)
    character(len=128) :: msg
    type(c_ptr) :: p
    character(kind=c_char), dimension(:), pointer :: s
    integer :: n, i
    msg = ''
    p = c_rrtmgpnn_last_error()
    if (.not. c_associated(p)) return
    n = int(c_strlen(p))
    call c_f_pointer(p, s, [max(n, 1)])
    do i = 1, min(n, 128)
      msg(i:i) = s(i)
    end do
  end function rrtmgpnn_error_message

  ! Map a C return code to the reference convention: '' on success, the message otherwise.
  function rrtmgpnn_check(rc, what) result(error_msg)
    integer(c_int), intent(in) :: rc
    character(len=*), intent(in) :: what
    character(len=128) :: error_msg
    error_msg = ''
    if (rc /= 0) error_msg = trim(what) // ": " // trim(rrtmgpnn_error_message())
  end function rrtmgpnn_check

  function dev_alloc(nfloats) result(d)
    integer, intent(in) :: nfloats
    type(c_ptr) :: d
    integer(c_int) :: rc
    rc = c_rrtmgpnn_malloc(rrtmgpnn_ctx(), int(max(nfloats, 1), c_long_long) * 4_c_long_long, d)
    if (rc /= 0) then
      write(*, '(a)') "rrtmgpnn: device allocation failed: " // trim(rrtmgpnn_error_message())
      error stop 1
    end if
  end function dev_alloc

  subroutine dev_free(d)
    type(c_ptr), intent(inout) :: d
    integer(c_int) :: rc
    if (c_associated(d)) rc = c_rrtmgpnn_free(rrtmgpnn_ctx(), d)
    d = c_null_ptr
  end subroutine dev_free

  subroutine h2d(d, h, nfloats)
    type(c_ptr), intent(in) :: d, h
    integer, intent(in) :: nfloats
    integer(c_int) :: rc
    if (nfloats <= 0) return
    rc = c_rrtmgpnn_memcpy_h2d(rrtmgpnn_ctx(), d, h, int(nfloats, c_long_long) * 4_c_long_long)
    if (rc /= 0) call fatal("host-to-device copy failed")
  end subroutine h2d

  subroutine d2h(h, d, nfloats)
    type(c_ptr), intent(in) :: h, d
    integer, intent(in) :: nfloats
    integer(c_int) :: rc
    if (nfloats <= 0) return
    rc = c_rrtmgpnn_memcpy_d2h(rrtmgpnn_ctx(), h, d, int(nfloats, c_long_long) * 4_c_long_long)
    if (rc /= 0) call fatal("device-to-host copy failed")
  end subroutine d2h

  ! Allocate n floats on the device and copy h(1:n) there (sequence association: any rank).
  function dev_upload(h, n) result(d)
    integer, intent(in) :: n
    real(c_float), dimension(n), intent(in), target :: h
    type(c_ptr) :: d
    d = dev_alloc(n)
    call h2d(d, c_loc(h), n)
  end function dev_upload

  function dev_upload_int(h, n) result(d)
    integer, intent(in) :: n
    integer(c_int), dimension(n), intent(in), target :: h
    type(c_ptr) :: d
    d = dev_alloc(n)
    call h2d(d, c_loc(h), n)
  end function dev_upload_int

  ! Copy n floats from device d into h(1:n); frees d when `release` is present and true.
  subroutine dev_download(h, d, n, release)
    integer, intent(in) :: n
    real(c_float), dimension(n), intent(inout), target :: h
    type(c_ptr), intent(inout) :: d
    logical, optional, intent(in) :: release
    call d2h(c_loc(h), d, n)
    if (present(release)) then
      if (release) call dev_free(d)
    end if
  end subroutine dev_download

  subroutine fatal(what)
    character(len=*), intent(in) :: what
    write(*, '(a)') "rrtmgpnn: " // what // ": " // trim(rrtmgpnn_error_message())
    error stop 1
  end subroutine fatal
end module mo_rrtmgpnn_c
