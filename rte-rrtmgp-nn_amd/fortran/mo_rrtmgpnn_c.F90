! mo_rrtmgpnn_c.F90 -- ISO_C_BINDING interfaces to include/rrtmgpnn.h (the C ABI of librrtmgpnn.so)
! plus the small device-memory helpers the Fortran class layer uses.  The Fortran modules in this
! directory keep the reference's module and type names (mo_rte_lw, mo_rte_sw, mo_gas_optics_rrtmgp,
! mod_network_rrtmgp, ...) so the reference's drivers compile against them unchanged; every
! computation runs in the HIP kernels behind this interface.
module mo_rrtmgpnn_c
  use, intrinsic :: iso_c_binding
  implicit none
  private
  public :: rrtmgpnn_ctx, rrtmgpnn_check, rrtmgpnn_error_message, rrtmgpnn_set_context, rrtmgpnn_sync, &
            rrtmgpnn_has_context
  ! the context's device data environment (include/rrtmgpnn.h, "Device data environment")
  public :: PRESENT_READ, PRESENT_WRITE, dev_present, dev_update_host, dev_update_device, dev_delete, dev_stage, &
            dev_scratch, dev_release, dev_copy_out, dev_copy_in, dev_copy_dd, dev_zero
  public :: c_rrtmgpnn_gas_optics_lw_nn, c_rrtmgpnn_gas_optics_sw_nn, c_rrtmgpnn_lw_solver_noscat_planck, &
            c_rrtmgpnn_sw_solver_noscat
  public :: c_rrtmgpnn_compute_heating_rate
  public :: c_rrtmgpnn_lw_solver_noscat_gpt, c_rrtmgpnn_lw_solver_noscat_planck_gpt, c_rrtmgpnn_sw_solver_2stream_gpt
  public :: c_rrtmgpnn_lw_solver_1rescl_gpt, c_rrtmgpnn_lw_solver_2stream_gpt, c_rrtmgpnn_sw_solver_noscat_gpt
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
  integer(c_int), parameter :: PRESENT_READ = 1, PRESENT_WRITE = 2

  interface
    integer(c_int) function c_rrtmgpnn_context_create(device, stream, ctx) bind(C, name="rrtmgpnn_context_create")
      import :: c_int, c_ptr
      integer(c_int), value :: device
      type(c_ptr), value :: stream
      type(c_ptr), intent(out) :: ctx
    end function
    integer(c_int) function c_rrtmgpnn_context_create_owned(device, ctx) bind(C, name="rrtmgpnn_context_create_owned")
      import :: c_int, c_ptr
      integer(c_int), value :: device
      type(c_ptr), intent(out) :: ctx
    end function
    integer(c_int) function c_rrtmgpnn_present(ctx, host, bytes, mode, dptr) bind(C, name="rrtmgpnn_present")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, host
      integer(c_long_long), value :: bytes
      integer(c_int), value :: mode
      type(c_ptr), intent(out) :: dptr
    end function
    integer(c_int) function c_rrtmgpnn_present_update_host(ctx, host) bind(C, name="rrtmgpnn_present_update_host")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, host
    end function
    integer(c_int) function c_rrtmgpnn_present_update_device(ctx, host) bind(C, name="rrtmgpnn_present_update_device")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, host
    end function
    integer(c_int) function c_rrtmgpnn_present_delete(ctx, host) bind(C, name="rrtmgpnn_present_delete")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, host
    end function
    integer(c_int) function c_rrtmgpnn_stage_h2d(ctx, host, bytes, dptr) bind(C, name="rrtmgpnn_stage_h2d")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, host
      integer(c_long_long), value :: bytes
      type(c_ptr), intent(out) :: dptr
    end function
    integer(c_int) function c_rrtmgpnn_scratch(ctx, bytes, dptr) bind(C, name="rrtmgpnn_scratch")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx
      integer(c_long_long), value :: bytes
      type(c_ptr), intent(out) :: dptr
    end function
    integer(c_int) function c_rrtmgpnn_release(ctx, dptr) bind(C, name="rrtmgpnn_release")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, dptr
    end function
    integer(c_int) function c_rrtmgpnn_copy_d2h(ctx, host, dptr, bytes) bind(C, name="rrtmgpnn_copy_d2h")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, host, dptr
      integer(c_long_long), value :: bytes
    end function
    integer(c_int) function c_rrtmgpnn_copy_h2d(ctx, dptr, host, bytes) bind(C, name="rrtmgpnn_copy_h2d")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, dptr, host
      integer(c_long_long), value :: bytes
    end function
    integer(c_int) function c_rrtmgpnn_copy_d2d(ctx, dst, src, bytes) bind(C, name="rrtmgpnn_copy_d2d")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, dst, src
      integer(c_long_long), value :: bytes
    end function
    integer(c_int) function c_rrtmgpnn_memset_async(ctx, dptr, val, bytes) bind(C, name="rrtmgpnn_memset_async")
      import :: c_int, c_ptr, c_long_long
      type(c_ptr), value :: ctx, dptr
      integer(c_int), value :: val
      integer(c_long_long), value :: bytes
    end function
    integer(c_int) function c_rrtmgpnn_gas_optics_lw_nn(ctx, ncol, nlay, ngpt, ninputs, play, tlay, plev, vmr_h2o, &
        gas_conc, gas_ndims, nets, nnets, tau, pfrac) bind(C, name="rrtmgpnn_gas_optics_lw_nn")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, play, tlay, plev, vmr_h2o, tau, pfrac
      integer(c_int), value :: ncol, nlay, ngpt, ninputs, nnets
      type(c_ptr), dimension(*), intent(in) :: gas_conc, nets
      integer(c_int), dimension(*), intent(in) :: gas_ndims
    end function
    integer(c_int) function c_rrtmgpnn_gas_optics_sw_nn(ctx, ncol, nlay, ngpt, ninputs, play, tlay, plev, vmr_h2o, &
        gas_conc, gas_ndims, nets, tau, ssa, g) bind(C, name="rrtmgpnn_gas_optics_sw_nn")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, play, tlay, plev, vmr_h2o, tau, ssa, g
      integer(c_int), value :: ncol, nlay, ngpt, ninputs
      type(c_ptr), dimension(*), intent(in) :: gas_conc, nets
      integer(c_int), dimension(*), intent(in) :: gas_ndims
    end function
    integer(c_int) function c_rrtmgpnn_lw_solver_noscat_planck(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, &
        inc_flux, tau, pfrac, nbnd, nPlanckTemp, tlay, tlev, tsfc, sfc_lay, band_lims_gpt, temp_ref_min, &
        totplnk_delta, totplnk, emis_by_band, sfc_emis, flux_up, flux_dn) bind(C, name="rrtmgpnn_lw_solver_noscat_planck")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx, inc_flux, tau, pfrac, tlay, tlev, tsfc, totplnk, sfc_emis, flux_up, flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1, nmus, nbnd, nPlanckTemp, sfc_lay, emis_by_band
      real(c_float), dimension(*), intent(in) :: Ds, weights
      integer(c_int), dimension(*), intent(in) :: band_lims_gpt
      real(c_float), value :: temp_ref_min, totplnk_delta
    end function
    integer(c_int) function c_rrtmgpnn_sw_solver_noscat(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, mu0, flux_dir) &
        bind(C, name="rrtmgpnn_sw_solver_noscat")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, inc_flux, tau, mu0, flux_dir
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1
    end function
    integer(c_int) function c_rrtmgpnn_context_synchronize(ctx) bind(C, name="rrtmgpnn_context_synchronize")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx
    end function
    type(c_ptr) function c_rrtmgpnn_last_error() bind(C, name="rrtmgpnn_last_error")
      import :: c_ptr
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
    ! ty_fluxes_flexible g-point outputs and lw_Ds (include/rrtmgpnn.h)
    integer(c_int) function c_rrtmgpnn_lw_solver_noscat_gpt(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, lw_Ds, &
        inc_flux, tau, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn, gpt_flux_up, gpt_flux_dn) &
        bind(C, name="rrtmgpnn_lw_solver_noscat_gpt")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx, lw_Ds, inc_flux, tau, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, &
                            flux_dn, gpt_flux_up, gpt_flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1, nmus
      real(c_float), dimension(*), intent(in) :: Ds, weights
    end function
    integer(c_int) function c_rrtmgpnn_lw_solver_noscat_planck_gpt(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, &
        lw_Ds, inc_flux, tau, pfrac, nbnd, nPlanckTemp, tlay, tlev, tsfc, sfc_lay, band_lims_gpt, temp_ref_min, &
        totplnk_delta, totplnk, emis_by_band, sfc_emis, flux_up, flux_dn, gpt_flux_up, gpt_flux_dn) &
        bind(C, name="rrtmgpnn_lw_solver_noscat_planck_gpt")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx, lw_Ds, inc_flux, tau, pfrac, tlay, tlev, tsfc, totplnk, sfc_emis, flux_up, flux_dn, &
                            gpt_flux_up, gpt_flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1, nmus, nbnd, nPlanckTemp, sfc_lay, emis_by_band
      real(c_float), dimension(*), intent(in) :: Ds, weights
      integer(c_int), dimension(*), intent(in) :: band_lims_gpt
      real(c_float), value :: temp_ref_min, totplnk_delta
    end function
    integer(c_int) function c_rrtmgpnn_sw_solver_2stream_gpt(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, inc_flux_dif, &
        tau, ssa, g, mu0, sfc_alb_dir_gpt, sfc_alb_dif_gpt, flux_up, flux_dn, flux_dir, gpt_flux_up, gpt_flux_dn, &
        gpt_flux_dir) bind(C, name="rrtmgpnn_sw_solver_2stream_gpt")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, inc_flux, inc_flux_dif, tau, ssa, g, mu0, sfc_alb_dir_gpt, sfc_alb_dif_gpt, &
                            flux_up, flux_dn, flux_dir, gpt_flux_up, gpt_flux_dn, gpt_flux_dir
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1
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
    integer(c_int) function c_rrtmgpnn_lw_solver_1rescl_gpt(ctx, ngpt, nlay, ncol, top_at_1, nmus, Ds, weights, &
        inc_flux, tau, ssa, g, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn, gpt_flux_up, &
        gpt_flux_dn) bind(C, name="rrtmgpnn_lw_solver_1rescl_gpt")
      import :: c_int, c_ptr, c_float
      type(c_ptr), value :: ctx, inc_flux, tau, ssa, g, lay_source, lev_source, sfc_emis_gpt, sfc_source, flux_up, &
                            flux_dn, gpt_flux_up, gpt_flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1, nmus
      real(c_float), dimension(*), intent(in) :: Ds, weights
    end function
    integer(c_int) function c_rrtmgpnn_lw_solver_2stream_gpt(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, ssa, g, &
        lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn, gpt_flux_up, gpt_flux_dn) &
        bind(C, name="rrtmgpnn_lw_solver_2stream_gpt")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, inc_flux, tau, ssa, g, lev_source, sfc_emis_gpt, sfc_source, flux_up, flux_dn, &
                            gpt_flux_up, gpt_flux_dn
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1
    end function
    integer(c_int) function c_rrtmgpnn_sw_solver_noscat_gpt(ctx, ngpt, nlay, ncol, top_at_1, inc_flux, tau, mu0, &
        flux_dir, gpt_flux_dir) bind(C, name="rrtmgpnn_sw_solver_noscat_gpt")
      import :: c_int, c_ptr
      type(c_ptr), value :: ctx, inc_flux, tau, mu0, flux_dir, gpt_flux_dir
      integer(c_int), value :: ngpt, nlay, ncol, top_at_1
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

  ! The calling thread's context (created on device 0 with a stream of its own, on first use): host threads with a
  ! context each -- OpenMP over blocks, rrtmgp_rfmip_lw.F90:364-367 -- run concurrently on the device.
  function rrtmgpnn_ctx() result(ctx)
    type(c_ptr) :: ctx
    integer(c_int) :: rc
    if (.not. c_associated(ctx_)) then
      rc = c_rrtmgpnn_context_create_owned(0_c_int, ctx_)
      if (rc /= 0) then
        write(*, '(a)') "rrtmgpnn: " // trim(rrtmgpnn_error_message())
        error stop 1
      end if
    end if
    ctx = ctx_
  end function rrtmgpnn_ctx

  ! Whether this thread has a context yet (host-only uses of the classes never create one).
  logical function rrtmgpnn_has_context()
    rrtmgpnn_has_context = c_associated(ctx_)
  end function rrtmgpnn_has_context

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

  ! Wait for the context's stream; keeps an earlier error message.
  subroutine rrtmgpnn_sync(error_msg, what)
    character(len=128), intent(inout) :: error_msg
    character(len=*), intent(in) :: what
    character(len=128) :: e
    e = rrtmgpnn_check(c_rrtmgpnn_context_synchronize(rrtmgpnn_ctx()), what)
    if (error_msg == '') error_msg = e
  end subroutine rrtmgpnn_sync

  ! ---- device data environment.  Sizes are element counts (4-byte reals or integers) in 64-bit integers: a C5
  ! shard's g-point arrays hold more than 2**31 elements.  h is any contiguous host array (sequence association).
  ! The device copy of h(1:n) in the context's data environment (mode PRESENT_READ: current data, uploaded when
  ! the host copy is newer; PRESENT_WRITE: the caller's kernel writes it).
  function dev_present(h, n, mode) result(d)
    real(c_float), dimension(*), intent(in), target :: h
    integer(c_long_long), intent(in) :: n
    integer(c_int), intent(in) :: mode
    type(c_ptr) :: d
    d = c_null_ptr
    if (n <= 0) call fatal("present: non-positive size")
    if (c_rrtmgpnn_present(rrtmgpnn_ctx(), c_loc(h), 4_c_long_long * n, mode, d) /= 0) call fatal("present")
  end function dev_present

  ! `!$acc update host`: copy a device-newer array back into h and wait for it.
  subroutine dev_update_host(h)
    real(c_float), dimension(*), intent(inout), target :: h
    if (.not. c_associated(ctx_)) return  ! no context yet: nothing is on the device
    if (c_rrtmgpnn_present_update_host(ctx_, c_loc(h)) /= 0) call fatal("update host")
  end subroutine dev_update_host

  ! `!$acc update device`: h changed on the host; it is uploaded when a kernel next reads it.
  subroutine dev_update_device(h)
    real(c_float), dimension(*), intent(in), target :: h
    if (.not. c_associated(ctx_)) return  ! no context yet: nothing is on the device
    if (c_rrtmgpnn_present_update_device(ctx_, c_loc(h)) /= 0) call fatal("update device")
  end subroutine dev_update_device

  ! `!$acc exit data delete`: drop h's device copy (its buffer returns to the pool).
  subroutine dev_delete(h)
    real(c_float), dimension(*), intent(in), target :: h
    if (.not. c_associated(ctx_)) return  ! no context yet: nothing is on the device
    if (c_rrtmgpnn_present_delete(ctx_, c_loc(h)) /= 0) call fatal("delete")
  end subroutine dev_delete

  ! A pool buffer holding a copy of h(1:n) (a call's input; release it when the call's kernels are enqueued).
  function dev_stage(h, n) result(d)
    real(c_float), dimension(*), intent(in), target :: h
    integer(c_long_long), intent(in) :: n
    type(c_ptr) :: d
    d = c_null_ptr
    if (n <= 0) call fatal("stage: non-positive size")
    if (c_rrtmgpnn_stage_h2d(rrtmgpnn_ctx(), c_loc(h), 4_c_long_long * n, d) /= 0) call fatal("host-to-device copy")
  end function dev_stage

  ! An uninitialised pool buffer of n floats.
  function dev_scratch(n) result(d)
    integer(c_long_long), intent(in) :: n
    type(c_ptr) :: d
    d = c_null_ptr
    if (n <= 0) call fatal("scratch: non-positive size")
    if (c_rrtmgpnn_scratch(rrtmgpnn_ctx(), 4_c_long_long * n, d) /= 0) call fatal("device allocation")
  end function dev_scratch

  subroutine dev_release(d)
    type(c_ptr), intent(inout) :: d
    if (c_associated(d)) then
      if (c_rrtmgpnn_release(rrtmgpnn_ctx(), d) /= 0) call fatal("release")
    end if
    d = c_null_ptr
  end subroutine dev_release

  ! Enqueue the copy of n floats from d into h (complete after rrtmgpnn_sync).
  subroutine dev_copy_out(h, d, n)
    real(c_float), dimension(*), intent(inout), target :: h
    type(c_ptr), intent(in) :: d
    integer(c_long_long), intent(in) :: n
    if (c_rrtmgpnn_copy_d2h(rrtmgpnn_ctx(), c_loc(h), d, 4_c_long_long * n) /= 0) call fatal("device-to-host copy")
  end subroutine dev_copy_out

  ! Enqueue the copy of h(1:n) into the device buffer d.
  subroutine dev_copy_in(d, h, n)
    type(c_ptr), intent(in) :: d
    real(c_float), dimension(*), intent(in), target :: h
    integer(c_long_long), intent(in) :: n
    if (c_rrtmgpnn_copy_h2d(rrtmgpnn_ctx(), d, c_loc(h), 4_c_long_long * n) /= 0) call fatal("host-to-device copy")
  end subroutine dev_copy_in

  ! Enqueue the copy of n floats from device buffer s into device buffer d.
  subroutine dev_copy_dd(d, src, n)
    type(c_ptr), intent(in) :: d, src
    integer(c_long_long), intent(in) :: n
    if (c_rrtmgpnn_copy_d2d(rrtmgpnn_ctx(), d, src, 4_c_long_long * n) /= 0) call fatal("device-to-device copy")
  end subroutine dev_copy_dd

  subroutine dev_zero(d, n)
    type(c_ptr), intent(in) :: d
    integer(c_long_long), intent(in) :: n
    if (c_rrtmgpnn_memset_async(rrtmgpnn_ctx(), d, 0_c_int, 4_c_long_long * n) /= 0) call fatal("memset")
  end subroutine dev_zero

  subroutine fatal(what)
    character(len=*), intent(in) :: what
    write(*, '(a)') "rrtmgpnn: " // what // ": " // trim(rrtmgpnn_error_message())
    error stop 1
  end subroutine fatal
end module mo_rrtmgpnn_c
