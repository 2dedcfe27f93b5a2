! mo_rte_lw -- drop-in for rte/mo_rte_lw.F90 (rte_lw, :60-424) in the fork's configuration
! (compute_Jac = .false., rte/mo_rte_rrtmgp_config.F90:28).
! The optical properties and sources are read from their device copies (mo_optical_props, mo_source_functions);
! sources gas_optics left unformed are formed inside the no-scattering solver from the Planck fraction
! (rrtmgpnn_lw_solver_noscat_planck, emissivity expanded by band in-kernel); the broadband reduction is fused into
! every solver, and the fluxes come back into the caller's flux_up / flux_dn / flux_net.
! 1scl: lw_solver_noscat_GaussQuad; 2str: the rescaled solution (default) or lw_solver_2stream
! (use_2stream).  ty_fluxes_flexible g-point fluxes through the *_gpt entries: no-scattering and rescaled solutions
! with one angle the g-point radiances (quirk B-5), with several the angle-summed fluxes; lw_solver_2stream the adding
! fluxes.  lw_Ds on 1scl properties; flux_up_Jac / flux_dn_Jac accepted and left untouched (compute_Jac = .false.),
! an error string only with use_2stream, as the reference.
module mo_rte_lw
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,         only: wp
  use mo_optical_props,    only: ty_optical_props_arry, ty_optical_props_1scl, ty_optical_props_2str, dev_g_read
  use mo_source_functions, only: ty_source_func_lw
  use mo_fluxes,           only: ty_fluxes_flexible
  use mo_rte_rrtmgp_config, only: check_values
  use mo_rrtmgpnn_c
  implicit none
  private
  public :: rte_lw

  integer,  parameter :: max_gauss_pts = 4
  ! Diffusivity angle (nmus = 1) and Gauss-Jacobi-5 quadrature (mo_rte_lw.F90:113-125)
  real(c_float), parameter, dimension(max_gauss_pts, max_gauss_pts) :: &
    gauss_Ds  = reshape([1.66_wp,         0._wp,           0._wp,           0._wp, &
                         1.18350343_wp,   2.81649655_wp,   0._wp,           0._wp, &
                         1.09719858_wp,   1.69338507_wp,   4.70941630_wp,   0._wp, &
                         1.06056257_wp,   1.38282560_wp,   2.40148179_wp,   7.15513024_wp], [4, 4]), &
    gauss_wts = reshape([0.5_wp,          0._wp,           0._wp,           0._wp, &
                         0.3180413817_wp, 0.1819586183_wp, 0._wp,           0._wp, &
                         0.2009319137_wp, 0.2292411064_wp, 0.0698269799_wp, 0._wp, &
                         0.1355069134_wp, 0.2034645680_wp, 0.1298475476_wp, 0.0311809710_wp], [4, 4])

contains

  function rte_lw(optical_props, top_at_1, sources, sfc_emis, fluxes, inc_flux, n_gauss_angles, use_2stream, &
                  lw_Ds, flux_up_Jac, flux_dn_Jac) result(error_msg)
    class(ty_optical_props_arry), intent(in) :: optical_props
    logical,                      intent(in) :: top_at_1
    type(ty_source_func_lw),      intent(in) :: sources
    real(wp), dimension(:,:),     intent(in) :: sfc_emis        ! (nband, ncol)
    class(ty_fluxes_flexible), intent(inout) :: fluxes
    real(wp), dimension(:,:), contiguous, target, optional, intent(in) :: inc_flux   ! (ngpt, ncol)
    integer,  optional, intent(in) :: n_gauss_angles
    logical,  optional, intent(in) :: use_2stream
    real(wp), dimension(:,:), optional, target, intent(in) :: lw_Ds   ! (ncol, ngpt) extents, read as (ngpt, ncol): B-12
    real(wp), dimension(:,:), target, optional, intent(inout) :: flux_up_Jac, flux_dn_Jac
    character(len=128) :: error_msg
    integer :: ncol, nlay, ngpt, nband, nmus
    integer(c_long_long) :: ng, nv, nsfc, ngv
    integer(c_int), allocatable :: lims(:,:)
    type(c_ptr) :: d_tau, d_ssa, d_g, d_lay, d_lev, d_sfc, d_jac, d_emis, d_emis_gpt, d_inc, d_up, d_dn
    type(c_ptr) :: d_ds, d_gup, d_gdn
    logical :: two_str, use_2s, src_tmp, g_tmp, gpt, du, dd
    real(wp), allocatable :: up(:,:), dn(:,:)

    ncol  = optical_props%get_ncol()
    nlay  = optical_props%get_nlay()
    ngpt  = optical_props%get_ngpt()
    nband = optical_props%get_nband()
    error_msg = ""
    if (.not. fluxes%are_desired()) then
      error_msg = "rte_lw: no space allocated for fluxes"; return
    end if
    error_msg = fluxes%check_extents(nlay + 1, ncol)
    if (error_msg /= '') return
    if (any([sources%get_ncol(), sources%get_nlay(), sources%get_ngpt()] /= [ncol, nlay, ngpt])) then
      error_msg = "rte_lw: sources and optical properties inconsistently sized"; return
    end if
    if (any(shape(sfc_emis) /= [nband, ncol])) then
      error_msg = "rte_lw: sfc_emis inconsistently sized"; return
    end if
    if (check_values) then
      if (any(sfc_emis < 0._wp .or. sfc_emis > 1._wp)) then
        error_msg = "rte_lw: sfc_emis has values < 0 or > 1"; return
      end if
    end if
    if (present(inc_flux)) then
      if (any(shape(inc_flux) /= [ngpt, ncol])) then
        error_msg = "rte_lw: inc_flux inconsistently sized"; return
      end if
      if (check_values) then
        if (any(inc_flux < 0._wp)) then
          error_msg = "rte_lw: inc_flux has values < 0"; return
        end if
      end if
    end if
    nmus = 1
    if (present(n_gauss_angles)) then
      if (n_gauss_angles > max_gauss_pts) then
        error_msg = "rte_lw: asking for too many quadrature points for no-scattering calculation"; return
      end if
      if (n_gauss_angles < 1) then
        error_msg = "rte_lw: have to ask for at least one quadrature point for no-scattering calculation"; return
      end if
      nmus = n_gauss_angles
    end if
    ! flux_up_Jac / flux_dn_Jac: accepted and left untouched, as in the reference, where compute_Jac is a .false.
    ! parameter (mo_rte_rrtmgp_config.F90:28): no extent check (:160-163), no write; rejected only with use_2stream
    ! on 2str properties (:252-253, below).
    if (associated(fluxes%gpt_flux_up)) then
      if (any(shape(fluxes%gpt_flux_up) /= [ngpt, nlay + 1, ncol])) then
        error_msg = "rte_lw: gpt_flux_up inconsistently sized"; return
      end if
    end if
    if (associated(fluxes%gpt_flux_dn)) then
      if (any(shape(fluxes%gpt_flux_dn) /= [ngpt, nlay + 1, ncol])) then
        error_msg = "rte_lw: gpt_flux_dn inconsistently sized"; return
      end if
    end if
    use_2s = .false.
    if (present(use_2stream)) use_2s = use_2stream
    two_str = .false.
    d_ssa = c_null_ptr
    d_g = c_null_ptr
    select type (optical_props)
    type is (ty_optical_props_1scl)
      if (use_2s) then
        error_msg = "rte_lw: can't use two-stream methods with only absorption optical depth"; return
      end if
      if (present(lw_Ds)) then  ! (:239-246)
        if (any(shape(lw_Ds) /= [ncol, ngpt])) then
          error_msg = "rte_lw: lw_Ds inconsistently sized"; return
        end if
        if (any(lw_Ds < 1._wp)) then
          error_msg = "rte_lw: one or more values of lw_Ds < 1."; return
        end if
        if (nmus /= 1) then
          error_msg = "rte_lw: providing lw_Ds incompatible with specifying n_gauss_angles"; return
        end if
      end if
    type is (ty_optical_props_2str)
      ! (:248-253) each check overwrites error_msg, so the last failing one is returned; the Jacobian check tests
      ! flux_up_Jac twice (`present(flux_up_Jac) .or. present(flux_up_Jac)`), so a lone flux_dn_Jac passes there too
      if (present(lw_Ds)) error_msg = "rte_lw: lw_Ds not valid input for _2str class"
      if (use_2s .and. nmus /= 1) &
        error_msg = "rte_lw: using_2stream=true incompatible with specifying n_gauss_angles"
      if (use_2s .and. present(flux_up_Jac)) &
        error_msg = "rte_lw: can't provide Jacobian of fluxes w.r.t surface temperature with 2-stream"
      if (error_msg /= '') return
      if (use_2s .or. check_values) error_msg = optical_props%validate()  ! unconditional for 2-stream (:360)
      if (error_msg /= '') return
      two_str = .true.
    class default
      error_msg = "lw_solver(...ty_optical_props_nstr...) not yet implemented"; return
    end select

    lims = optical_props%get_band_lims_gpoint()
    ng = int(ngpt, c_long_long) * nlay * ncol
    nv = int(nlay + 1, c_long_long) * ncol
    nsfc = int(ngpt, c_long_long) * ncol
    d_tau = dev_present(optical_props%tau, ng, PRESENT_READ)
    d_emis = dev_stage(sfc_emis, int(nband, c_long_long) * ncol)
    d_inc = c_null_ptr
    if (present(inc_flux)) d_inc = dev_stage(inc_flux, nsfc)
    d_up = dev_scratch(nv)
    d_dn = dev_scratch(nv)
    ! ty_fluxes_flexible g-point outputs and lw_Ds: the *_gpt entries (NULL outputs: the plain solvers)
    gpt = fluxes%are_desired_gpt()
    ngv = int(ngpt, c_long_long) * (nlay + 1) * ncol
    d_ds = c_null_ptr
    d_gup = c_null_ptr
    d_gdn = c_null_ptr
    if (present(lw_Ds)) d_ds = dev_stage(lw_Ds, nsfc)
    if (gpt) then
      d_gup = dev_scratch(ngv)
      d_gdn = dev_scratch(ngv)
    end if
    d_emis_gpt = c_null_ptr
    if (.not. two_str .and. sources%planck_deferred) then
      ! lw_solver_noscat_GaussQuad (:326-353) with compute_Planck_source_nn (gas_optics, :398-404) and expand(sfc_emis)
      ! (:429-447) inside the solver
      error_msg = rrtmgpnn_check(c_rrtmgpnn_lw_solver_noscat_planck_gpt(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                    merge(1_c_int, 0_c_int, top_at_1), nmus, gauss_Ds(1:nmus, nmus), gauss_wts(1:nmus, nmus), d_ds, &
                    d_inc, d_tau, dev_present(sources%lay_source, ng, PRESENT_READ), nband, sources%pk_ntemp, &
                    dev_present(sources%pk_tlay, size(sources%pk_tlay, kind=c_long_long), PRESENT_READ), &
                    dev_present(sources%pk_tlev, size(sources%pk_tlev, kind=c_long_long), PRESENT_READ), &
                    dev_present(sources%pk_tsfc, size(sources%pk_tsfc, kind=c_long_long), PRESENT_READ), &
                    sources%pk_sfc_lay, lims, sources%pk_tmin, sources%pk_tdelta, sources%pk_totplnk, 1_c_int, d_emis, &
                    d_up, d_dn, d_gup, d_gdn), "rte_lw: lw_solver_noscat")
    else
      src_tmp = .false.
      g_tmp = .false.
      error_msg = sources%device_sources(d_lay, d_lev, d_sfc, d_jac, src_tmp)
      if (error_msg == '') then
        d_emis_gpt = dev_scratch(nsfc)
        ! sfc_emis expanded to g-points (:429-447), then the solver (:326-387)
        error_msg = rrtmgpnn_check(c_rrtmgpnn_expand_band_to_gpt(rrtmgpnn_ctx(), nband, ngpt, ncol, lims, d_emis, &
                                                                 d_emis_gpt), "rte_lw: expand")
      end if
      if (error_msg == '') then
        select type (optical_props)
        type is (ty_optical_props_2str)
          d_ssa = dev_present(optical_props%ssa, ng, PRESENT_READ)
          d_g = dev_g_read(optical_props, g_tmp)
        end select
        if (two_str .and. use_2s) then
          error_msg = rrtmgpnn_check(c_rrtmgpnn_lw_solver_2stream_gpt(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                                     merge(1_c_int, 0_c_int, top_at_1), d_inc, d_tau, d_ssa, d_g, d_lev, d_emis_gpt, &
                                     d_sfc, d_up, d_dn, d_gup, d_gdn), "rte_lw: lw_solver_2stream")
        else if (two_str) then
          error_msg = rrtmgpnn_check(c_rrtmgpnn_lw_solver_1rescl_gpt(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                                     merge(1_c_int, 0_c_int, top_at_1), nmus, gauss_Ds(1:nmus, nmus), &
                                     gauss_wts(1:nmus, nmus), d_inc, d_tau, d_ssa, d_g, d_lay, d_lev, d_emis_gpt, &
                                     d_sfc, d_up, d_dn, d_gup, d_gdn), "rte_lw: lw_solver_noscat (rescaled)")
        else
          error_msg = rrtmgpnn_check(c_rrtmgpnn_lw_solver_noscat_gpt(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                                     merge(1_c_int, 0_c_int, top_at_1), nmus, gauss_Ds(1:nmus, nmus), &
                                     gauss_wts(1:nmus, nmus), d_ds, d_inc, d_tau, d_lay, d_lev, d_emis_gpt, d_sfc, &
                                     d_up, d_dn, d_gup, d_gdn), "rte_lw: lw_solver_noscat")
        end if
      end if
      if (src_tmp) then
        call dev_release(d_lay); call dev_release(d_lev); call dev_release(d_sfc); call dev_release(d_jac)
      end if
      if (g_tmp) call dev_release(d_g)
    end if
    ! broadband fluxes go straight into the caller's arrays when they are contiguous (and no net flux is wanted from
    ! them); otherwise into temporaries copied after the sync
    du = .false.; dd = .false.
    if (.not. associated(fluxes%flux_net)) then
      du = direct_ok(fluxes%flux_up, nv); dd = direct_ok(fluxes%flux_dn, nv)
    end if
    allocate(up(nlay + 1, ncol), dn(nlay + 1, ncol))
    if (error_msg == '') then
      if (du) then
        call dev_copy_out(fluxes%flux_up, d_up, nv)
      else
        call dev_copy_out(up, d_up, nv)
      end if
      if (dd) then
        call dev_copy_out(fluxes%flux_dn, d_dn, nv)
      else
        call dev_copy_out(dn, d_dn, nv)
      end if
      if (gpt) then
        if (associated(fluxes%gpt_flux_up)) call dev_copy_out(fluxes%gpt_flux_up, d_gup, ngv)
        if (associated(fluxes%gpt_flux_dn)) call dev_copy_out(fluxes%gpt_flux_dn, d_gdn, ngv)
      end if
    end if
    call rrtmgpnn_sync(error_msg, "rte_lw")
    if (error_msg == '') then
      if (associated(fluxes%flux_up) .and. .not. du) fluxes%flux_up = up
      if (associated(fluxes%flux_dn) .and. .not. dd) fluxes%flux_dn = dn
      if (associated(fluxes%flux_net)) fluxes%flux_net = dn - up
    end if
    call dev_release(d_emis); call dev_release(d_emis_gpt); call dev_release(d_inc)
    call dev_release(d_up); call dev_release(d_dn)
    call dev_release(d_ds); call dev_release(d_gup); call dev_release(d_gdn)
  end function rte_lw

  ! whether the device fluxes can be copied into f itself: associated, contiguous and n elements (the extents were
  ! checked on entry, fluxes%check_extents)
  logical function direct_ok(f, n)
    real(wp), dimension(:,:), pointer, intent(in) :: f
    integer(c_long_long), intent(in) :: n
    direct_ok = .false.
    if (associated(f)) direct_ok = is_contiguous(f) .and. size(f, kind=c_long_long) == n
  end function direct_ok
end module mo_rte_lw
