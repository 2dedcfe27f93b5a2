! mo_rte_sw -- drop-in for rte/mo_rte_sw.F90 (rte_sw, :48-266; the fork passes surface albedos per
! g-point).  The two-stream solver (sw_solver_2stream, rte/kernels/mo_rte_solver_kernels.F90:541-692)
! runs as one HIP kernel per call with the broadband reduction fused in; the no-scattering (1scl)
! shortwave path and g-point fluxes return an error string.
module mo_rte_sw
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,      only: wp
  use mo_optical_props, only: ty_optical_props_arry, ty_optical_props_2str
  use mo_fluxes,        only: ty_fluxes_flexible
  use mo_rte_rrtmgp_config, only: check_values
  use mo_rrtmgpnn_c
  implicit none
  private
  public :: rte_sw

contains

  function rte_sw(atmos, top_at_1, mu0, inc_flux, sfc_alb_dir_gpt, sfc_alb_dif_gpt, fluxes, inc_flux_dif) &
      result(error_msg)
    class(ty_optical_props_arry), intent(in) :: atmos
    logical,                      intent(in) :: top_at_1
    real(wp), dimension(:),       intent(in) :: mu0                 ! (ncol)
    real(wp), dimension(:,:),     intent(in) :: inc_flux, sfc_alb_dir_gpt, sfc_alb_dif_gpt   ! (ngpt, ncol)
    class(ty_fluxes_flexible), intent(inout) :: fluxes
    real(wp), dimension(:,:), optional, contiguous, target, intent(in) :: inc_flux_dif      ! (ngpt, ncol)
    character(len=128) :: error_msg
    integer :: ncol, nlay, ngpt
    type(c_ptr) :: d_tau, d_ssa, d_g, d_mu0, d_inc, d_dif, d_adir, d_adif, d_up, d_dn, d_dir
    real(wp), allocatable :: up(:,:), dn(:,:), dir(:,:)
    character(len=128) :: e

    ncol = atmos%get_ncol()
    nlay = atmos%get_nlay()
    ngpt = atmos%get_ngpt()
    error_msg = ""
    if (.not. fluxes%are_desired()) then
      error_msg = "rte_sw: no space allocated for fluxes"; return
    end if
    if (fluxes%are_desired_gpt()) then
      error_msg = "rte_sw: g-point fluxes are not produced by this build (broadband only)"; return
    end if
    if (size(mu0) /= ncol) then
      error_msg = "rte_sw: mu0 inconsistently sized"; return
    end if
    if (check_values .and. any(mu0 < 0._wp .or. mu0 > 1._wp)) then
      error_msg = "rte_sw: one or more mu0 <= 0 or > 1"; return
    end if
    if (any(shape(inc_flux) /= [ngpt, ncol])) then
      error_msg = "rte_sw: inc_flux inconsistently sized"; return
    end if
    if (check_values .and. any(inc_flux < 0._wp)) then
      error_msg = "rte_sw: one or more inc_flux < 0"; return
    end if
    if (present(inc_flux_dif)) then
      if (any(shape(inc_flux_dif) /= [ngpt, ncol])) then
        error_msg = "rte_sw: inc_flux_dif inconsistently sized"; return
      end if
      if (check_values .and. any(inc_flux_dif < 0._wp)) then
        error_msg = "rte_sw: one or more inc_flux_dif < 0"; return
      end if
    end if
    if (any(shape(sfc_alb_dir_gpt) /= [ngpt, ncol])) then
      error_msg = "rte_sw: sfc_alb_dir inconsistently sized"; return
    end if
    if (check_values .and. any(sfc_alb_dir_gpt < 0._wp .or. sfc_alb_dir_gpt > 1._wp)) then
      error_msg = "rte_sw: sfc_alb_dir out of bounds [0,1]"; return
    end if
    if (any(shape(sfc_alb_dif_gpt) /= [ngpt, ncol])) then
      error_msg = "rte_sw: sfc_alb_dif inconsistently sized"; return
    end if
    if (check_values .and. any(sfc_alb_dif_gpt < 0._wp .or. sfc_alb_dif_gpt > 1._wp)) then
      error_msg = "rte_sw: sfc_alb_dif out of bounds [0,1]"; return
    end if

    select type (atmos)
    class is (ty_optical_props_2str)
      d_tau = dev_upload(atmos%tau, ngpt * nlay * ncol)
      d_ssa = dev_upload(atmos%ssa, ngpt * nlay * ncol)
      d_g   = dev_upload(atmos%g, ngpt * nlay * ncol)
    class default
      error_msg = "rte_sw: the no-scattering (1scl) shortwave solver is not implemented (2str only)"; return
    end select
    d_mu0  = dev_upload(mu0, ncol)
    d_inc  = dev_upload(inc_flux, ngpt * ncol)
    d_dif  = c_null_ptr
    if (present(inc_flux_dif)) d_dif = dev_upload(inc_flux_dif, ngpt * ncol)
    d_adir = dev_upload(sfc_alb_dir_gpt, ngpt * ncol)
    d_adif = dev_upload(sfc_alb_dif_gpt, ngpt * ncol)
    d_up  = dev_alloc((nlay + 1) * ncol)
    d_dn  = dev_alloc((nlay + 1) * ncol)
    d_dir = dev_alloc((nlay + 1) * ncol)
    error_msg = rrtmgpnn_check(c_rrtmgpnn_sw_solver_2stream(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                               merge(1_c_int, 0_c_int, top_at_1), d_inc, d_dif, d_tau, d_ssa, d_g, d_mu0, &
                               d_adir, d_adif, d_up, d_dn, d_dir), "rte_sw: sw_solver_2stream")
    e = rrtmgpnn_check(c_rrtmgpnn_context_synchronize(rrtmgpnn_ctx()), "rte_sw")
    if (error_msg == '') error_msg = e
    if (error_msg == '') then
      allocate(up(nlay + 1, ncol), dn(nlay + 1, ncol), dir(nlay + 1, ncol))
      call dev_download(up, d_up, (nlay + 1) * ncol)
      call dev_download(dn, d_dn, (nlay + 1) * ncol)
      call dev_download(dir, d_dir, (nlay + 1) * ncol)
      if (associated(fluxes%flux_up))     fluxes%flux_up = up
      if (associated(fluxes%flux_dn))     fluxes%flux_dn = dn
      if (associated(fluxes%flux_dn_dir)) fluxes%flux_dn_dir = dir
      if (associated(fluxes%flux_net))    fluxes%flux_net = dn - up
    end if
    call dev_free(d_tau); call dev_free(d_ssa); call dev_free(d_g); call dev_free(d_mu0); call dev_free(d_inc)
    call dev_free(d_dif); call dev_free(d_adir); call dev_free(d_adif)
    call dev_free(d_up); call dev_free(d_dn); call dev_free(d_dir)
  end function rte_sw
end module mo_rte_sw
