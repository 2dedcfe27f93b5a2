! mo_heating_rates -- drop-in for extensions/mo_heating_rates.F90 (compute_heating_rate, :26-53): layer heating
! rate [K/s] = (up(l+1) - up(l) - dn(l+1) + dn(l)) * grav / (cp_dry * (p(l+1) - p(l))), evaluated by one HIP kernel
! (rrtmgpnn_compute_heating_rate) with grav and cp_dry of rrtmgp/mo_rrtmgp_constants.F90:50,53.
! The reference extension predates this fork's flux layout; here the arrays are the fork's: fluxes and plev
! (nlay+1, ncol), heating_rate (nlay, ncol), so the rte_lw / rte_sw outputs go in as they come out.
module mo_heating_rates
  use, intrinsic :: iso_c_binding
  use mo_rte_kind, only: wp
  use mo_rrtmgpnn_c
  implicit none
  private
  public :: compute_heating_rate
contains
  function compute_heating_rate(flux_up, flux_dn, plev, heating_rate) result(error_msg)
    real(wp), dimension(:,:), intent(in ) :: flux_up, flux_dn, plev   ! (nlay+1, ncol) [W/m2], [Pa]
    real(wp), dimension(:,:), intent(out) :: heating_rate             ! (nlay, ncol) [K/s]
    character(len=128) :: error_msg
    integer :: ncol, nlay
    integer(c_long_long) :: nv
    type(c_ptr) :: d_up, d_dn, d_p, d_hr

    error_msg = ""
    nlay = size(flux_up, 1) - 1
    ncol = size(flux_up, 2)
    if (any(shape(flux_dn) /= [nlay + 1, ncol])) then
      error_msg = "heating_rate: flux_dn array inconsistently sized."; return
    end if
    if (any(shape(plev) /= [nlay + 1, ncol])) then
      error_msg = "heating_rate: plev array inconsistently sized."; return
    end if
    if (any(shape(heating_rate) /= [nlay, ncol])) then
      error_msg = "heating_rate: heating_rate array inconsistently sized."; return
    end if
    nv = int(nlay + 1, c_long_long) * ncol
    d_up = dev_stage(flux_up, nv)
    d_dn = dev_stage(flux_dn, nv)
    d_p  = dev_stage(plev, nv)
    d_hr = dev_scratch(int(nlay, c_long_long) * ncol)
    error_msg = rrtmgpnn_check(c_rrtmgpnn_compute_heating_rate(rrtmgpnn_ctx(), ncol, nlay, d_up, d_dn, d_p, d_hr), &
                               "heating_rate")
    if (error_msg == '') call dev_copy_out(heating_rate, d_hr, int(nlay, c_long_long) * ncol)
    call rrtmgpnn_sync(error_msg, "heating_rate")
    call dev_release(d_up); call dev_release(d_dn); call dev_release(d_p); call dev_release(d_hr)
  end function compute_heating_rate
end module mo_heating_rates
