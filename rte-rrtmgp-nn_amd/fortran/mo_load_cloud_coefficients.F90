! mo_load_cloud_coefficients -- drop-in for examples/all-sky/mo_load_cloud_coefficients.F90: load_cld_lutcoeff
! and load_cld_padecoeff fill a ty_cloud_optics from rrtmgp-cloud-optics-coeffs-{lw,sw}.nc.  The file is read by
! the library's native classic-netCDF reader (netcdf-fortran is absent here) instead of nf90 calls; errors stop
! the program, as the reference's stop_on_err does.
module mo_load_cloud_coefficients
  use mo_cloud_optics, only: ty_cloud_optics
  implicit none
  private
  public :: load_cld_lutcoeff, load_cld_padecoeff

contains

  subroutine load_cld_lutcoeff(cloud_spec, cld_coeff_file)
    class(ty_cloud_optics), intent(inout) :: cloud_spec
    character(len=*),       intent(in)    :: cld_coeff_file
    call stop_on_err(cloud_spec%load_rbin(cld_coeff_file, .true.))
  end subroutine load_cld_lutcoeff

  subroutine load_cld_padecoeff(cloud_spec, cld_coeff_file)
    class(ty_cloud_optics), intent(inout) :: cloud_spec
    character(len=*),       intent(in)    :: cld_coeff_file
    call stop_on_err(cloud_spec%load_rbin(cld_coeff_file, .false.))
  end subroutine load_cld_padecoeff

  subroutine stop_on_err(msg)
    character(len=*), intent(in) :: msg
    if (len_trim(msg) > 0) then
      write(*, '(a)') trim(msg)
      error stop 1
    end if
  end subroutine stop_on_err
end module mo_load_cloud_coefficients
