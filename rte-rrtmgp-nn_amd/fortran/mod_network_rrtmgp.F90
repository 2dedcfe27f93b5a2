! mod_network_rrtmgp -- drop-in for the reference module of the same name (neural/mod_network_rrtmgp.F90).
! rrtmgp_network_type keeps the public components the drivers read (layers(:)%w_transposed, layers(:)%b,
! input_names, coeffs_input_min/max, coeffs_output_mean/std) and `load_netcdf(filename)`; the model is
! uploaded once to the device (MFMA-packed weight image) and evaluated by the fused HIP MLP kernels.
! netcdf-fortran is absent in this image, so `load_netcdf` reads the RBIN conversion of the model
! (tools/convert_reference_data.py); the file layout of every variable is unchanged.
module mod_network_rrtmgp
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,      only: sp
  use mo_rrtmgpnn_c,    only: rrtmgpnn_ctx, c_rrtmgpnn_network_load, rrtmgpnn_error_message
  use mo_rrtmgpnn_rbin, only: rbin_real1, rbin_real2, rbin_int1, rbin_strings
  implicit none
  private
  public :: rrtmgp_network_type, layer_type

  type :: layer_type
    real(sp), allocatable :: b(:)
    real(sp), allocatable :: w(:,:)             ! (n_in, n_out)
    real(sp), allocatable :: w_transposed(:,:)  ! (n_out, n_in)
  end type layer_type

  type :: rrtmgp_network_type
    type(layer_type), allocatable :: layers(:)
    integer, allocatable :: dims(:)
    real(sp),      dimension(:), allocatable :: coeffs_input_min, coeffs_input_max
    real(sp),      dimension(:), allocatable :: coeffs_output_mean, coeffs_output_std
    character(32), dimension(:), allocatable :: input_names
    type(c_ptr) :: handle = c_null_ptr           ! rrtmgpnn_network (device resident)
  contains
    procedure, public :: load_netcdf
  end type rrtmgp_network_type

contains

  subroutine load_netcdf(self, filename)
    class(rrtmgp_network_type), intent(inout) :: self
    character(len=*), intent(in) :: filename
    character(len=128) :: err
    integer :: n, nl
    real(sp), allocatable :: wflat(:,:)
    integer(c_int) :: rc
    character(len=8) :: cn
    call rbin_int1(filename, "dims", self%dims, err)
    if (err /= '') call fail(err)
    nl = size(self%dims) - 1
    allocate(self%layers(nl))
    do n = 1, nl
      write(cn, '(i0)') n
      call rbin_real2(filename, "w" // trim(cn), wflat, err)  ! C (n_in,n_out) -> Fortran (n_out,n_in)
      if (err /= '') call fail(err)
      self%layers(n)%w_transposed = wflat
      self%layers(n)%w = transpose(wflat)
      call rbin_real1(filename, "b" // trim(cn), self%layers(n)%b, err)
      if (err /= '') call fail(err)
    end do
    call rbin_real1(filename, "input_min", self%coeffs_input_min, err)
    call rbin_real1(filename, "input_max", self%coeffs_input_max, err)
    call rbin_strings(filename, "input_names", self%input_names, err)
    call rbin_real1(filename, "output_mean", self%coeffs_output_mean, err)
    if (err /= '' .and. allocated(self%coeffs_output_mean)) deallocate(self%coeffs_output_mean)
    call rbin_real1(filename, "output_std", self%coeffs_output_std, err)
    if (err /= '' .and. allocated(self%coeffs_output_std)) deallocate(self%coeffs_output_std)
    rc = c_rrtmgpnn_network_load(rrtmgpnn_ctx(), trim(filename) // c_null_char, self%handle)
    if (rc /= 0) call fail("mod_network_rrtmgp:load_netcdf: " // trim(rrtmgpnn_error_message()))
  contains
    subroutine fail(msg)
      character(len=*), intent(in) :: msg
      write(*, '(a)') "mod_network_rrtmgp:load_netcdf: " // trim(msg)
      error stop 1
    end subroutine fail
  end subroutine load_netcdf
end module mod_network_rrtmgp
