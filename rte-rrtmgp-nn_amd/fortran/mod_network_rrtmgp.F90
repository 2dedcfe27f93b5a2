! mod_network_rrtmgp -- drop-in for the reference module of the same name (neural/mod_network_rrtmgp.F90).
! rrtmgp_network_type keeps the public components the drivers read (layers(:)%w_transposed, layers(:)%b,
! input_names, coeffs_input_min/max, coeffs_output_mean/std) and `load_netcdf(filename)`; the model is
! uploaded once to the device (MFMA-packed weight image) and evaluated by the fused HIP MLP kernels.
! `load_netcdf` reads the reference's netCDF model file with the library's native reader (netcdf-fortran is
! absent in this image), or the RBIN conversion of it (tools/convert_reference_data.py).
module mod_network_rrtmgp
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,      only: sp
  use mo_rrtmgpnn_c,    only: rrtmgpnn_ctx, c_rrtmgpnn_network_load, rrtmgpnn_error_message
  use mo_rrtmgpnn_file, only: ty_data_file
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

  ! load_netcdf (neural/mod_network_rrtmgp.F90:58-122): the reference's netCDF model file, read natively
  ! (mo_rrtmgpnn_file), or its RBIN conversion; both hold the same arrays.
  subroutine load_netcdf(self, filename)
    class(rrtmgp_network_type), intent(inout) :: self
    character(len=*), intent(in) :: filename
    type(ty_data_file) :: f
    character(len=128) :: err
    integer :: n, nl
    real(sp), allocatable :: wflat(:,:), mn(:)
    integer(c_int), allocatable :: hidden(:)
    integer(c_int) :: rc
    logical :: nc
    character(len=8) :: cn
    err = f%open(filename)
    if (err /= '') call fail(err)
    nc = f%has("nn_dimsize")
    if (nc) then
      call check(f%int1("nn_dimsize", hidden))
      call check(f%real1("nn_input_coeffs_min", mn))
      self%dims = [size(mn), int(hidden)]                  ! nn_dim_input, nn_dimsize
    else
      call check(f%int1("dims", hidden))
      self%dims = int(hidden)
    end if
    nl = size(self%dims) - 1
    if (allocated(self%layers)) deallocate(self%layers)
    allocate(self%layers(nl))
    do n = 1, nl
      write(cn, '(i0)') n
      ! file (n_in, n_out) C order = Fortran (n_out, n_in): w_transposed as is, w its transpose (:92-95)
      call check(f%real2(pick("nn_weights_" // trim(cn), "w" // trim(cn)), wflat))
      self%layers(n)%w_transposed = wflat
      self%layers(n)%w = transpose(wflat)
      call check(f%real1(pick("nn_bias_" // trim(cn), "b" // trim(cn)), self%layers(n)%b))
    end do
    call check(f%real1(pick("nn_input_coeffs_min", "input_min"), self%coeffs_input_min))
    call check(f%real1(pick("nn_input_coeffs_max", "input_max"), self%coeffs_input_max))
    if (f%has(pick("nn_inputs_char", "input_names"))) &
      call check(f%strings(pick("nn_inputs_char", "input_names"), self%input_names))
    if (f%has(pick("nn_output_coeffs_mean", "output_mean"))) then
      call check(f%real1(pick("nn_output_coeffs_mean", "output_mean"), self%coeffs_output_mean))
      call check(f%real1(pick("nn_output_coeffs_std", "output_std"), self%coeffs_output_std))
    end if
    call f%close()
    rc = c_rrtmgpnn_network_load(rrtmgpnn_ctx(), trim(filename) // c_null_char, self%handle)
    if (rc /= 0) call fail(trim(rrtmgpnn_error_message()))
  contains
    ! the netCDF variable name, or the RBIN conversion's
    function pick(nc_name, rbin_name) result(name)
      character(len=*), intent(in) :: nc_name, rbin_name
      character(len=:), allocatable :: name
      if (nc) then
        name = nc_name
      else
        name = rbin_name
      end if
    end function pick
    subroutine check(msg)
      character(len=*), intent(in) :: msg
      if (msg /= '') call fail(msg)
    end subroutine check
    subroutine fail(msg)
      character(len=*), intent(in) :: msg
      write(*, '(a)') "mod_network_rrtmgp:load_netcdf: " // trim(msg)
      error stop 1
    end subroutine fail
  end subroutine load_netcdf
end module mod_network_rrtmgp
