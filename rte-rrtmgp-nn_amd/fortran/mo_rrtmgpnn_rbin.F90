! mo_rrtmgpnn_rbin.F90 -- Fortran reader of RBIN files (format: rte-rrtmgp-nn_amd/rrtmgpnn/rbin.py), the
! framework's replacement for the netCDF files the reference reads through netcdf-fortran (absent here):
! NN models (neural/mod_network_rrtmgp.F90:58-122) and RFMIP inputs (examples/rfmip-clear-sky/mo_rfmip_io.F90).
! Arrays are stored C-order with shape (d1,...,dn); read into Fortran arrays of shape (dn,...,d1), i.e. the
! same memory, which is the reference's own (column-major) layout.
module mo_rrtmgpnn_rbin
  use, intrinsic :: iso_c_binding, only: c_float, c_int32_t, c_int8_t
  implicit none
  private
  public :: rbin_find, rbin_real, rbin_real1, rbin_real2, rbin_real3, rbin_int1, rbin_int2, rbin_strings
  public :: rbin_write_begin, rbin_write_real, rbin_write_end

contains

  ! Locate entry `name`: returns the stream position of its payload (0 if absent), dtype, ndim, dims (C order).
  subroutine rbin_find(filename, name, pos, dtype, ndim, dims)
    character(len=*), intent(in) :: filename, name
    integer(8), intent(out) :: pos
    integer, intent(out) :: dtype, ndim, dims(8)
    integer :: u, ios, ver, cnt, e, dt, nd, k, isz
    integer(c_int32_t) :: i4, d4(8)
    character(len=4) :: magic
    character(len=64) :: ename
    integer(8) :: p, n
    pos = 0; dtype = -1; ndim = 0; dims = 0
    open(newunit=u, file=filename, access='stream', form='unformatted', status='old', action='read', iostat=ios)
    if (ios /= 0) return
    read(u) magic
    read(u) i4; ver = i4
    read(u) i4; cnt = i4
    if (magic /= 'RBIN' .or. ver /= 1) then
      close(u); return
    end if
    p = 13
    do e = 1, cnt
      read(u, pos=p) ename
      read(u) i4; dt = i4
      read(u) i4; nd = i4
      d4 = 0
      if (nd > 0) read(u) d4(1:nd)
      p = p + 64 + 8 + 4 * nd
      n = 1
      do k = 1, nd
        n = n * d4(k)
      end do
      isz = merge(1, 4, dt == 2)
      k = index(ename, char(0))
      if (k == 0) k = 65
      if (ename(1:k-1) == name) then
        pos = p; dtype = dt; ndim = nd; dims(1:nd) = int(d4(1:nd))
        close(u); return
      end if
      p = p + n * isz
    end do
    close(u)
  end subroutine rbin_find

  subroutine rbin_real(filename, name, buf, n, ok)
    character(len=*), intent(in) :: filename, name
    integer, intent(in) :: n
    real(c_float), intent(out) :: buf(n)
    logical, intent(out) :: ok
    integer(8) :: pos
    integer :: dt, nd, dims(8), u
    call rbin_find(filename, name, pos, dt, nd, dims)
    if (pos == 0 .or. dt /= 0) then
      ok = .false.; return
    end if
    open(newunit=u, file=filename, access='stream', form='unformatted', status='old', action='read')
    read(u, pos=pos) buf
    close(u)
    ok = .true.
  end subroutine rbin_real

  function entry_size(filename, name, want_dt, nd_out, dims_out) result(n)
    character(len=*), intent(in) :: filename, name
    integer, intent(in) :: want_dt
    integer, intent(out) :: nd_out, dims_out(8)
    integer :: n, dt
    integer(8) :: pos
    call rbin_find(filename, name, pos, dt, nd_out, dims_out)
    n = -1
    if (pos == 0 .or. dt /= want_dt) return
    n = product(dims_out(1:nd_out))
  end function entry_size

  subroutine rbin_real1(filename, name, a, error_msg)
    character(len=*), intent(in) :: filename, name
    real(c_float), allocatable, intent(out) :: a(:)
    character(len=128), intent(out) :: error_msg
    integer :: n, nd, dims(8)
    logical :: ok
    error_msg = ''
    n = entry_size(filename, name, 0, nd, dims)
    if (n < 0) then
      error_msg = "rbin: " // trim(name) // " missing in " // trim(filename); return
    end if
    allocate(a(n))
    call rbin_real(filename, name, a, n, ok)
  end subroutine rbin_real1

  subroutine rbin_real2(filename, name, a, error_msg)
    character(len=*), intent(in) :: filename, name
    real(c_float), allocatable, intent(out) :: a(:,:)
    character(len=128), intent(out) :: error_msg
    integer :: n, nd, dims(8)
    logical :: ok
    error_msg = ''
    n = entry_size(filename, name, 0, nd, dims)
    if (n < 0 .or. nd /= 2) then
      error_msg = "rbin: 2-D " // trim(name) // " missing in " // trim(filename); return
    end if
    allocate(a(dims(2), dims(1)))
    call rbin_real(filename, name, a, n, ok)
  end subroutine rbin_real2

  subroutine rbin_real3(filename, name, a, error_msg)
    character(len=*), intent(in) :: filename, name
    real(c_float), allocatable, intent(out) :: a(:,:,:)
    character(len=128), intent(out) :: error_msg
    integer :: n, nd, dims(8)
    logical :: ok
    error_msg = ''
    n = entry_size(filename, name, 0, nd, dims)
    if (n < 0 .or. nd /= 3) then
      error_msg = "rbin: 3-D " // trim(name) // " missing in " // trim(filename); return
    end if
    allocate(a(dims(3), dims(2), dims(1)))
    call rbin_real(filename, name, a, n, ok)
  end subroutine rbin_real3

  subroutine rbin_int1(filename, name, a, error_msg)
    character(len=*), intent(in) :: filename, name
    integer, allocatable, intent(out) :: a(:)
    character(len=128), intent(out) :: error_msg
    integer :: n, nd, dims(8), u
    integer(8) :: pos
    integer(c_int32_t), allocatable :: b(:)
    integer :: dt
    error_msg = ''
    n = entry_size(filename, name, 1, nd, dims)
    if (n < 0) then
      error_msg = "rbin: " // trim(name) // " missing in " // trim(filename); return
    end if
    call rbin_find(filename, name, pos, dt, nd, dims)
    allocate(b(n), a(n))
    open(newunit=u, file=filename, access='stream', form='unformatted', status='old', action='read')
    read(u, pos=pos) b
    close(u)
    a = int(b)
  end subroutine rbin_int1

  subroutine rbin_int2(filename, name, a, error_msg)
    character(len=*), intent(in) :: filename, name
    integer, allocatable, intent(out) :: a(:,:)
    character(len=128), intent(out) :: error_msg
    integer, allocatable :: flat(:)
    integer :: nd, dims(8), n
    error_msg = ''
    n = entry_size(filename, name, 1, nd, dims)
    if (n < 0 .or. nd /= 2) then
      error_msg = "rbin: 2-D " // trim(name) // " missing in " // trim(filename); return
    end if
    call rbin_int1(filename, name, flat, error_msg)
    allocate(a(dims(2), dims(1)))
    a = reshape(flat, [dims(2), dims(1)])
  end subroutine rbin_int2

  ! Character array stored (n, width) uint8, space padded -> strings(n)
  subroutine rbin_strings(filename, name, strings, error_msg)
    character(len=*), intent(in) :: filename, name
    character(len=32), allocatable, intent(out) :: strings(:)
    character(len=128), intent(out) :: error_msg
    integer :: nd, dims(8), n, u, i, dt
    integer(8) :: pos
    character(len=:), allocatable :: raw
    error_msg = ''
    n = entry_size(filename, name, 2, nd, dims)
    if (n < 0 .or. nd /= 2) then
      error_msg = "rbin: strings " // trim(name) // " missing in " // trim(filename); return
    end if
    call rbin_find(filename, name, pos, dt, nd, dims)
    allocate(character(len=n) :: raw)
    open(newunit=u, file=filename, access='stream', form='unformatted', status='old', action='read')
    read(u, pos=pos) raw
    close(u)
    allocate(strings(dims(1)))
    do i = 1, dims(1)
      strings(i) = raw((i-1)*dims(2)+1 : (i-1)*dims(2)+min(dims(2), 32))
    end do
  end subroutine rbin_strings

  ! Writer: rbin_write_begin(file, count) -> unit; `count` rbin_write_real calls; rbin_write_end(unit).
  function rbin_write_begin(filename, count) result(u)
    character(len=*), intent(in) :: filename
    integer, intent(in) :: count
    integer :: u
    open(newunit=u, file=filename, access='stream', form='unformatted', status='replace', action='write')
    write(u) 'RBIN', int(1, c_int32_t), int(count, c_int32_t)
  end function rbin_write_begin

  ! Fortran array of shape fshape(1:nd) (any rank, sequence-associated) stored as C-order reversed dims.
  subroutine rbin_write_real(u, name, a, fshape)
    integer, intent(in) :: u
    character(len=*), intent(in) :: name
    integer, dimension(:), intent(in) :: fshape
    real(c_float), dimension(product(fshape)), intent(in) :: a
    character(len=64) :: ename
    integer :: k, nd
    nd = size(fshape)
    ename = repeat(char(0), 64)
    ename(1:len_trim(name)) = trim(name)
    write(u) ename, int(0, c_int32_t), int(nd, c_int32_t)
    write(u) (int(fshape(nd + 1 - k), c_int32_t), k = 1, nd)
    write(u) a
  end subroutine rbin_write_real

  subroutine rbin_write_end(u)
    integer, intent(in) :: u
    close(u)
  end subroutine rbin_write_end
end module mo_rrtmgpnn_rbin
