! mo_rrtmgpnn_file -- the native data-file readers of librrtmgpnn (rrtmgpnn_file_*, csrc/datafile.cpp) for the
! Fortran layer: the reference's netCDF files (classic netCDF, or netCDF-4 through the HDF5 library bound at
! run time) and the RBIN conversions, read whole on open.  Arrays come back with the file's dimensions
! reversed, i.e. in the shape netCDF-Fortran gives the reference (SURVEY.md 8(f) row f-3).
module mo_rrtmgpnn_file
  use, intrinsic :: iso_c_binding
  use mo_rrtmgpnn_c, only: rrtmgpnn_check
  implicit none
  private
  public :: ty_data_file

  type :: ty_data_file
    type(c_ptr) :: h = c_null_ptr
  contains
    procedure, public :: open => file_open
    procedure, public :: close => file_close
    procedure, public :: has
    procedure, public :: real1
    procedure, public :: real2
    procedure, public :: int1
    procedure, public :: strings
  end type ty_data_file

  interface
    integer(c_int) function c_file_open(path, f) bind(C, name="rrtmgpnn_file_open")
      import :: c_int, c_ptr, c_char
      character(kind=c_char), dimension(*), intent(in) :: path
      type(c_ptr), intent(out) :: f
    end function
    integer(c_int) function c_file_close(f) bind(C, name="rrtmgpnn_file_close")
      import :: c_int, c_ptr
      type(c_ptr), value :: f
    end function
    integer(c_int) function c_file_var(f, name, dtype, ndim, dims) bind(C, name="rrtmgpnn_file_var")
      import :: c_int, c_ptr, c_char, c_long_long
      type(c_ptr), value :: f
      character(kind=c_char), dimension(*), intent(in) :: name
      integer(c_int), intent(out) :: dtype, ndim
      integer(c_long_long), dimension(8), intent(out) :: dims
    end function
    integer(c_int) function c_file_read(f, name, dtype, out, count) bind(C, name="rrtmgpnn_file_read")
      import :: c_int, c_ptr, c_char, c_long_long
      type(c_ptr), value :: f, out
      character(kind=c_char), dimension(*), intent(in) :: name
      integer(c_int), value :: dtype
      integer(c_long_long), value :: count
    end function
  end interface

contains

  function file_open(this, path) result(error_msg)
    class(ty_data_file), intent(inout) :: this
    character(len=*), intent(in) :: path
    character(len=128) :: error_msg
    error_msg = rrtmgpnn_check(c_file_open(trim(path) // c_null_char, this%h), "file")
  end function file_open

  subroutine file_close(this)
    class(ty_data_file), intent(inout) :: this
    integer(c_int) :: rc
    if (c_associated(this%h)) rc = c_file_close(this%h)
    this%h = c_null_ptr
  end subroutine file_close

  ! dtype and the Fortran shape (file dimensions reversed) of a variable; ndim < 0 when absent
  subroutine info(this, name, dtype, ndim, shp)
    class(ty_data_file), intent(in) :: this
    character(len=*), intent(in) :: name
    integer, intent(out) :: dtype, ndim, shp(8)
    integer(c_int) :: dt, nd
    integer(c_long_long) :: dims(8)
    integer :: k
    ndim = -1
    dtype = -1
    shp = 1
    if (c_file_var(this%h, trim(name) // c_null_char, dt, nd, dims) /= 0) return
    dtype = dt
    ndim = nd
    do k = 1, nd
      shp(k) = int(dims(nd - k + 1))
    end do
  end subroutine info

  logical function has(this, name)
    class(ty_data_file), intent(in) :: this
    character(len=*), intent(in) :: name
    integer :: dt, nd, shp(8)
    call info(this, name, dt, nd, shp)
    has = nd >= 0
  end function has

  function real1(this, name, a) result(error_msg)
    class(ty_data_file), intent(in) :: this
    character(len=*), intent(in) :: name
    real(c_float), allocatable, target, intent(out) :: a(:)
    character(len=128) :: error_msg
    integer :: dt, nd, shp(8)
    call info(this, name, dt, nd, shp)
    if (nd < 0 .or. dt == 2) then
      error_msg = "file: numeric variable " // trim(name) // " missing"; return
    end if
    allocate(a(product(shp(1:max(nd, 1)))))
    error_msg = rrtmgpnn_check(c_file_read(this%h, trim(name) // c_null_char, 0_c_int, c_loc(a), &
                                           int(size(a), c_long_long)), "file")
  end function real1

  function real2(this, name, a) result(error_msg)
    class(ty_data_file), intent(in) :: this
    character(len=*), intent(in) :: name
    real(c_float), allocatable, target, intent(out) :: a(:,:)
    character(len=128) :: error_msg
    integer :: dt, nd, shp(8)
    call info(this, name, dt, nd, shp)
    if (nd /= 2 .or. dt == 2) then
      error_msg = "file: 2-D numeric variable " // trim(name) // " missing"; return
    end if
    allocate(a(shp(1), shp(2)))
    error_msg = rrtmgpnn_check(c_file_read(this%h, trim(name) // c_null_char, 0_c_int, c_loc(a), &
                                           int(size(a), c_long_long)), "file")
  end function real2

  function int1(this, name, a) result(error_msg)
    class(ty_data_file), intent(in) :: this
    character(len=*), intent(in) :: name
    integer(c_int), allocatable, target, intent(out) :: a(:)
    character(len=128) :: error_msg
    integer :: dt, nd, shp(8)
    call info(this, name, dt, nd, shp)
    if (nd < 0 .or. dt == 2) then
      error_msg = "file: numeric variable " // trim(name) // " missing"; return
    end if
    allocate(a(product(shp(1:max(nd, 1)))))
    error_msg = rrtmgpnn_check(c_file_read(this%h, trim(name) // c_null_char, 1_c_int, c_loc(a), &
                                           int(size(a), c_long_long)), "file")
  end function int1

  ! A (string_len, n) character variable as n strings (the reference's read_char_vec)
  function strings(this, name, s) result(error_msg)
    class(ty_data_file), intent(in) :: this
    character(len=*), intent(in) :: name
    character(len=32), allocatable, intent(out) :: s(:)
    character(len=128) :: error_msg
    integer :: dt, nd, shp(8), i, j, w
    character(kind=c_char), allocatable, target :: raw(:)
    call info(this, name, dt, nd, shp)
    if (nd /= 2 .or. dt /= 2) then
      error_msg = "file: character variable " // trim(name) // " missing"; return
    end if
    allocate(raw(shp(1) * shp(2)), s(shp(2)))
    error_msg = rrtmgpnn_check(c_file_read(this%h, trim(name) // c_null_char, 2_c_int, c_loc(raw), &
                                           int(size(raw), c_long_long)), "file")
    if (error_msg /= '') return
    w = min(shp(1), 32)
    do i = 1, shp(2)
      s(i) = ''
      do j = 1, w
        if (raw((i - 1) * shp(1) + j) /= c_null_char) s(i)(j:j) = raw((i - 1) * shp(1) + j)
      end do
    end do
  end function strings
end module mo_rrtmgpnn_file
