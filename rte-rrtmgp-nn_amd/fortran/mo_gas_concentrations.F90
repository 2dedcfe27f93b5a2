! mo_gas_concentrations -- drop-in for rrtmgp/mo_gas_concentrations.F90 (ty_gas_concs): per-gas volume
! mixing ratios stored as conc(1,1) (scalar), conc(nlay,1) (1-D) or conc(nlay,ncol) (2-D), as :50-59.
! Each concentration array has a device copy in the calling thread's context, uploaded when gas optics first
! reads it after set_vmr (the reference copies it in set_vmr, `!$acc enter data copyin`, :166).
module mo_gas_concentrations
  use, intrinsic :: iso_c_binding, only: c_ptr, c_long_long
  use mo_rte_kind, only: wp
  use mo_rrtmgpnn_c, only: dev_present, dev_delete, PRESENT_READ
  implicit none
  private
  integer, parameter, public :: GAS_NOT_IN_LIST = 0

  type, public :: conc_field
    real(wp), dimension(:,:), allocatable :: conc
  contains
    final :: final_conc  ! drops the device copy with the array
  end type conc_field

  type, public :: ty_gas_concs
    character(len=32), dimension(:), allocatable :: gas_name
    type(conc_field),  dimension(:), allocatable :: concs
    integer :: nlay = 0, ncol = 0
  contains
    procedure, public :: init
    procedure, private :: set_vmr_scalar, set_vmr_1d, set_vmr_2d
    generic,   public :: set_vmr => set_vmr_scalar, set_vmr_1d, set_vmr_2d
    procedure, public :: get_gas_names
    procedure, public :: find_gas
    procedure, public :: get_conc_dims_and_igas
    procedure, public :: device_conc
  end type ty_gas_concs

contains

  function init(this, gas_names) result(error_msg)
    class(ty_gas_concs), intent(inout) :: this
    character(len=*), dimension(:), intent(in) :: gas_names
    character(len=128) :: error_msg
    integer :: i, j
    error_msg = ''
    do i = 1, size(gas_names)
      do j = i + 1, size(gas_names)
        if (lower(gas_names(i)) == lower(gas_names(j))) then
          error_msg = 'ty_gas_concs%init(): duplicate gas names aren''t allowed'
          return
        end if
      end do
    end do
    if (allocated(this%gas_name)) deallocate(this%gas_name)
    if (allocated(this%concs)) then
      do i = 1, size(this%concs)
        call drop_conc(this%concs(i))
      end do
      deallocate(this%concs)
    end if
    allocate(this%gas_name(size(gas_names)), this%concs(size(gas_names)))
    do i = 1, size(gas_names)
      this%gas_name(i) = lower(gas_names(i))
    end do
    this%nlay = 0
    this%ncol = 0
  end function init

  function set_vmr_scalar(this, gas, w) result(error_msg)
    class(ty_gas_concs), intent(inout) :: this
    character(len=*), intent(in) :: gas
    real(wp), intent(in) :: w
    character(len=128) :: error_msg
    integer :: igas
    error_msg = ''
    if (w < 0._wp .or. w > 1._wp) then
      error_msg = 'ty_gas_concs%set_vmr(): concentrations should be >= 0, <= 1'; return
    end if
    igas = this%find_gas(gas)
    if (igas == GAS_NOT_IN_LIST) then
      error_msg = 'ty_gas_concs%set_vmr(): trying to set ' // trim(gas) // ' but name not present'; return
    end if
    call drop_conc(this%concs(igas))
    allocate(this%concs(igas)%conc(1,1))
    this%concs(igas)%conc(1,1) = w
  end function set_vmr_scalar

  function set_vmr_1d(this, gas, w) result(error_msg)
    class(ty_gas_concs), intent(inout) :: this
    character(len=*), intent(in) :: gas
    real(wp), dimension(:), intent(in) :: w
    character(len=128) :: error_msg
    integer :: igas
    error_msg = ''
    if (any(w < 0._wp .or. w > 1._wp)) then
      error_msg = 'ty_gas_concs%set_vmr(): concentrations should be >= 0, <= 1'; return
    end if
    if (this%nlay > 0 .and. size(w) /= this%nlay) then
      error_msg = 'ty_gas_concs%set_vmr(): different dimension (nlay)'; return
    end if
    igas = this%find_gas(gas)
    if (igas == GAS_NOT_IN_LIST) then
      error_msg = 'ty_gas_concs%set_vmr(): trying to set ' // trim(gas) // ' but name not present'; return
    end if
    this%nlay = size(w)
    call drop_conc(this%concs(igas))
    allocate(this%concs(igas)%conc(this%nlay, 1))
    this%concs(igas)%conc(:,1) = w
  end function set_vmr_1d

  function set_vmr_2d(this, gas, w) result(error_msg)
    class(ty_gas_concs), intent(inout) :: this
    character(len=*), intent(in) :: gas
    real(wp), dimension(:,:), intent(in) :: w   ! (nlay, ncol)
    character(len=128) :: error_msg
    integer :: igas
    error_msg = ''
    if (any(w < 0._wp .or. w > 1._wp)) then
      error_msg = 'ty_gas_concs%set_vmr(): concentrations should be >= 0, <= 1'; return
    end if
    if ((this%nlay > 0 .and. size(w, 1) /= this%nlay) .or. (this%ncol > 0 .and. size(w, 2) /= this%ncol)) then
      error_msg = 'ty_gas_concs%set_vmr(): different dimension (nlay, ncol)'; return
    end if
    igas = this%find_gas(gas)
    if (igas == GAS_NOT_IN_LIST) then
      error_msg = 'ty_gas_concs%set_vmr(): trying to set ' // trim(gas) // ' but name not present'; return
    end if
    this%nlay = size(w, 1)
    this%ncol = size(w, 2)
    call drop_conc(this%concs(igas))
    allocate(this%concs(igas)%conc(this%nlay, this%ncol))
    this%concs(igas)%conc = w
  end function set_vmr_2d

  function get_gas_names(this) result(names)
    class(ty_gas_concs), intent(in) :: this
    character(len=32), dimension(size(this%gas_name)) :: names
    names = this%gas_name
  end function get_gas_names

  integer function find_gas(this, gas)
    class(ty_gas_concs), intent(in) :: this
    character(len=*), intent(in) :: gas
    integer :: i
    find_gas = GAS_NOT_IN_LIST
    if (.not. allocated(this%gas_name)) return
    do i = 1, size(this%gas_name)
      if (trim(this%gas_name(i)) == trim(lower(gas))) then
        find_gas = i; return
      end if
    end do
  end function find_gas

  ! mo_gas_concentrations.F90 get_conc_dims_and_igas: ndims 0 (scalar), 1 (nlay) or 2 (nlay,ncol)
  function get_conc_dims_and_igas(this, gas, ndims, igas) result(error_msg)
    class(ty_gas_concs), intent(in) :: this
    character(len=*), intent(in) :: gas
    integer, intent(out) :: ndims, igas
    character(len=128) :: error_msg
    error_msg = ''
    ndims = 0
    igas = this%find_gas(gas)
    if (igas == GAS_NOT_IN_LIST) then
      error_msg = 'gas ' // trim(gas) // ' not found'; return
    end if
    if (.not. allocated(this%concs(igas)%conc)) then
      error_msg = 'gas ' // trim(gas) // ' concentration not set'; igas = GAS_NOT_IN_LIST; return
    end if
    if (size(this%concs(igas)%conc, 2) > 1) then
      ndims = 2
    else if (size(this%concs(igas)%conc, 1) > 1) then
      ndims = 1
    end if
  end function get_conc_dims_and_igas

  ! The device copy of gas igas's concentration array (uploaded when set_vmr changed it since the last read).
  function device_conc(this, igas) result(d)
    class(ty_gas_concs), intent(in) :: this
    integer, intent(in) :: igas
    type(c_ptr) :: d
    d = dev_present(this%concs(igas)%conc, size(this%concs(igas)%conc, kind=c_long_long), PRESENT_READ)
  end function device_conc

  subroutine drop_conc(f)
    type(conc_field), intent(inout) :: f
    if (allocated(f%conc)) then
      call dev_delete(f%conc)
      deallocate(f%conc)
    end if
  end subroutine drop_conc

  subroutine final_conc(f)
    type(conc_field), intent(inout) :: f
    if (allocated(f%conc)) call dev_delete(f%conc)
  end subroutine final_conc

  pure function lower(s) result(r)
    character(len=*), intent(in) :: s
    character(len=len(s)) :: r
    integer :: i, c
    r = s
    do i = 1, len(s)
      c = iachar(s(i:i))
      if (c >= 65 .and. c <= 90) r(i:i) = achar(c + 32)
    end do
    r = adjustl(r)
  end function lower
end module mo_gas_concentrations
