! mo_source_functions -- drop-in for rte/mo_source_functions.F90 (ty_source_func_lw, :26-136).
module mo_source_functions
  use mo_rte_kind,      only: wp
  use mo_optical_props, only: ty_optical_props
  implicit none
  private

  type, extends(ty_optical_props), public :: ty_source_func_lw
    real(wp), allocatable, dimension(:,:,:) :: lev_source, lay_source   ! (ngpt, nlay[+1], ncol)
    real(wp), allocatable, dimension(:,:  ) :: sfc_source, sfc_source_Jac
  contains
    procedure, private :: alloc_lw
    procedure, private :: copy_and_alloc_lw
    generic,   public  :: alloc => alloc_lw, copy_and_alloc_lw
    procedure, public  :: is_allocated => is_allocated_lw
    procedure, public  :: finalize => finalize_lw
    procedure, public  :: get_ncol => get_ncol_lw
    procedure, public  :: get_nlay => get_nlay_lw
  end type ty_source_func_lw

contains

  pure logical function is_allocated_lw(this)
    class(ty_source_func_lw), intent(in) :: this
    is_allocated_lw = this%is_initialized() .and. allocated(this%sfc_source)
  end function is_allocated_lw

  function alloc_lw(this, ncol, nlay) result(err_message)
    class(ty_source_func_lw), intent(inout) :: this
    integer, intent(in) :: ncol, nlay
    character(len=128) :: err_message
    integer :: ngpt
    err_message = ''
    if (.not. this%is_initialized()) then
      err_message = "source_func_lw%alloc: not initialized so can't allocate"; return
    end if
    if (any([ncol, nlay] <= 0)) then
      err_message = "source_func_lw%alloc: must provide positive extents for ncol, nlay"; return
    end if
    call finalize_arrays(this)
    ngpt = this%get_ngpt()
    allocate(this%sfc_source(ngpt, ncol), this%sfc_source_Jac(ngpt, ncol), this%lay_source(ngpt, nlay, ncol), &
             this%lev_source(ngpt, nlay+1, ncol))
  end function alloc_lw

  function copy_and_alloc_lw(this, ncol, nlay, spectral_desc) result(err_message)
    class(ty_source_func_lw), intent(inout) :: this
    integer, intent(in) :: ncol, nlay
    class(ty_optical_props), intent(in) :: spectral_desc
    character(len=128) :: err_message
    err_message = this%init(spectral_desc)
    if (err_message /= '') return
    err_message = this%alloc_lw(ncol, nlay)
  end function copy_and_alloc_lw

  subroutine finalize_arrays(this)
    class(ty_source_func_lw), intent(inout) :: this
    if (allocated(this%sfc_source)) deallocate(this%sfc_source)
    if (allocated(this%sfc_source_Jac)) deallocate(this%sfc_source_Jac)
    if (allocated(this%lay_source)) deallocate(this%lay_source)
    if (allocated(this%lev_source)) deallocate(this%lev_source)
  end subroutine finalize_arrays

  subroutine finalize_lw(this)
    class(ty_source_func_lw), intent(inout) :: this
    call finalize_arrays(this)
    if (allocated(this%band2gpt)) deallocate(this%band2gpt)
    if (allocated(this%band_lims_wvn)) deallocate(this%band_lims_wvn)
  end subroutine finalize_lw

  pure integer function get_ncol_lw(this)
    class(ty_source_func_lw), intent(in) :: this
    get_ncol_lw = 0
    if (allocated(this%lay_source)) get_ncol_lw = size(this%lay_source, 3)
  end function get_ncol_lw

  pure integer function get_nlay_lw(this)
    class(ty_source_func_lw), intent(in) :: this
    get_nlay_lw = 0
    if (allocated(this%lay_source)) get_nlay_lw = size(this%lay_source, 2)
  end function get_nlay_lw
end module mo_source_functions
