! mo_source_functions -- drop-in for rte/mo_source_functions.F90 (ty_source_func_lw, :26-136).
!
! Device residency as in mo_optical_props.  In addition, gas_optics with neural networks may leave the Planck
! sources unformed (planck_deferred): lay_source's device copy then holds the network's Planck fraction and the
! object keeps device copies of the temperatures, so rte_lw forms the sources inside the solver
! (rrtmgpnn_lw_solver_noscat_planck) and lay_source / lev_source never travel through HBM.  Any consumer that needs
! the sources themselves -- update_host(), the two-stream solvers -- forms them first with compute_Planck_source_nn
! (rrtmgp/kernels/mo_gas_optics_kernels.F90:615-683), the same values bit for bit.
module mo_source_functions
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,      only: wp
  use mo_optical_props, only: ty_optical_props
  use mo_rrtmgpnn_c
  implicit none
  private

  type, extends(ty_optical_props), public :: ty_source_func_lw
    real(wp), allocatable, dimension(:,:,:) :: lev_source, lay_source   ! (ngpt, nlay[+1], ncol)
    real(wp), allocatable, dimension(:,:  ) :: sfc_source, sfc_source_Jac
    ! deferred Planck sources (no reference counterpart): the device copies of pk_tlay / pk_tlev / pk_tsfc hold the
    ! temperatures (the host arrays are only their keys), pk_totplnk the k-distribution's table in the context
    logical :: planck_deferred = .false.
    real(wp), allocatable, dimension(:,:) :: pk_tlay, pk_tlev
    real(wp), allocatable, dimension(:)   :: pk_tsfc
    type(c_ptr) :: pk_totplnk = c_null_ptr
    integer  :: pk_ntemp = 0, pk_sfc_lay = 1
    real(wp) :: pk_tmin = 0._wp, pk_tdelta = 0._wp
  contains
    procedure, private :: alloc_lw
    procedure, private :: copy_and_alloc_lw
    generic,   public  :: alloc => alloc_lw, copy_and_alloc_lw
    procedure, public  :: is_allocated => is_allocated_lw
    procedure, public  :: finalize => finalize_lw
    procedure, public  :: get_ncol => get_ncol_lw
    procedure, public  :: get_nlay => get_nlay_lw
    procedure, public  :: form_planck_sources
    procedure, public  :: device_sources
    procedure, public  :: update_host
    procedure, public  :: update_device
    final :: final_lw
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
    call drop2(this%sfc_source)
    call drop2(this%sfc_source_Jac)
    call drop3(this%lay_source)
    call drop3(this%lev_source)
    call drop2(this%pk_tlay)
    call drop2(this%pk_tlev)
    call drop(this%pk_tsfc)
    this%planck_deferred = .false.
  contains
    subroutine drop(a)
      real(wp), allocatable, intent(inout) :: a(:)
      if (allocated(a)) then
        call dev_delete(a)
        deallocate(a)
      end if
    end subroutine drop
    subroutine drop2(a)
      real(wp), allocatable, intent(inout) :: a(:,:)
      if (allocated(a)) then
        call dev_delete(a)
        deallocate(a)
      end if
    end subroutine drop2
    subroutine drop3(a)
      real(wp), allocatable, intent(inout) :: a(:,:,:)
      if (allocated(a)) then
        call dev_delete(a)
        deallocate(a)
      end if
    end subroutine drop3
  end subroutine finalize_arrays

  subroutine finalize_lw(this)
    class(ty_source_func_lw), intent(inout) :: this
    call finalize_arrays(this)
    if (allocated(this%band2gpt)) deallocate(this%band2gpt)
    if (allocated(this%band_lims_wvn)) deallocate(this%band_lims_wvn)
  end subroutine finalize_lw

  ! an object going out of scope (or a private copy of one) drops its device copies
  subroutine final_lw(this)
    type(ty_source_func_lw), intent(inout) :: this
    if (allocated(this%sfc_source)) call dev_delete(this%sfc_source)
    if (allocated(this%sfc_source_Jac)) call dev_delete(this%sfc_source_Jac)
    if (allocated(this%lay_source)) call dev_delete(this%lay_source)
    if (allocated(this%lev_source)) call dev_delete(this%lev_source)
    if (allocated(this%pk_tlay)) call dev_delete(this%pk_tlay)
    if (allocated(this%pk_tlev)) call dev_delete(this%pk_tlev)
    if (allocated(this%pk_tsfc)) call dev_delete(this%pk_tsfc)
  end subroutine final_lw

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

  ! Form deferred Planck sources on the device: compute_Planck_source_nn from the kept Planck fraction and
  ! temperatures (no-op when the sources are formed already).
  function form_planck_sources(this) result(error_msg)
    class(ty_source_func_lw), intent(inout) :: this
    character(len=128) :: error_msg
    integer :: ncol, nlay, ngpt
    integer(c_long_long) :: nlay_g, nlev_g, nsfc
    type(c_ptr) :: d_tlay, d_tlev, d_tsfc, d_lay, d_lev, d_sfc, d_jac
    error_msg = ''
    if (.not. this%planck_deferred) return
    ncol = this%get_ncol()
    nlay = this%get_nlay()
    ngpt = this%get_ngpt()
    nlay_g = int(ngpt, c_long_long) * nlay * ncol
    nlev_g = int(ngpt, c_long_long) * (nlay + 1) * ncol
    nsfc = int(ngpt, c_long_long) * ncol
    d_tlay = dev_present(this%pk_tlay, size(this%pk_tlay, kind=c_long_long), PRESENT_READ)
    d_tlev = dev_present(this%pk_tlev, size(this%pk_tlev, kind=c_long_long), PRESENT_READ)
    d_tsfc = dev_present(this%pk_tsfc, size(this%pk_tsfc, kind=c_long_long), PRESENT_READ)
    d_lay = dev_present(this%lay_source, nlay_g, ior(PRESENT_READ, PRESENT_WRITE))
    d_lev = dev_present(this%lev_source, nlev_g, PRESENT_WRITE)
    d_sfc = dev_present(this%sfc_source, nsfc, PRESENT_WRITE)
    d_jac = dev_present(this%sfc_source_Jac, nsfc, PRESENT_WRITE)
    error_msg = rrtmgpnn_check(c_rrtmgpnn_compute_planck_source_nn(rrtmgpnn_ctx(), ncol, nlay, this%get_nband(), ngpt, &
                  this%pk_ntemp, d_tlay, d_tlev, d_tsfc, this%pk_sfc_lay, this%band2gpt, this%pk_tmin, &
                  this%pk_tdelta, this%pk_totplnk, d_sfc, d_jac, d_lay, d_lev), "compute_planck_source_nn")
    if (error_msg == '') this%planck_deferred = .false.
  end function form_planck_sources

  ! The sources' device data for a solver that reads them (the object is left as it is): the device copies, or, when
  ! deferred, scratch buffers the caller releases (tmp) holding the sources formed from the Planck fraction.
  function device_sources(this, d_lay, d_lev, d_sfc, d_jac, tmp) result(error_msg)
    class(ty_source_func_lw), intent(in) :: this
    type(c_ptr), intent(out) :: d_lay, d_lev, d_sfc, d_jac
    logical, intent(out) :: tmp
    character(len=128) :: error_msg
    integer :: ncol, nlay, ngpt
    integer(c_long_long) :: nlay_g, nlev_g, nsfc
    error_msg = ''
    ncol = this%get_ncol()
    nlay = this%get_nlay()
    ngpt = this%get_ngpt()
    nlay_g = int(ngpt, c_long_long) * nlay * ncol
    nlev_g = int(ngpt, c_long_long) * (nlay + 1) * ncol
    nsfc = int(ngpt, c_long_long) * ncol
    tmp = this%planck_deferred
    if (.not. tmp) then
      d_lay = dev_present(this%lay_source, nlay_g, PRESENT_READ)
      d_lev = dev_present(this%lev_source, nlev_g, PRESENT_READ)
      d_sfc = dev_present(this%sfc_source, nsfc, PRESENT_READ)
      d_jac = c_null_ptr
      return
    end if
    d_lay = dev_scratch(nlay_g)
    call dev_copy_dd(d_lay, dev_present(this%lay_source, nlay_g, PRESENT_READ), nlay_g)  ! the Planck fraction
    d_lev = dev_scratch(nlev_g)
    d_sfc = dev_scratch(nsfc)
    d_jac = dev_scratch(nsfc)
    error_msg = rrtmgpnn_check(c_rrtmgpnn_compute_planck_source_nn(rrtmgpnn_ctx(), ncol, nlay, this%get_nband(), ngpt, &
                  this%pk_ntemp, dev_present(this%pk_tlay, size(this%pk_tlay, kind=c_long_long), PRESENT_READ), &
                  dev_present(this%pk_tlev, size(this%pk_tlev, kind=c_long_long), PRESENT_READ), &
                  dev_present(this%pk_tsfc, size(this%pk_tsfc, kind=c_long_long), PRESENT_READ), this%pk_sfc_lay, &
                  this%band2gpt, this%pk_tmin, this%pk_tdelta, this%pk_totplnk, d_sfc, d_jac, d_lay, d_lev), &
                  "compute_planck_source_nn")
  end function device_sources

  ! `!$acc update host`: the sources (formed first if deferred) copied into the host arrays
  subroutine update_host(this)
    class(ty_source_func_lw), intent(inout) :: this
    character(len=128) :: e
    e = this%form_planck_sources()
    if (e /= '') then
      write(*, '(a)') trim(e)
      error stop 1
    end if
    if (allocated(this%lay_source)) call dev_update_host(this%lay_source)
    if (allocated(this%lev_source)) call dev_update_host(this%lev_source)
    if (allocated(this%sfc_source)) call dev_update_host(this%sfc_source)
    if (allocated(this%sfc_source_Jac)) call dev_update_host(this%sfc_source_Jac)
  end subroutine update_host

  ! `!$acc update device`: the host arrays were written; kernels read them from the host copies next
  subroutine update_device(this)
    class(ty_source_func_lw), intent(inout) :: this
    this%planck_deferred = .false.
    if (allocated(this%lay_source)) call dev_update_device(this%lay_source)
    if (allocated(this%lev_source)) call dev_update_device(this%lev_source)
    if (allocated(this%sfc_source)) call dev_update_device(this%sfc_source)
    if (allocated(this%sfc_source_Jac)) call dev_update_device(this%sfc_source_Jac)
  end subroutine update_device
end module mo_source_functions
