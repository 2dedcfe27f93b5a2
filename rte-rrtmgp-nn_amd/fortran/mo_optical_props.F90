! mo_optical_props -- drop-in for rte/mo_optical_props.F90: spectral discretisation and the
! (ngpt, nlay, ncol) optical-property arrays, g-point fastest (the fork's layout, :99,179-180).
module mo_optical_props
  use mo_rte_kind, only: wp
  implicit none
  private

  type, public :: ty_optical_props
    integer,  dimension(:,:), allocatable :: band2gpt      ! (2, nband)
    real(wp), dimension(:,:), allocatable :: band_lims_wvn ! (2, nband)
    character(len=128) :: name = ""
  contains
    procedure, private :: init_base
    procedure, private :: init_base_from_copy
    generic,   public  :: init => init_base, init_base_from_copy
    procedure, public  :: is_initialized
    procedure, public  :: get_nband
    procedure, public  :: get_ngpt
    procedure, public  :: get_band_lims_gpoint
    procedure, public  :: get_band_lims_wavenumber
    procedure, public  :: get_gpoint_bands
    procedure, public  :: set_name
    procedure, public  :: get_name
  end type ty_optical_props

  type, extends(ty_optical_props), public :: ty_optical_props_arry
    real(wp), dimension(:,:,:), allocatable :: tau  ! (ngpt, nlay, ncol)
  contains
    procedure, public :: get_ncol
    procedure, public :: get_nlay
  end type ty_optical_props_arry

  type, extends(ty_optical_props_arry), public :: ty_optical_props_1scl
  contains
    procedure, private :: alloc_only_1scl
    procedure, private :: init_and_alloc_1scl
    procedure, private :: copy_and_alloc_1scl
    generic,   public  :: alloc_1scl => alloc_only_1scl, init_and_alloc_1scl, copy_and_alloc_1scl
    procedure, public  :: finalize => finalize_1scl
  end type ty_optical_props_1scl

  type, extends(ty_optical_props_arry), public :: ty_optical_props_2str
    real(wp), dimension(:,:,:), allocatable :: ssa, g
  contains
    procedure, private :: alloc_only_2str
    procedure, private :: init_and_alloc_2str
    procedure, private :: copy_and_alloc_2str
    generic,   public  :: alloc_2str => alloc_only_2str, init_and_alloc_2str, copy_and_alloc_2str
    procedure, public  :: finalize => finalize_2str
  end type ty_optical_props_2str

contains

  function init_base(this, band_lims_wvn, band_lims_gpt, name) result(err_message)
    class(ty_optical_props), intent(inout) :: this
    real(wp), dimension(:,:), intent(in) :: band_lims_wvn
    integer,  dimension(:,:), optional, intent(in) :: band_lims_gpt
    character(len=*), optional, intent(in) :: name
    character(len=128) :: err_message
    integer :: i
    err_message = ''
    if (size(band_lims_wvn, 1) /= 2) then
      err_message = "optical_props%init(): band_lims_wvn 1st dim should be 2"; return
    end if
    if (any(band_lims_wvn < 0._wp)) then
      err_message = "optical_props%init(): band_lims_wvn has values <  0., respectively"; return
    end if
    if (allocated(this%band2gpt)) deallocate(this%band2gpt)
    if (allocated(this%band_lims_wvn)) deallocate(this%band_lims_wvn)
    if (present(band_lims_gpt)) then
      if (size(band_lims_gpt, 1) /= 2 .or. size(band_lims_gpt, 2) /= size(band_lims_wvn, 2)) then
        err_message = "optical_props%init(): band_lims_gpt size inconsistent with band_lims_wvn"; return
      end if
      if (any(band_lims_gpt < 1)) then
        err_message = "optical_props%init(): band_lims_gpt has values < 1"; return
      end if
      this%band2gpt = band_lims_gpt
    else
      allocate(this%band2gpt(2, size(band_lims_wvn, 2)))
      do i = 1, size(band_lims_wvn, 2)
        this%band2gpt(:, i) = i
      end do
    end if
    this%band_lims_wvn = band_lims_wvn
    if (present(name)) this%name = name
  end function init_base

  function init_base_from_copy(this, spectral_desc) result(err_message)
    class(ty_optical_props), intent(inout) :: this
    class(ty_optical_props), intent(in) :: spectral_desc
    character(len=128) :: err_message
    if (.not. spectral_desc%is_initialized()) then
      err_message = "optical_props%init(): can't initialize based on un-initialized input"; return
    end if
    err_message = this%init_base(spectral_desc%band_lims_wvn, spectral_desc%band2gpt)
  end function init_base_from_copy

  pure logical function is_initialized(this)
    class(ty_optical_props), intent(in) :: this
    is_initialized = allocated(this%band2gpt)
  end function is_initialized

  pure integer function get_nband(this)
    class(ty_optical_props), intent(in) :: this
    get_nband = 0
    if (allocated(this%band2gpt)) get_nband = size(this%band2gpt, 2)
  end function get_nband

  pure integer function get_ngpt(this)
    class(ty_optical_props), intent(in) :: this
    get_ngpt = 0
    if (allocated(this%band2gpt)) get_ngpt = maxval(this%band2gpt)
  end function get_ngpt

  pure function get_band_lims_gpoint(this)
    class(ty_optical_props), intent(in) :: this
    integer, dimension(size(this%band2gpt, 1), size(this%band2gpt, 2)) :: get_band_lims_gpoint
    get_band_lims_gpoint = this%band2gpt
  end function get_band_lims_gpoint

  pure function get_band_lims_wavenumber(this)
    class(ty_optical_props), intent(in) :: this
    real(wp), dimension(size(this%band_lims_wvn, 1), size(this%band_lims_wvn, 2)) :: get_band_lims_wavenumber
    get_band_lims_wavenumber = this%band_lims_wvn
  end function get_band_lims_wavenumber

  pure function get_gpoint_bands(this)
    class(ty_optical_props), intent(in) :: this
    integer, dimension(maxval(this%band2gpt)) :: get_gpoint_bands
    integer :: i
    do i = 1, size(this%band2gpt, 2)
      get_gpoint_bands(this%band2gpt(1, i):this%band2gpt(2, i)) = i
    end do
  end function get_gpoint_bands

  subroutine set_name(this, name)
    class(ty_optical_props), intent(inout) :: this
    character(len=*), intent(in) :: name
    this%name = trim(name)
  end subroutine set_name

  function get_name(this)
    class(ty_optical_props), intent(in) :: this
    character(len=len_trim(this%name)) :: get_name
    get_name = trim(this%name)
  end function get_name

  pure integer function get_ncol(this)
    class(ty_optical_props_arry), intent(in) :: this
    get_ncol = 0
    if (allocated(this%tau)) get_ncol = size(this%tau, 3)
  end function get_ncol

  pure integer function get_nlay(this)
    class(ty_optical_props_arry), intent(in) :: this
    get_nlay = 0
    if (allocated(this%tau)) get_nlay = size(this%tau, 2)
  end function get_nlay

  function alloc_only_1scl(this, ncol, nlay) result(err_message)
    class(ty_optical_props_1scl) :: this
    integer, intent(in) :: ncol, nlay
    character(len=128) :: err_message
    err_message = ''
    if (any([ncol, nlay] <= 0)) then
      err_message = "optical_props%alloc: must provide positive extents for ncol, nlay"; return
    end if
    if (.not. this%is_initialized()) then
      err_message = "optical_props%alloc: spectral discretization hasn't been provided"; return
    end if
    if (allocated(this%tau)) deallocate(this%tau)
    allocate(this%tau(this%get_ngpt(), nlay, ncol))
  end function alloc_only_1scl

  function init_and_alloc_1scl(this, ncol, nlay, band_lims_wvn, band_lims_gpt, name) result(err_message)
    class(ty_optical_props_1scl) :: this
    integer, intent(in) :: ncol, nlay
    real(wp), dimension(:,:), intent(in) :: band_lims_wvn
    integer,  dimension(:,:), optional, intent(in) :: band_lims_gpt
    character(len=*), optional, intent(in) :: name
    character(len=128) :: err_message
    err_message = this%init(band_lims_wvn, band_lims_gpt, name)
    if (err_message /= '') return
    err_message = this%alloc_only_1scl(ncol, nlay)
  end function init_and_alloc_1scl

  function copy_and_alloc_1scl(this, ncol, nlay, spectral_desc, name) result(err_message)
    class(ty_optical_props_1scl) :: this
    integer, intent(in) :: ncol, nlay
    class(ty_optical_props), intent(in) :: spectral_desc
    character(len=*), optional, intent(in) :: name
    character(len=128) :: err_message
    err_message = this%init(spectral_desc)
    if (err_message /= '') return
    if (present(name)) this%name = name
    err_message = this%alloc_only_1scl(ncol, nlay)
  end function copy_and_alloc_1scl

  subroutine finalize_1scl(this)
    class(ty_optical_props_1scl), intent(inout) :: this
    if (allocated(this%tau)) deallocate(this%tau)
    if (allocated(this%band2gpt)) deallocate(this%band2gpt)
    if (allocated(this%band_lims_wvn)) deallocate(this%band_lims_wvn)
  end subroutine finalize_1scl

  function alloc_only_2str(this, ncol, nlay) result(err_message)
    class(ty_optical_props_2str) :: this
    integer, intent(in) :: ncol, nlay
    character(len=128) :: err_message
    err_message = ''
    if (any([ncol, nlay] <= 0)) then
      err_message = "optical_props%alloc: must provide positive extents for ncol, nlay"; return
    end if
    if (.not. this%is_initialized()) then
      err_message = "optical_props%alloc: spectral discretization hasn't been provided"; return
    end if
    if (allocated(this%tau)) deallocate(this%tau)
    if (allocated(this%ssa)) deallocate(this%ssa)
    if (allocated(this%g)) deallocate(this%g)
    allocate(this%tau(this%get_ngpt(), nlay, ncol), this%ssa(this%get_ngpt(), nlay, ncol), &
             this%g(this%get_ngpt(), nlay, ncol))
  end function alloc_only_2str

  function init_and_alloc_2str(this, ncol, nlay, band_lims_wvn, band_lims_gpt, name) result(err_message)
    class(ty_optical_props_2str) :: this
    integer, intent(in) :: ncol, nlay
    real(wp), dimension(:,:), intent(in) :: band_lims_wvn
    integer,  dimension(:,:), optional, intent(in) :: band_lims_gpt
    character(len=*), optional, intent(in) :: name
    character(len=128) :: err_message
    err_message = this%init(band_lims_wvn, band_lims_gpt, name)
    if (err_message /= '') return
    err_message = this%alloc_only_2str(ncol, nlay)
  end function init_and_alloc_2str

  function copy_and_alloc_2str(this, ncol, nlay, spectral_desc, name) result(err_message)
    class(ty_optical_props_2str) :: this
    integer, intent(in) :: ncol, nlay
    class(ty_optical_props), intent(in) :: spectral_desc
    character(len=*), optional, intent(in) :: name
    character(len=128) :: err_message
    err_message = this%init(spectral_desc)
    if (err_message /= '') return
    if (present(name)) this%name = name
    err_message = this%alloc_only_2str(ncol, nlay)
  end function copy_and_alloc_2str

  subroutine finalize_2str(this)
    class(ty_optical_props_2str), intent(inout) :: this
    if (allocated(this%tau)) deallocate(this%tau)
    if (allocated(this%ssa)) deallocate(this%ssa)
    if (allocated(this%g)) deallocate(this%g)
    if (allocated(this%band2gpt)) deallocate(this%band2gpt)
    if (allocated(this%band_lims_wvn)) deallocate(this%band_lims_wvn)
  end subroutine finalize_2str
end module mo_optical_props
