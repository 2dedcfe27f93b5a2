! mo_optical_props -- drop-in for rte/mo_optical_props.F90: spectral discretisation and the
! (ngpt, nlay, ncol) optical-property arrays, g-point fastest (the fork's layout, :99,179-180).
! increment (:882-1023) and delta_scale (:565-604) run in the HIP kernels behind the C ABI.
!
! Device residency, as in the reference's OpenACC build (the arrays are created on the device by the constructors,
! examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:325-327): every array has a device copy in the calling thread's
! context (mo_rrtmgpnn_c: dev_present).  Arrays the library produces (gas_optics, cloud_optics, increment,
! delta_scale) stay on the device until a consumer reads them there (rte_lw, rte_sw, increment); the host copy is
! refreshed only by update_host() (`!$acc update host`).  Arrays the caller fills on the host are uploaded when a
! kernel first reads them; after host writes to an array the library had produced, call update_device()
! (`!$acc update device`).
module mo_optical_props
  use, intrinsic :: iso_c_binding
  use mo_rte_kind, only: wp
  use mo_rrtmgpnn_c
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
    procedure, public  :: bands_are_equal
    procedure, public  :: gpoints_are_equal
  end type ty_optical_props

  type, extends(ty_optical_props), public :: ty_optical_props_arry
    real(wp), dimension(:,:,:), allocatable :: tau  ! (ngpt, nlay, ncol)
  contains
    procedure, public :: get_ncol
    procedure, public :: get_nlay
    procedure, public :: increment
    procedure, public :: update_host
    procedure, public :: update_device
    final :: final_arry
  end type ty_optical_props_arry

  type, extends(ty_optical_props_arry), public :: ty_optical_props_1scl
  contains
    procedure, private :: alloc_only_1scl
    procedure, private :: init_and_alloc_1scl
    procedure, private :: copy_and_alloc_1scl
    generic,   public  :: alloc_1scl => alloc_only_1scl, init_and_alloc_1scl, copy_and_alloc_1scl
    procedure, public  :: finalize => finalize_1scl
    procedure, public  :: delta_scale => delta_scale_1scl
  end type ty_optical_props_1scl

  type, extends(ty_optical_props_arry), public :: ty_optical_props_2str
    real(wp), dimension(:,:,:), allocatable :: ssa, g
    ! g is identically zero and its device copy was never written (gas_optics' NN shortwave, which sets g = 0,
    ! mo_gas_optics_rrtmgp.F90:560-567): rte_sw passes no g array; other device consumers fill it first
    logical :: g_zero = .false.
  contains
    procedure, private :: alloc_only_2str
    procedure, private :: init_and_alloc_2str
    procedure, private :: copy_and_alloc_2str
    generic,   public  :: alloc_2str => alloc_only_2str, init_and_alloc_2str, copy_and_alloc_2str
    procedure, public  :: finalize => finalize_2str
    procedure, public  :: delta_scale => delta_scale_2str
    procedure, public  :: validate => validate_2stream
    final :: final_2str
  end type ty_optical_props_2str
  public :: dev_g, dev_g_read

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

  ! Same number of bands, limits within 5 spacings (rte/mo_optical_props.F90:1204-1214)
  pure logical function bands_are_equal(this, that)
    class(ty_optical_props), intent(in) :: this, that
    bands_are_equal = this%get_nband() == that%get_nband() .and. this%get_nband() > 0
    if (.not. bands_are_equal) return
    bands_are_equal = all(abs(this%band_lims_wvn - that%band_lims_wvn) < 5._wp * spacing(this%band_lims_wvn))
  end function bands_are_equal

  ! Same bands, same g-points, same band <-> g-point mapping (:1220-1229)
  pure logical function gpoints_are_equal(this, that)
    class(ty_optical_props), intent(in) :: this, that
    gpoints_are_equal = this%bands_are_equal(that) .and. this%get_ngpt() == that%get_ngpt()
    if (.not. gpoints_are_equal) return
    gpoints_are_equal = all(this%get_gpoint_bands() == that%get_gpoint_bands())
  end function gpoints_are_equal

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
    call drop_arrays(this)
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
    call drop_arrays(this)
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
    call drop_arrays(this)
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
    call drop_arrays(this)
    if (allocated(this%band2gpt)) deallocate(this%band2gpt)
    if (allocated(this%band_lims_wvn)) deallocate(this%band_lims_wvn)
  end subroutine finalize_2str

  ! op_in%increment(op_io) (rte/mo_optical_props.F90:882-1023): add op_in to op_io, at the same g-point
  ! resolution or, when op_in is defined by band, by band into op_io's g-points.  On the device copies.
  function increment(op_in, op_io) result(err_message)
    class(ty_optical_props_arry), intent(in)    :: op_in
    class(ty_optical_props_arry), intent(inout) :: op_io
    character(len=128) :: err_message
    integer :: ncol, nlay, ngpt
    integer(c_long_long) :: n_io, n_in
    logical :: same, g2_tmp
    type(c_ptr) :: t1, s1, g1, t2, s2, g2

    err_message = ""
    if (.not. op_in%bands_are_equal(op_io)) then
      err_message = "ty_optical_props%increment: optical properties objects have different band structures"; return
    end if
    ncol = op_io%get_ncol()
    nlay = op_io%get_nlay()
    ngpt = op_io%get_ngpt()
    if (op_in%get_ncol() /= ncol .or. op_in%get_nlay() /= nlay) then
      err_message = "ty_optical_props%increment: optical properties objects have different extents"; return
    end if
    same = op_in%gpoints_are_equal(op_io)
    if (.not. same .and. op_in%get_ngpt() /= op_io%get_nband()) then  ! by band: ngpt() = nband() (:955-958)
      err_message = "ty_optical_props%increment: optical properties objects have incompatible g-point structures"
      return
    end if
    n_io = size(op_io%tau, kind=c_long_long)
    n_in = size(op_in%tau, kind=c_long_long)
    s1 = c_null_ptr; g1 = c_null_ptr; s2 = c_null_ptr; g2 = c_null_ptr
    g2_tmp = .false.
    t2 = dev_present(op_in%tau, n_in, PRESENT_READ)
    select type (op_in)
    class is (ty_optical_props_2str)
      s2 = dev_present(op_in%ssa, n_in, PRESENT_READ)
      if (op_in%g_zero) then  ! op_in is intent(in): a zero-filled scratch copy stands in for its g
        g2 = dev_scratch(n_in)
        call dev_zero(g2, n_in)
        g2_tmp = .true.
      else
        g2 = dev_present(op_in%g, n_in, PRESENT_READ)
      end if
    end select
    t1 = dev_present(op_io%tau, n_io, ior(PRESENT_READ, PRESENT_WRITE))
    select type (op_io)
    class is (ty_optical_props_2str)
      s1 = dev_present(op_io%ssa, n_io, ior(PRESENT_READ, PRESENT_WRITE))
      g1 = dev_g(op_io)
    end select
    if (same) then
      err_message = rrtmgpnn_check(c_rrtmgpnn_increment(rrtmgpnn_ctx(), ncol, nlay, ngpt, t1, s1, g1, t2, s2, g2), &
                                   "ty_optical_props%increment")
    else
      err_message = rrtmgpnn_check(c_rrtmgpnn_increment_bybnd(rrtmgpnn_ctx(), ncol, nlay, ngpt, op_io%get_nband(), &
                                   op_io%band2gpt, t1, s1, g1, t2, s2, g2), "ty_optical_props%increment")
    end if
    if (g2_tmp) call dev_release(g2)
  end function increment

  ! The device copy of a two-stream g for a kernel that reads and writes it: an identically zero g (g_zero) is
  ! filled on the device first.
  function dev_g(op) result(d)
    class(ty_optical_props_2str), intent(inout) :: op
    type(c_ptr) :: d
    integer(c_long_long) :: n
    n = size(op%g, kind=c_long_long)
    if (op%g_zero) then
      d = dev_present(op%g, n, PRESENT_WRITE)
      call dev_zero(d, n)
      op%g_zero = .false.
    else
      d = dev_present(op%g, n, ior(PRESENT_READ, PRESENT_WRITE))
    end if
  end function dev_g

  ! The device copy of a two-stream g for a kernel that only reads it; for an identically zero g (g_zero) a
  ! zero-filled scratch buffer the caller releases (tmp), leaving op untouched.
  function dev_g_read(op, tmp) result(d)
    class(ty_optical_props_2str), intent(in) :: op
    logical, intent(out) :: tmp
    type(c_ptr) :: d
    integer(c_long_long) :: n
    n = size(op%g, kind=c_long_long)
    tmp = op%g_zero
    if (tmp) then
      d = dev_scratch(n)
      call dev_zero(d, n)
    else
      d = dev_present(op%g, n, PRESENT_READ)
    end if
  end function dev_g_read

  ! `!$acc update host`: refresh the host arrays from their device copies
  subroutine update_host(this)
    class(ty_optical_props_arry), intent(inout) :: this
    if (allocated(this%tau)) call dev_update_host(this%tau)
    select type (this)
    class is (ty_optical_props_2str)
      if (allocated(this%ssa)) call dev_update_host(this%ssa)
      if (this%g_zero) then
        this%g = 0._wp
        this%g_zero = .false.
        call dev_delete(this%g)
      else if (allocated(this%g)) then
        call dev_update_host(this%g)
      end if
    end select
  end subroutine update_host

  ! `!$acc update device`: the host arrays were written; kernels read them from the host copies next
  subroutine update_device(this)
    class(ty_optical_props_arry), intent(inout) :: this
    if (allocated(this%tau)) call dev_update_device(this%tau)
    select type (this)
    class is (ty_optical_props_2str)
      if (allocated(this%ssa)) call dev_update_device(this%ssa)
      if (allocated(this%g)) call dev_update_device(this%g)
      this%g_zero = .false.
    end select
  end subroutine update_device

  ! drop the device copies of the arrays and deallocate them
  subroutine drop_arrays(this)
    class(ty_optical_props_arry), intent(inout) :: this
    if (allocated(this%tau)) then
      call dev_delete(this%tau)
      deallocate(this%tau)
    end if
    select type (this)
    class is (ty_optical_props_2str)
      if (allocated(this%ssa)) then
        call dev_delete(this%ssa)
        deallocate(this%ssa)
      end if
      if (allocated(this%g)) then
        call dev_delete(this%g)
        deallocate(this%g)
      end if
      this%g_zero = .false.
    end select
  end subroutine drop_arrays

  ! finalizers: an object going out of scope (or a private copy of one) drops its device copies, so a later
  ! array at the same address never finds them
  subroutine final_arry(this)
    type(ty_optical_props_arry), intent(inout) :: this
    if (allocated(this%tau)) call dev_delete(this%tau)
  end subroutine final_arry

  subroutine final_2str(this)
    type(ty_optical_props_2str), intent(inout) :: this
    if (allocated(this%ssa)) call dev_delete(this%ssa)
    if (allocated(this%g)) call dev_delete(this%g)
  end subroutine final_2str

  ! validate_2stream (:635-671), on the current values (a device-newer array is checked from a copy of its device
  ! data; the host arrays are left as they are)
  function validate_2stream(this) result(err_message)
    class(ty_optical_props_2str), intent(in) :: this
    character(len=128) :: err_message
    real(wp), allocatable :: tau(:,:,:), ssa(:,:,:), g(:,:,:)
    err_message = ''
    if (.not. all([allocated(this%tau), allocated(this%ssa), allocated(this%g)])) then
      err_message = "validate: arrays not allocated/initialized"; return
    end if
    if (any(shape(this%ssa) /= shape(this%tau)) .or. any(shape(this%g) /= shape(this%tau))) then
      err_message = "validate: arrays not sized consistently"; return
    end if
    call current(this%tau, tau)
    call current(this%ssa, ssa)
    if (this%g_zero) then
      allocate(g(size(this%g, 1), size(this%g, 2), size(this%g, 3)))
      g = 0._wp
    else
      call current(this%g, g)
    end if
    if (any(tau < 0._wp)) err_message = "validate: tau values out of range"
    if (any(ssa < 0._wp .or. ssa > 1.0001_wp)) err_message = "validate: ssa values out of range"
    if (any(g < -1._wp .or. g > 1._wp)) err_message = "validate: g values out of range"
  contains
    subroutine current(a, c)
      real(wp), intent(in) :: a(:,:,:)
      real(wp), allocatable, intent(out) :: c(:,:,:)
      character(len=128) :: e
      integer(c_long_long) :: n
      allocate(c(size(a, 1), size(a, 2), size(a, 3)))
      if (.not. rrtmgpnn_has_context()) then
        c = a
        return
      end if
      n = size(a, kind=c_long_long)
      call dev_copy_out(c, dev_present(a, n, PRESENT_READ), n)
      e = ''
      call rrtmgpnn_sync(e, "validate")
    end subroutine current
  end function validate_2stream

  ! delta_scale_1scl (:565-574): absorption optical depth needs no scaling
  function delta_scale_1scl(this, for) result(err_message)
    class(ty_optical_props_1scl), intent(inout) :: this
    real(wp), dimension(:,:,:), optional, intent(in) :: for
    character(len=128) :: err_message
    err_message = ''
  end function delta_scale_1scl

  ! delta_scale_2str (:576-604): forward-scattering fraction `for`, g**2 if absent; on the device copies
  function delta_scale_2str(this, for) result(err_message)
    class(ty_optical_props_2str), intent(inout) :: this
    real(wp), dimension(:,:,:), optional, intent(in) :: for
    character(len=128) :: err_message
    integer(c_long_long) :: n
    type(c_ptr) :: dt, ds, dg, df
    err_message = ''
    n = size(this%tau, kind=c_long_long)
    df = c_null_ptr
    if (present(for)) then
      if (any(shape(for) /= shape(this%tau))) then
        err_message = "delta_scale: dimension of 'for' don't match optical properties arrays"; return
      end if
      if (any(for < 0._wp .or. for > 1._wp)) then
        err_message = "delta_scale: values of 'for' out of bounds [0,1]"; return
      end if
      df = dev_stage(for, n)
    end if
    dt = dev_present(this%tau, n, ior(PRESENT_READ, PRESENT_WRITE))
    ds = dev_present(this%ssa, n, ior(PRESENT_READ, PRESENT_WRITE))
    dg = dev_g(this)
    err_message = rrtmgpnn_check(c_rrtmgpnn_delta_scale_2str(rrtmgpnn_ctx(), n, dt, ds, dg, df), "delta_scale")
    call dev_release(df)
  end function delta_scale_2str
end module mo_optical_props
