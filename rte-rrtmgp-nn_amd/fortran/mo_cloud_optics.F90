! mo_cloud_optics -- drop-in for extensions/cloud_optics/mo_cloud_optics.F90 (ty_cloud_optics): liquid and
! ice cloud optical properties by band, from a lookup table (load_lut) or Pade approximants (load_pade) of
! effective radius.  The coefficient tables live on the device inside an rrtmgpnn_cloud_optics handle;
! cloud_optics (:354-535) runs as one HIP kernel over (band, layer, column).  load_rbin reads the coefficient
! file rrtmgp-cloud-optics-coeffs-{lw,sw}.nc itself (classic netCDF, native reader) or its RBIN conversion --
! what the example drivers' mo_load_cloud_coefficients does with netcdf-fortran.
module mo_cloud_optics
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,          only: wp
  use mo_rte_rrtmgp_config, only: check_values
  use mo_optical_props,     only: ty_optical_props, ty_optical_props_arry, ty_optical_props_2str
  use mo_rrtmgpnn_c
  implicit none
  private

  type, extends(ty_optical_props), public :: ty_cloud_optics
    private
    type(c_ptr) :: h = c_null_ptr
    integer     :: icergh = 0, nrghice = 0  ! ice roughness (1 = none, 2 = medium, 3 = high)
    real(wp)    :: radliq_lwr = 0._wp, radliq_upr = 0._wp
    real(wp)    :: radice_lwr = 0._wp, radice_upr = 0._wp
  contains
    generic,   public  :: load => load_lut, load_pade
    procedure, public  :: load_rbin
    procedure, public  :: finalize
    procedure, public  :: cloud_optics
    procedure, public  :: get_min_radius_liq
    procedure, public  :: get_min_radius_ice
    procedure, public  :: get_max_radius_liq
    procedure, public  :: get_max_radius_ice
    procedure, public  :: get_num_ice_roughness_types
    procedure, public  :: set_ice_roughness
    procedure, private :: load_lut
    procedure, private :: load_pade
    procedure, private :: adopt
  end type ty_cloud_optics

contains

  ! load_lut (:91-173).  lut_*liq (nsize_liq, nbnd); lut_*ice (nsize_ice, nbnd, nrghice).
  function load_lut(this, band_lims_wvn, radliq_lwr, radliq_upr, radliq_fac, radice_lwr, radice_upr, radice_fac, &
                    lut_extliq, lut_ssaliq, lut_asyliq, lut_extice, lut_ssaice, lut_asyice) result(error_msg)
    class(ty_cloud_optics),     intent(inout) :: this
    real(wp), dimension(:,:),   intent(in)    :: band_lims_wvn
    real(wp),                   intent(in)    :: radliq_lwr, radliq_upr, radliq_fac
    real(wp),                   intent(in)    :: radice_lwr, radice_upr, radice_fac
    real(wp), dimension(:,:),   intent(in)    :: lut_extliq, lut_ssaliq, lut_asyliq
    real(wp), dimension(:,:,:), intent(in)    :: lut_extice, lut_ssaice, lut_asyice
    character(len=128) :: error_msg
    integer :: nbnd
    type(c_ptr) :: h

    nbnd = size(lut_extliq, dim=2)
    error_msg = this%init(band_lims_wvn, name="RRTMGP cloud optics")
    if (error_msg /= '') return
    if (nbnd /= this%get_nband()) &
      error_msg = "cloud_optics%init(): number of bands inconsistent between lookup tables, spectral discretization"
    if (size(lut_extice, 2) /= nbnd) error_msg = "cloud_optics%init(): array lut_extice has the wrong number of bands"
    if (any(shape(lut_ssaliq) /= shape(lut_extliq))) error_msg = "cloud_optics%init(): array lut_ssaliq isn't consistently sized"
    if (any(shape(lut_asyliq) /= shape(lut_extliq))) error_msg = "cloud_optics%init(): array lut_asyliq isn't consistently sized"
    if (any(shape(lut_ssaice) /= shape(lut_extice))) error_msg = "cloud_optics%init(): array lut_ssaice  isn't consistently sized"
    if (any(shape(lut_asyice) /= shape(lut_extice))) error_msg = "cloud_optics%init(): array lut_asyice  isn't consistently sized"
    if (error_msg /= '') return
    error_msg = rrtmgpnn_check(c_rrtmgpnn_cloud_optics_create_lut(rrtmgpnn_ctx(), nbnd, this%band_lims_wvn, &
                               size(lut_extliq, 1), size(lut_extice, 1), size(lut_extice, 3), radliq_lwr, radliq_upr, &
                               radice_lwr, radice_upr, lut_extliq, lut_ssaliq, lut_asyliq, lut_extice, lut_ssaice, &
                               lut_asyice, h), "cloud_optics%load_lut")
    if (error_msg /= '') return
    error_msg = this%adopt(h)
  end function load_lut

  ! load_pade (:179-301).  pade_*liq (nbnd, nsizereg, ncoef); pade_*ice (nbnd, nsizereg, ncoef, nrghice);
  ! size-regime boundaries (nsizereg + 1).
  function load_pade(this, band_lims_wvn, pade_extliq, pade_ssaliq, pade_asyliq, pade_extice, pade_ssaice, &
                     pade_asyice, pade_sizreg_extliq, pade_sizreg_ssaliq, pade_sizreg_asyliq, pade_sizreg_extice, &
                     pade_sizreg_ssaice, pade_sizreg_asyice) result(error_msg)
    class(ty_cloud_optics),       intent(inout) :: this
    real(wp), dimension(:,:),     intent(in)    :: band_lims_wvn
    real(wp), dimension(:,:,:),   intent(in)    :: pade_extliq, pade_ssaliq, pade_asyliq
    real(wp), dimension(:,:,:,:), intent(in)    :: pade_extice, pade_ssaice, pade_asyice
    real(wp), dimension(:),       intent(in)    :: pade_sizreg_extliq, pade_sizreg_ssaliq, pade_sizreg_asyliq
    real(wp), dimension(:),       intent(in)    :: pade_sizreg_extice, pade_sizreg_ssaice, pade_sizreg_asyice
    character(len=128) :: error_msg
    integer :: nbnd, nsizereg, nbound
    type(c_ptr) :: h

    nbnd     = size(pade_extliq, dim=1)
    nsizereg = size(pade_extliq, dim=2)
    nbound   = size(pade_sizreg_extliq)
    if (nsizereg /= 3) then
      error_msg = "cloud optics: code assumes exactly three size regimes for Pade approximants but data is otherwise"
      return
    end if
    error_msg = this%init(band_lims_wvn, name="RRTMGP cloud optics")
    if (error_msg /= '') return
    if (nbnd /= this%get_nband()) &
      error_msg = "cloud_optics%init(): number of bands inconsistent between lookup tables, spectral discretization"
    if (any(shape(pade_asyliq) /= shape(pade_ssaliq))) error_msg = "cloud_optics%init(): array pade_asyliq isn't consistently sized"
    if (size(pade_extice, 1) /= nbnd .or. size(pade_extice, 2) /= nsizereg .or. &
        size(pade_extice, 3) /= size(pade_extliq, 3)) &
      error_msg = "cloud_optics%init(): array pade_extice isn't consistently sized"
    if (any(shape(pade_ssaice) /= shape(pade_asyice))) error_msg = "cloud_optics%init(): array pade_ssaice isn't consistently sized"
    if (size(pade_sizreg_ssaliq) /= nbound .or. size(pade_sizreg_asyliq) /= nbound .or. &
        size(pade_sizreg_extice) /= nbound .or. size(pade_sizreg_ssaice) /= nbound .or. &
        size(pade_sizreg_asyice) /= nbound .or. nbound /= nsizereg + 1) &
      error_msg = "cloud_optics%init(): one or more Pade size regime arrays are inconsistently sized"
    if (error_msg /= '') return
    error_msg = rrtmgpnn_check(c_rrtmgpnn_cloud_optics_create_pade(rrtmgpnn_ctx(), nbnd, this%band_lims_wvn, &
                               nsizereg, size(pade_extliq, 3), size(pade_ssaliq, 3), size(pade_extice, 4), &
                               pade_extliq, pade_ssaliq, pade_asyliq, pade_extice, pade_ssaice, pade_asyice, &
                               pade_sizreg_extliq, pade_sizreg_ssaliq, pade_sizreg_asyliq, pade_sizreg_extice, &
                               pade_sizreg_ssaice, pade_sizreg_asyice, h), "cloud_optics%load_pade")
    if (error_msg /= '') return
    error_msg = this%adopt(h)
  end function load_pade

  ! rrtmgp-cloud-optics-coeffs-{lw,sw}.nc (classic netCDF) or its RBIN conversion, read by the library's native
  ! readers; use_lut selects load_lut or load_pade (mo_load_cloud_coefficients wraps this for the drivers).
  function load_rbin(this, filename, use_lut) result(error_msg)
    class(ty_cloud_optics), intent(inout) :: this
    character(len=*),       intent(in)    :: filename
    logical,                intent(in)    :: use_lut
    character(len=128) :: error_msg
    type(c_ptr) :: h
    integer(c_int) :: nb, nr
    real(c_float) :: radii(4)
    real(wp), allocatable :: wvn(:,:)
    error_msg = rrtmgpnn_check(c_rrtmgpnn_cloud_optics_load(rrtmgpnn_ctx(), trim(filename) // c_null_char, &
                               merge(1_c_int, 0_c_int, use_lut), h), "cloud_optics%load")
    if (error_msg /= '') return
    error_msg = rrtmgpnn_check(c_rrtmgpnn_cloud_optics_get(h, nb, nr, radii), "cloud_optics%load")
    if (error_msg /= '') return
    allocate(wvn(2, nb))
    error_msg = band_limits_of(filename, wvn)
    if (error_msg /= '') return
    error_msg = this%init(wvn, name="RRTMGP cloud optics")
    if (error_msg /= '') return
    error_msg = this%adopt(h)
  end function load_rbin

  function band_limits_of(filename, wvn) result(error_msg)
    use mo_rrtmgpnn_file, only: ty_data_file
    character(len=*), intent(in) :: filename
    real(wp), dimension(:,:), intent(out) :: wvn
    character(len=128) :: error_msg
    type(ty_data_file) :: f
    real(wp), allocatable :: a(:,:)
    error_msg = f%open(filename)
    if (error_msg /= '') return
    error_msg = f%real2("bnd_limits_wavenumber", a)
    call f%close()
    if (error_msg /= '') return
    if (any(shape(a) /= shape(wvn))) then
      error_msg = "cloud_optics%load: bnd_limits_wavenumber inconsistently sized"; return
    end if
    wvn = a
  end function band_limits_of

  ! Take ownership of a device table handle; ice roughness starts at 1 (:172, :300)
  function adopt(this, h) result(error_msg)
    class(ty_cloud_optics), intent(inout) :: this
    type(c_ptr), intent(in) :: h
    character(len=128) :: error_msg
    integer(c_int) :: nb, nr, rc
    real(c_float) :: radii(4)
    if (c_associated(this%h)) rc = c_rrtmgpnn_cloud_optics_destroy(this%h)
    this%h = h
    error_msg = rrtmgpnn_check(c_rrtmgpnn_cloud_optics_get(h, nb, nr, radii), "cloud_optics%load")
    if (error_msg /= '') return
    this%nrghice = nr
    this%radliq_lwr = radii(1); this%radliq_upr = radii(2)
    this%radice_lwr = radii(3); this%radice_upr = radii(4)
    error_msg = this%set_ice_roughness(1)
  end function adopt

  subroutine finalize(this)
    class(ty_cloud_optics), intent(inout) :: this
    integer(c_int) :: rc
    if (c_associated(this%h)) rc = c_rrtmgpnn_cloud_optics_destroy(this%h)
    this%h = c_null_ptr
    this%icergh = 0
    this%nrghice = 0
    if (allocated(this%band2gpt)) deallocate(this%band2gpt)
    if (allocated(this%band_lims_wvn)) deallocate(this%band_lims_wvn)
  end subroutine finalize

  ! cloud_optics (:354-535): clwp, ciwp [g/m2], reliq, reice [microns], all (nlay, ncol) -> optical properties
  ! by band: absorption optical depth for 1scl, tau/ssa/g for 2str.
  function cloud_optics(this, clwp, ciwp, reliq, reice, optical_props) result(error_msg)
    class(ty_cloud_optics),       intent(in)    :: this
    real(wp), dimension(:,:),     intent(in)    :: clwp, ciwp, reliq, reice
    class(ty_optical_props_arry), intent(inout) :: optical_props
    character(len=128) :: error_msg
    integer :: ncol, nlay, nbnd
    integer(c_long_long) :: n, nl
    type(c_ptr) :: d_lwp, d_iwp, d_rel, d_rei, d_tau, d_ssa, d_g

    error_msg = ''
    if (.not. c_associated(this%h)) then
      error_msg = 'cloud optics: no data has been initialized'; return
    end if
    nlay = size(clwp, 1)
    ncol = size(clwp, 2)
    nbnd = this%get_nband()
    if (size(ciwp, 1) /= nlay .or. size(ciwp, 2) /= ncol) error_msg = "cloud optics: ciwp has wrong extents"
    if (size(reliq, 1) /= nlay .or. size(reliq, 2) /= ncol) error_msg = "cloud optics: reliq has wrong extents"
    if (size(reice, 1) /= nlay .or. size(reice, 2) /= ncol) error_msg = "cloud optics: reice has wrong extents"
    if (optical_props%get_ncol() /= ncol .or. optical_props%get_nlay() /= nlay) &
      error_msg = "cloud optics: optical_props have wrong extents"
    if (error_msg /= "") return
    if (.not. this%bands_are_equal(optical_props)) &
      error_msg = "cloud optics: optical properties don't have the same band structure"
    if (optical_props%get_nband() /= optical_props%get_ngpt()) &
      error_msg = "cloud optics: optical properties must be requested by band not g-points"
    if (error_msg /= "") return
    if (check_values) then  ! :436-444
      if (any(clwp > 0._wp .and. (reliq < this%radliq_lwr .or. reliq > this%radliq_upr))) &
        error_msg = 'cloud optics: liquid effective radius is out of bounds'
      if (any(ciwp > 0._wp .and. (reice < this%radice_lwr .or. reice > this%radice_upr))) &
        error_msg = 'cloud optics: ice effective radius is out of bounds'
      if (error_msg /= "") return
    end if

    n = int(nbnd, c_long_long) * nlay * ncol
    nl = int(nlay, c_long_long) * ncol
    d_lwp = dev_stage(clwp, nl)
    d_iwp = dev_stage(ciwp, nl)
    d_rel = dev_stage(reliq, nl)
    d_rei = dev_stage(reice, nl)
    d_tau = dev_present(optical_props%tau, n, PRESENT_WRITE)
    d_ssa = c_null_ptr
    d_g   = c_null_ptr
    select type (optical_props)
    class is (ty_optical_props_2str)
      d_ssa = dev_present(optical_props%ssa, n, PRESENT_WRITE)
      d_g   = dev_present(optical_props%g, n, PRESENT_WRITE)
      optical_props%g_zero = .false.
    end select
    ! the cloud optical properties stay on the device for increment / delta_scale / the solvers
    error_msg = rrtmgpnn_check(c_rrtmgpnn_cloud_optics_compute(rrtmgpnn_ctx(), this%h, ncol, nlay, d_lwp, d_iwp, &
                               d_rel, d_rei, d_tau, d_ssa, d_g), "cloud optics")
    call dev_release(d_lwp); call dev_release(d_iwp); call dev_release(d_rel); call dev_release(d_rei)
  end function cloud_optics

  ! set_ice_roughness (:541-554)
  function set_ice_roughness(this, icergh) result(error_msg)
    class(ty_cloud_optics), intent(inout) :: this
    integer,                intent(in)    :: icergh
    character(len=128) :: error_msg
    error_msg = ""
    if (.not. c_associated(this%h)) &
      error_msg = "cloud_optics%set_ice_roughness(): can't set before initialization"
    if (icergh < 1 .or. icergh > this%get_num_ice_roughness_types()) &
      error_msg = 'cloud optics: cloud ice surface roughness flag is out of bounds'
    if (error_msg /= "") return
    error_msg = rrtmgpnn_check(c_rrtmgpnn_cloud_optics_set_ice_roughness(this%h, icergh), "set_ice_roughness")
    if (error_msg == "") this%icergh = icergh
  end function set_ice_roughness

  pure integer function get_num_ice_roughness_types(this)
    class(ty_cloud_optics), intent(in) :: this
    get_num_ice_roughness_types = this%nrghice
  end function get_num_ice_roughness_types

  pure real(wp) function get_min_radius_liq(this)
    class(ty_cloud_optics), intent(in) :: this
    get_min_radius_liq = this%radliq_lwr
  end function get_min_radius_liq

  pure real(wp) function get_max_radius_liq(this)
    class(ty_cloud_optics), intent(in) :: this
    get_max_radius_liq = this%radliq_upr
  end function get_max_radius_liq

  pure real(wp) function get_min_radius_ice(this)
    class(ty_cloud_optics), intent(in) :: this
    get_min_radius_ice = this%radice_lwr
  end function get_min_radius_ice

  pure real(wp) function get_max_radius_ice(this)
    class(ty_cloud_optics), intent(in) :: this
    get_max_radius_ice = this%radice_upr
  end function get_max_radius_ice
end module mo_cloud_optics
