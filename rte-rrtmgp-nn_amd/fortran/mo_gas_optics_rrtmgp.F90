! mo_gas_optics_rrtmgp -- drop-in for rrtmgp/mo_gas_optics_rrtmgp.F90, neural-network branch.
! ty_gas_optics_rrtmgp keeps the reference's generic `gas_optics` (gas_optics_int :239-428 for the
! longwave / internal source, gas_optics_ext :433-602 for the shortwave / external source) with the
! same arguments, error strings and optional `neural_nets`.  The state arrays are copied to the device per call
! (gas_optics' `!$acc enter data copyin`, :281), gas concentrations once per set_vmr; compute_nn_inputs,
! get_col_dry and the networks run as one fused kernel (rrtmgpnn_gas_optics_{lw,sw}_nn) writing the optical
! properties' device copies, which stay there for rte_lw / rte_sw (mo_optical_props).  The longwave Planck sources
! are left to be formed inside the solver (ty_source_func_lw%planck_deferred).  Nothing waits for the device here:
! errors of the enqueued kernels surface at the next synchronising call.
! The lookup-table branch (compute_gas_optics) needs the k-distribution netCDF files that are absent
! from the reference; calling gas_optics without neural_nets returns an error string.
module mo_gas_optics_rrtmgp
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,           only: wp
  use mo_optical_props,      only: ty_optical_props, ty_optical_props_arry, ty_optical_props_1scl, &
                                   ty_optical_props_2str
  use mo_source_functions,   only: ty_source_func_lw
  use mo_gas_concentrations, only: ty_gas_concs, GAS_NOT_IN_LIST
  use mod_network_rrtmgp,    only: rrtmgp_network_type
  use mo_rrtmgpnn_c
  use mo_rrtmgpnn_rbin,      only: rbin_real1, rbin_real2, rbin_int2
  implicit none
  private

  integer, parameter :: MAX_INPUTS = 32

  type, extends(ty_optical_props), public :: ty_gas_optics_rrtmgp
    real(wp) :: press_ref_min = 0._wp, press_ref_max = 110000._wp
    real(wp) :: temp_ref_min = 0._wp, temp_ref_max = 0._wp
    real(wp) :: totplnk_delta = 0._wp
    real(wp), dimension(:,:), allocatable :: totplnk        ! (nPlanckTemp, nband)
    real(wp), dimension(:),   allocatable :: solar_source   ! (ngpt)
    character(len=32), dimension(:), allocatable :: gas_names
  contains
    procedure, public :: load_rbin
    procedure, public :: source_is_internal
    procedure, public :: source_is_external
    procedure, public :: get_ngas
    procedure, public :: get_gases
    procedure, public :: get_press_min
    procedure, public :: get_press_max
    procedure, public :: get_temp_min
    procedure, public :: get_temp_max
    procedure, public :: get_nPlanckTemp
    procedure, public :: set_tsi
    procedure, public :: gas_optics_int
    procedure, public :: gas_optics_ext
    generic,   public :: gas_optics => gas_optics_int, gas_optics_ext
  end type ty_gas_optics_rrtmgp

contains

  ! Spectral discretisation and source tables from an RBIN k-distribution file (the surrogate tables of
  ! tools/convert_reference_data.py); plays the role of load_int / load_ext (:1130-1326).
  function load_rbin(this, filename, gas_names) result(error_msg)
    class(ty_gas_optics_rrtmgp), intent(inout) :: this
    character(len=*), intent(in) :: filename
    character(len=*), dimension(:), optional, intent(in) :: gas_names
    character(len=128) :: error_msg
    real(wp), allocatable :: wvn(:,:), tmp(:)
    integer, allocatable :: gpt(:,:)
    character(len=128) :: e
    call rbin_int2(filename, "band_lims_gpt", gpt, error_msg)
    if (error_msg /= '') return
    call rbin_real2(filename, "band_lims_wvn", wvn, error_msg)
    if (error_msg /= '') return
    error_msg = this%init(wvn, gpt)
    if (error_msg /= '') return
    call rbin_real1(filename, "press_ref_min", tmp, error_msg); if (error_msg /= '') return
    this%press_ref_min = tmp(1)
    call rbin_real1(filename, "temp_ref_min", tmp, error_msg); if (error_msg /= '') return
    this%temp_ref_min = tmp(1)
    call rbin_real1(filename, "temp_ref_max", tmp, error_msg); if (error_msg /= '') return
    this%temp_ref_max = tmp(1)
    if (allocated(this%totplnk)) then
      call dev_delete(this%totplnk)
      deallocate(this%totplnk)
    end if
    if (allocated(this%solar_source)) deallocate(this%solar_source)
    call rbin_real2(filename, "totplnk", this%totplnk, e)
    if (e == '') then
      ! totplnk_delta = (temp_ref_max - temp_ref_min) / (nPlanckTemp - 1)   (:1218)
      this%totplnk_delta = (this%temp_ref_max - this%temp_ref_min) / real(size(this%totplnk, 1) - 1, wp)
    else
      call rbin_real1(filename, "solar_source", this%solar_source, e)
      if (e /= '') then
        error_msg = "load_rbin: " // trim(filename) // " holds neither totplnk nor solar_source"; return
      end if
    end if
    if (present(gas_names)) then
      this%gas_names = gas_names
    else if (.not. allocated(this%gas_names)) then
      allocate(this%gas_names(0))
    end if
  end function load_rbin

  pure logical function source_is_internal(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    source_is_internal = allocated(this%totplnk)
  end function source_is_internal

  pure logical function source_is_external(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    source_is_external = allocated(this%solar_source)
  end function source_is_external

  pure integer function get_ngas(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    get_ngas = 0
    if (allocated(this%gas_names)) get_ngas = size(this%gas_names)
  end function get_ngas

  pure function get_gases(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    character(32), dimension(get_ngas(this)) :: get_gases
    if (get_ngas(this) > 0) get_gases = this%gas_names
  end function get_gases

  pure real(wp) function get_press_min(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    get_press_min = this%press_ref_min
  end function get_press_min

  pure real(wp) function get_press_max(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    get_press_max = this%press_ref_max
  end function get_press_max

  pure real(wp) function get_temp_min(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    get_temp_min = this%temp_ref_min
  end function get_temp_min

  pure real(wp) function get_temp_max(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    get_temp_max = this%temp_ref_max
  end function get_temp_max

  pure integer function get_nPlanckTemp(this)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    get_nPlanckTemp = 0
    if (allocated(this%totplnk)) get_nPlanckTemp = size(this%totplnk, 1)
  end function get_nPlanckTemp

  ! set_tsi (:1097-1120)
  function set_tsi(this, tsi) result(error_msg)
    class(ty_gas_optics_rrtmgp), intent(inout) :: this
    real(wp), intent(in) :: tsi
    character(len=128) :: error_msg
    real(wp) :: norm
    error_msg = ''
    if (tsi < 0._wp) then
      error_msg = 'tsi out of range'
    else if (allocated(this%solar_source)) then
      norm = 1._wp / sum(this%solar_source(:))
      this%solar_source(:) = this%solar_source(:) * tsi * norm
    end if
  end function set_tsi

  ! ---------------------------------------------------------------------------------------------------
  ! Network inputs on the device, shared by both entry points: the gas concentrations of inputs 3.. (their device
  ! copies, cached per set_vmr), h2o as a (nlay, ncol) array for get_col_dry (:347-363).  On success d_h2o must be
  ! released by the caller when h2o_tmp is set.
  function gas_inputs(nlay, ncol, gas_desc, net, gas_ptr, gas_nd, d_h2o, h2o_tmp) result(error_msg)
    integer, intent(in) :: nlay, ncol
    type(ty_gas_concs), intent(in) :: gas_desc
    type(rrtmgp_network_type), intent(in) :: net
    type(c_ptr), intent(out) :: gas_ptr(MAX_INPUTS), d_h2o
    integer(c_int), intent(out) :: gas_nd(MAX_INPUTS)
    logical, intent(out) :: h2o_tmp
    character(len=128) :: error_msg
    integer :: ninputs, k, igas, nd
    real(wp), allocatable :: h2o(:,:)
    character(len=128) :: e
    error_msg = ''
    gas_ptr = c_null_ptr
    gas_nd = 2
    d_h2o = c_null_ptr
    h2o_tmp = .false.
    ninputs = size(net%layers(1)%w_transposed, 2)
    if (ninputs > MAX_INPUTS .or. ninputs < 3) then
      error_msg = "compute_nn_inputs: unsupported number of network inputs"; return
    end if
    if (.not. allocated(net%input_names)) then
      error_msg = "compute_nn_inputs: network has no input_names"; return
    end if
    do k = 3, min(4, ninputs)
      if (gas_desc%find_gas(net%input_names(k)) == GAS_NOT_IN_LIST) then
        error_msg = "compute_nn_inputs: gas " // trim(net%input_names(k)) // " not found"; return
      end if
    end do
    e = gas_desc%get_conc_dims_and_igas('h2o', nd, igas)
    if (e /= '') then
      error_msg = "gas_optics(): h2o concentration is required"; return
    end if
    if (nd == 2) then
      d_h2o = gas_desc%device_conc(igas)
    else
      allocate(h2o(nlay, ncol))
      h2o = spread_conc(gas_desc%concs(igas)%conc, nd, nlay, ncol)
      d_h2o = dev_stage(h2o, int(nlay, c_long_long) * ncol)
      h2o_tmp = .true.
    end if
    do k = 3, ninputs
      igas = gas_desc%find_gas(net%input_names(k))
      if (igas == GAS_NOT_IN_LIST) cycle  ! missing gases are zero (quirk B-2)
      if (.not. allocated(gas_desc%concs(igas)%conc)) cycle
      e = gas_desc%get_conc_dims_and_igas(net%input_names(k), nd, igas)
      gas_nd(k) = nd
      gas_ptr(k) = gas_desc%device_conc(igas)
    end do
  end function gas_inputs

  function spread_conc(conc, nd, nlay, ncol) result(full)
    real(wp), dimension(:,:), intent(in) :: conc
    integer, intent(in) :: nd, nlay, ncol
    real(wp) :: full(nlay, ncol)
    integer :: icol
    select case (nd)
    case (0)
      full = conc(1, 1)
    case (1)
      do icol = 1, ncol
        full(:, icol) = conc(:, 1)
      end do
    case default
      full = conc
    end select
  end function spread_conc

  ! compute_nn_inputs + get_col_dry (or the caller's col_dry) as separate kernels into scratch buffers: the path
  ! of a user col_dry= (the fused kernels form the column amounts from h2o themselves)
  function staged_nn_inputs(nlay, ncol, net, d_play, d_tlay, gas_ptr, gas_nd, col_dry, d_x, d_cd) result(error_msg)
    integer, intent(in) :: nlay, ncol
    type(rrtmgp_network_type), intent(in) :: net
    type(c_ptr), intent(in) :: d_play, d_tlay, gas_ptr(MAX_INPUTS)
    integer(c_int), intent(in) :: gas_nd(MAX_INPUTS)
    real(wp), dimension(:,:), intent(in) :: col_dry
    type(c_ptr), intent(out) :: d_x, d_cd
    character(len=128) :: error_msg
    integer :: ninputs
    ninputs = size(net%layers(1)%w_transposed, 2)
    d_cd = dev_stage(col_dry, int(nlay, c_long_long) * ncol)
    d_x = dev_scratch(int(ninputs, c_long_long) * nlay * ncol)
    error_msg = rrtmgpnn_check(c_rrtmgpnn_compute_nn_inputs(rrtmgpnn_ctx(), ncol, nlay, ninputs, d_play, d_tlay, &
                               gas_ptr, gas_nd, net%handle, d_x), "compute_nn_inputs")
  end function staged_nn_inputs

  ! ---------------------------------------------------------------------------------------------------
  ! gas_optics_int (:239-428): LW optical depth and Planck sources.
  function gas_optics_int(this, play, plev, tlay, tsfc, gas_desc, optical_props, sources, col_dry, tlev, &
                          neural_nets) result(error_msg)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    real(wp), dimension(:,:), intent(in) :: play, plev, tlay
    real(wp), dimension(:),   intent(in) :: tsfc
    type(ty_gas_concs),       intent(in) :: gas_desc
    class(ty_optical_props_arry), intent(inout) :: optical_props
    class(ty_source_func_lw),     intent(inout) :: sources
    real(wp), dimension(:,:), intent(in), optional :: col_dry
    real(wp), dimension(:,:), intent(in), optional :: tlev
    type(rrtmgp_network_type), dimension(:), intent(in), optional :: neural_nets
    character(len=128) :: error_msg
    integer :: ncol, nlay, ngpt, nband, ninputs, n
    integer(c_long_long) :: nl, nv, ng
    type(c_ptr) :: d_play, d_plev, d_tlay, d_tlev, d_tsfc, d_tau, d_pf, d_h2o, d_x, d_cd
    type(c_ptr) :: nets(2), gas_ptr(MAX_INPUTS)
    integer(c_int) :: gas_nd(MAX_INPUTS)
    logical :: h2o_tmp

    ncol  = size(play, dim=2)
    nlay  = size(play, dim=1)
    ngpt  = this%get_ngpt()
    nband = this%get_nband()
    error_msg = ''
    if (any(shape(play) /= [nlay, ncol]))     error_msg = "gas_optics(): array play has wrong size"
    if (any(shape(tlay) /= [nlay, ncol]))     error_msg = "gas_optics(): array tlay has wrong size"
    if (any(shape(plev) /= [nlay + 1, ncol])) error_msg = "gas_optics(): array plev has wrong size"
    if (size(tsfc) /= ncol)                   error_msg = "gas_optics(): array tsfc has wrong size"
    if (present(tlev)) then
      if (any(shape(tlev) /= [nlay + 1, ncol])) error_msg = "gas_optics(): array tlev has wrong size"
    end if
    if (present(col_dry)) then
      if (any(shape(col_dry) /= [nlay, ncol])) error_msg = "gas_optics(): array col_dry has wrong size"
    end if
    if (any([sources%get_ncol(), sources%get_nlay(), sources%get_ngpt()] /= [ncol, nlay, ngpt])) &
      error_msg = "gas_optics%gas_optics: source function arrays inconsistently sized"
    if (any([optical_props%get_ncol(), optical_props%get_nlay(), optical_props%get_ngpt()] /= [ncol, nlay, ngpt])) &
      error_msg = "gas_optics(): optical properties inconsistently sized"
    if (.not. this%source_is_internal()) error_msg = "gas_optics(): this k-distribution has no internal source"
    if (error_msg /= '') return
    if (.not. present(neural_nets)) then
      error_msg = "gas_optics(): the lookup-table branch is not available (k-distribution files missing); " // &
                  "pass neural_nets"
      return
    end if
    n = size(neural_nets)
    if (n < 1 .or. n > 2) then
      error_msg = "gas_optics(): neural_nets must hold 1 (combined) or 2 (absorption, Planck fraction) models"
      return
    end if
    ninputs = size(neural_nets(1)%layers(1)%w_transposed, 2)
    error_msg = gas_inputs(nlay, ncol, gas_desc, neural_nets(1), gas_ptr, gas_nd, d_h2o, h2o_tmp)
    if (error_msg /= '') return
    nl = int(nlay, c_long_long) * ncol
    nv = int(nlay + 1, c_long_long) * ncol
    ng = int(ngpt, c_long_long) * nlay * ncol

    ! the temperatures the deferred Planck sources need live on in the source object's device copies
    call keep_shape2(sources%pk_tlay, nlay, ncol)
    call keep_shape2(sources%pk_tlev, nlay + 1, ncol)
    if (allocated(sources%pk_tsfc)) then
      if (size(sources%pk_tsfc) /= ncol) deallocate(sources%pk_tsfc)
    end if
    if (.not. allocated(sources%pk_tsfc)) allocate(sources%pk_tsfc(ncol))
    d_tlay = dev_present(sources%pk_tlay, nl, PRESENT_WRITE)
    call dev_copy_in(d_tlay, tlay, nl)
    d_tsfc = dev_present(sources%pk_tsfc, int(ncol, c_long_long), PRESENT_WRITE)
    call dev_copy_in(d_tsfc, tsfc, int(ncol, c_long_long))
    d_play = dev_stage(play, nl)
    d_plev = dev_stage(plev, nv)
    d_tlev = dev_present(sources%pk_tlev, nv, PRESENT_WRITE)
    if (present(tlev)) then
      call dev_copy_in(d_tlev, tlev, nv)
    else  ! level temperatures interpolated from the layers (:317-337)
      error_msg = rrtmgpnn_check(c_rrtmgpnn_interpolate_tlev(rrtmgpnn_ctx(), ncol, nlay, d_play, d_plev, d_tlay, &
                                                             d_tlev), "interpolate_tlev")
    end if
    d_tau = dev_present(optical_props%tau, ng, PRESENT_WRITE)
    d_pf = dev_present(sources%lay_source, ng, PRESENT_WRITE)  ! the Planck fraction until the sources are formed
    nets = c_null_ptr
    nets(1) = neural_nets(1)%handle
    if (n == 2) nets(2) = neural_nets(2)%handle
    if (error_msg == '') then
      if (present(col_dry)) then  ! B-3 fixed: the caller's column amounts are used (:342-346)
        error_msg = staged_nn_inputs(nlay, ncol, neural_nets(1), d_play, d_tlay, gas_ptr, gas_nd, col_dry, d_x, d_cd)
        if (error_msg == '') &
          error_msg = rrtmgpnn_check(c_rrtmgpnn_predict_nn_lw(rrtmgpnn_ctx(), ncol, nlay, ngpt, ninputs, d_x, d_cd, &
                                                              nets, n, d_tau, d_pf), "predict_nn_lw")
        call dev_release(d_x)
        call dev_release(d_cd)
      else  ! compute_nn_inputs + get_col_dry + predict_nn_lw_blas in one kernel (:342-391)
        error_msg = rrtmgpnn_check(c_rrtmgpnn_gas_optics_lw_nn(rrtmgpnn_ctx(), ncol, nlay, ngpt, ninputs, d_play, &
                                   d_tlay, d_plev, d_h2o, gas_ptr, gas_nd, nets, n, d_tau, d_pf), "gas_optics_lw_nn")
      end if
    end if
    call dev_release(d_play)
    call dev_release(d_plev)
    if (h2o_tmp) call dev_release(d_h2o)
    if (error_msg /= '') return
    ! Planck source from the predicted Planck fraction (:398-404), deferred to the solver; surface at index 1 if
    ! pressure decreases with index
    sources%planck_deferred = .true.
    sources%pk_sfc_lay = merge(1, nlay, play(1, 1) > play(nlay, 1))
    sources%pk_ntemp = this%get_nPlanckTemp()
    sources%pk_tmin = this%temp_ref_min
    sources%pk_tdelta = this%totplnk_delta
    sources%pk_totplnk = dev_present(this%totplnk, size(this%totplnk, kind=c_long_long), PRESENT_READ)
  end function gas_optics_int

  subroutine keep_shape2(a, n1, n2)
    real(wp), allocatable, intent(inout) :: a(:,:)
    integer, intent(in) :: n1, n2
    if (allocated(a)) then
      if (size(a, 1) /= n1 .or. size(a, 2) /= n2) then
        call dev_delete(a)
        deallocate(a)
      end if
    end if
    if (.not. allocated(a)) allocate(a(n1, n2))
  end subroutine keep_shape2

  ! ---------------------------------------------------------------------------------------------------
  ! gas_optics_ext (:433-602): SW optical depth (+ Rayleigh single-scattering albedo for 2str, g = 0) and the
  ! top-of-atmosphere source.
  function gas_optics_ext(this, play, plev, tlay, gas_desc, optical_props, toa_src, col_dry, neural_nets) &
      result(error_msg)
    class(ty_gas_optics_rrtmgp), intent(in) :: this
    real(wp), dimension(:,:), intent(in) :: play, plev, tlay
    type(ty_gas_concs),       intent(in) :: gas_desc
    class(ty_optical_props_arry), intent(inout) :: optical_props
    real(wp), dimension(:,:), intent(out) :: toa_src
    real(wp), dimension(:,:), intent(in), optional :: col_dry
    type(rrtmgp_network_type), dimension(2), intent(in), optional :: neural_nets
    character(len=128) :: error_msg
    integer :: ncol, nlay, ngpt, ninputs, icol
    integer(c_long_long) :: nl, nv, ng
    type(c_ptr) :: d_play, d_plev, d_tlay, d_tau, d_ssa, d_h2o, d_x, d_cd
    type(c_ptr) :: nets(2), gas_ptr(MAX_INPUTS)
    integer(c_int) :: gas_nd(MAX_INPUTS)
    logical :: h2o_tmp

    ncol = size(play, dim=2)
    nlay = size(play, dim=1)
    ngpt = this%get_ngpt()
    error_msg = ''
    if (any(shape(play) /= [nlay, ncol]))     error_msg = "gas_optics(): array play has wrong size"
    if (any(shape(tlay) /= [nlay, ncol]))     error_msg = "gas_optics(): array tlay has wrong size"
    if (any(shape(plev) /= [nlay + 1, ncol])) error_msg = "gas_optics(): array plev has wrong size"
    if (present(col_dry)) then
      if (any(shape(col_dry) /= [nlay, ncol])) error_msg = "gas_optics(): array col_dry has wrong size"
    end if
    if (any([optical_props%get_ncol(), optical_props%get_nlay(), optical_props%get_ngpt()] /= [ncol, nlay, ngpt])) &
      error_msg = "gas_optics(): optical properties inconsistently sized"
    if (.not. this%source_is_external()) error_msg = "gas_optics(): this k-distribution has no external source"
    if (error_msg /= '') return
    if (any(shape(toa_src) /= [ngpt, ncol])) then
      error_msg = "gas_optics(): array toa_src has wrong size"; return
    end if
    if (.not. present(neural_nets)) then
      error_msg = "gas_optics(): the lookup-table branch is not available (k-distribution files missing); " // &
                  "pass neural_nets"
      return
    end if
    ninputs = size(neural_nets(1)%layers(1)%w_transposed, 2)
    error_msg = gas_inputs(nlay, ncol, gas_desc, neural_nets(1), gas_ptr, gas_nd, d_h2o, h2o_tmp)
    if (error_msg /= '') return
    nl = int(nlay, c_long_long) * ncol
    nv = int(nlay + 1, c_long_long) * ncol
    ng = int(ngpt, c_long_long) * nlay * ncol
    d_play = dev_stage(play, nl)
    d_plev = dev_stage(plev, nv)
    d_tlay = dev_stage(tlay, nl)
    nets(1) = neural_nets(1)%handle
    nets(2) = neural_nets(2)%handle
    d_tau = dev_present(optical_props%tau, ng, PRESENT_WRITE)
    d_ssa = c_null_ptr
    select type (optical_props)
    type is (ty_optical_props_2str)
      d_ssa = dev_present(optical_props%ssa, ng, PRESENT_WRITE)
    end select
    if (present(col_dry)) then
      error_msg = staged_nn_inputs(nlay, ncol, neural_nets(1), d_play, d_tlay, gas_ptr, gas_nd, col_dry, d_x, d_cd)
      if (error_msg == '') &
        error_msg = rrtmgpnn_check(c_rrtmgpnn_predict_nn_sw(rrtmgpnn_ctx(), ncol, nlay, ngpt, ninputs, d_x, d_cd, &
                                                            nets, d_tau, d_ssa, c_null_ptr), "predict_nn_sw")
      call dev_release(d_x)
      call dev_release(d_cd)
    else
      error_msg = rrtmgpnn_check(c_rrtmgpnn_gas_optics_sw_nn(rrtmgpnn_ctx(), ncol, nlay, ngpt, ninputs, d_play, d_tlay, &
                                 d_plev, d_h2o, gas_ptr, gas_nd, nets, d_tau, d_ssa, c_null_ptr), "gas_optics_sw_nn")
    end if
    call dev_release(d_play)
    call dev_release(d_plev)
    call dev_release(d_tlay)
    if (h2o_tmp) call dev_release(d_h2o)
    if (error_msg /= '') return
    select type (optical_props)
    type is (ty_optical_props_2str)
      optical_props%g_zero = .true.  ! g = 0 (:560-567), left implicit on the device
    end select
    do icol = 1, ncol
      toa_src(:, icol) = this%solar_source(:)
    end do
  end function gas_optics_ext
end module mo_gas_optics_rrtmgp
