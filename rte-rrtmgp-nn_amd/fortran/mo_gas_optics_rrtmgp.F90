! mo_gas_optics_rrtmgp -- drop-in for rrtmgp/mo_gas_optics_rrtmgp.F90, neural-network branch.
! ty_gas_optics_rrtmgp keeps the reference's generic `gas_optics` (gas_optics_int :239-428 for the
! longwave / internal source, gas_optics_ext :433-602 for the shortwave / external source) with the
! same arguments, error strings and optional `neural_nets`.  Inputs are staged to the device once per
! call, the whole chain (col_dry, tlev, compute_nn_inputs, fused MLP, Planck source) runs in the HIP
! kernels of librrtmgpnn.so, and the outputs come back into the caller's host arrays.
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
    type(c_ptr) :: d_totplnk = c_null_ptr
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
    if (allocated(this%totplnk)) deallocate(this%totplnk)
    if (allocated(this%solar_source)) deallocate(this%solar_source)
    call dev_free(this%d_totplnk)
    call rbin_real2(filename, "totplnk", this%totplnk, e)
    if (e == '') then
      ! totplnk_delta = (temp_ref_max - temp_ref_min) / (nPlanckTemp - 1)   (:1218)
      this%totplnk_delta = (this%temp_ref_max - this%temp_ref_min) / real(size(this%totplnk, 1) - 1, wp)
      this%d_totplnk = dev_upload(this%totplnk, size(this%totplnk))
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
  ! Device staging shared by both entry points: col_dry (given or from h2o, :347-363) and the network
  ! input tensor (compute_nn_inputs, :618-798).  On success d_coldry and d_x are device arrays the caller
  ! frees.
  function stage_inputs(nlay, ncol, play, plev, tlay, gas_desc, col_dry, net, d_play, d_plev, d_tlay, &
                        d_coldry, d_x) result(error_msg)
    integer, intent(in) :: nlay, ncol
    real(wp), dimension(:,:), intent(in) :: play, plev, tlay
    type(ty_gas_concs), intent(in) :: gas_desc
    real(wp), dimension(:,:), optional, intent(in) :: col_dry
    type(rrtmgp_network_type), intent(in) :: net
    type(c_ptr), intent(out) :: d_play, d_plev, d_tlay, d_coldry, d_x
    character(len=128) :: error_msg
    type(c_ptr) :: d_h2o, gas_ptr(MAX_INPUTS)
    integer(c_int) :: gas_nd(MAX_INPUTS)
    integer :: ninputs, k, igas, nd
    real(wp), allocatable :: h2o(:,:)
    character(len=128) :: e
    error_msg = ''
    d_play = c_null_ptr; d_plev = c_null_ptr; d_tlay = c_null_ptr; d_coldry = c_null_ptr; d_x = c_null_ptr
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
    d_play = dev_upload(play, nlay * ncol)
    d_plev = dev_upload(plev, (nlay + 1) * ncol)
    d_tlay = dev_upload(tlay, nlay * ncol)
    if (present(col_dry)) then
      d_coldry = dev_upload(col_dry, nlay * ncol)
    else
      d_coldry = dev_alloc(nlay * ncol)
      e = gas_desc%get_conc_dims_and_igas('h2o', nd, igas)
      if (e /= '') then
        error_msg = "gas_optics(): h2o concentration is required"; return
      end if
      allocate(h2o(nlay, ncol))
      h2o = spread_conc(gas_desc%concs(igas)%conc, nd, nlay, ncol)
      d_h2o = dev_upload(h2o, nlay * ncol)
      error_msg = rrtmgpnn_check(c_rrtmgpnn_get_col_dry(rrtmgpnn_ctx(), ncol, nlay, d_h2o, d_plev, d_coldry), &
                                 "get_col_dry")
      call dev_free(d_h2o)
      if (error_msg /= '') return
    end if
    gas_ptr = c_null_ptr
    gas_nd = 2
    do k = 3, ninputs
      igas = gas_desc%find_gas(net%input_names(k))
      if (igas == GAS_NOT_IN_LIST) cycle
      if (.not. allocated(gas_desc%concs(igas)%conc)) cycle
      e = gas_desc%get_conc_dims_and_igas(net%input_names(k), nd, igas)
      gas_nd(k) = nd
      gas_ptr(k) = dev_upload(gas_desc%concs(igas)%conc, size(gas_desc%concs(igas)%conc))
    end do
    d_x = dev_alloc(ninputs * nlay * ncol)
    error_msg = rrtmgpnn_check(c_rrtmgpnn_compute_nn_inputs(rrtmgpnn_ctx(), ncol, nlay, ninputs, d_play, d_tlay, &
                               gas_ptr, gas_nd, net%handle, d_x), "compute_nn_inputs")
    e = rrtmgpnn_check(c_rrtmgpnn_context_synchronize(rrtmgpnn_ctx()), "compute_nn_inputs")
    if (error_msg == '') error_msg = e
    do k = 3, ninputs
      call dev_free(gas_ptr(k))
    end do
  end function stage_inputs

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
    integer :: ncol, nlay, ngpt, nband, ninputs, n, sfc_lay
    type(c_ptr) :: d_play, d_plev, d_tlay, d_coldry, d_x, d_tsfc, d_tlev, d_tau, d_lay, d_lev, d_sfc, d_jac
    type(c_ptr) :: nets(2)
    integer(c_int), allocatable :: lims(:,:)
    character(len=128) :: e

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

    error_msg = stage_inputs(nlay, ncol, play, plev, tlay, gas_desc, col_dry, neural_nets(1), &
                             d_play, d_plev, d_tlay, d_coldry, d_x)
    if (error_msg == '') then
      if (present(tlev)) then
        d_tlev = dev_upload(tlev, (nlay + 1) * ncol)
      else
        d_tlev = dev_alloc((nlay + 1) * ncol)
        error_msg = rrtmgpnn_check(c_rrtmgpnn_interpolate_tlev(rrtmgpnn_ctx(), ncol, nlay, d_play, d_plev, d_tlay, &
                                                               d_tlev), "interpolate_tlev")
      end if
      d_tsfc = dev_upload(tsfc, ncol)
      d_tau = dev_alloc(ngpt * nlay * ncol)
      d_lay = dev_alloc(ngpt * nlay * ncol)
      d_lev = dev_alloc(ngpt * (nlay + 1) * ncol)
      d_sfc = dev_alloc(ngpt * ncol)
      d_jac = dev_alloc(ngpt * ncol)
      nets = c_null_ptr
      nets(1) = neural_nets(1)%handle
      if (n == 2) nets(2) = neural_nets(2)%handle
      if (error_msg == '') &
        error_msg = rrtmgpnn_check(c_rrtmgpnn_predict_nn_lw(rrtmgpnn_ctx(), ncol, nlay, ngpt, ninputs, d_x, d_coldry, &
                                                            nets, n, d_tau, d_lay), "predict_nn_lw")
      ! Planck source from the predicted Planck fraction (:398-404); surface at index 1 if pressure decreases
      sfc_lay = merge(1, nlay, play(1, 1) > play(nlay, 1))
      lims = this%get_band_lims_gpoint()
      if (error_msg == '') &
        error_msg = rrtmgpnn_check(c_rrtmgpnn_compute_planck_source_nn(rrtmgpnn_ctx(), ncol, nlay, nband, ngpt, &
                      this%get_nPlanckTemp(), d_tlay, d_tlev, d_tsfc, sfc_lay, lims, this%temp_ref_min, &
                      this%totplnk_delta, this%d_totplnk, d_sfc, d_jac, d_lay, d_lev), "compute_planck_source_nn")
      e = rrtmgpnn_check(c_rrtmgpnn_context_synchronize(rrtmgpnn_ctx()), "gas_optics")
      if (error_msg == '') error_msg = e
      if (error_msg == '') then
        call dev_download(optical_props%tau, d_tau, ngpt * nlay * ncol)
        call dev_download(sources%lay_source, d_lay, ngpt * nlay * ncol)
        call dev_download(sources%lev_source, d_lev, ngpt * (nlay + 1) * ncol)
        call dev_download(sources%sfc_source, d_sfc, ngpt * ncol)
        call dev_download(sources%sfc_source_Jac, d_jac, ngpt * ncol)
      end if
      call dev_free(d_tlev); call dev_free(d_tsfc); call dev_free(d_tau); call dev_free(d_lay)
      call dev_free(d_lev); call dev_free(d_sfc); call dev_free(d_jac)
    end if
    call dev_free(d_play); call dev_free(d_plev); call dev_free(d_tlay); call dev_free(d_coldry); call dev_free(d_x)
  end function gas_optics_int

  ! ---------------------------------------------------------------------------------------------------
  ! gas_optics_ext (:433-602): SW optical depth (+ Rayleigh single-scattering albedo for 2str) and the
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
    type(c_ptr) :: d_play, d_plev, d_tlay, d_coldry, d_x, d_tau, d_ssa, d_g
    type(c_ptr) :: nets(2)
    character(len=128) :: e

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
    if (.not. present(neural_nets)) then
      error_msg = "gas_optics(): the lookup-table branch is not available (k-distribution files missing); " // &
                  "pass neural_nets"
      return
    end if
    ninputs = size(neural_nets(1)%layers(1)%w_transposed, 2)
    error_msg = stage_inputs(nlay, ncol, play, plev, tlay, gas_desc, col_dry, neural_nets(1), &
                             d_play, d_plev, d_tlay, d_coldry, d_x)
    if (error_msg == '') then
      nets(1) = neural_nets(1)%handle
      nets(2) = neural_nets(2)%handle
      d_tau = dev_alloc(ngpt * nlay * ncol)
      d_ssa = c_null_ptr; d_g = c_null_ptr
      select type (optical_props)
      type is (ty_optical_props_2str)
        d_ssa = dev_alloc(ngpt * nlay * ncol)
        d_g = dev_alloc(ngpt * nlay * ncol)
      end select
      error_msg = rrtmgpnn_check(c_rrtmgpnn_predict_nn_sw(rrtmgpnn_ctx(), ncol, nlay, ngpt, ninputs, d_x, d_coldry, &
                                                          nets, d_tau, d_ssa, d_g), "predict_nn_sw")
      e = rrtmgpnn_check(c_rrtmgpnn_context_synchronize(rrtmgpnn_ctx()), "gas_optics")
      if (error_msg == '') error_msg = e
      if (error_msg == '') then
        call dev_download(optical_props%tau, d_tau, ngpt * nlay * ncol)
        select type (optical_props)
        type is (ty_optical_props_2str)
          call dev_download(optical_props%ssa, d_ssa, ngpt * nlay * ncol)
          call dev_download(optical_props%g, d_g, ngpt * nlay * ncol)
        end select
      end if
      call dev_free(d_tau); call dev_free(d_ssa); call dev_free(d_g)
    end if
    call dev_free(d_play); call dev_free(d_plev); call dev_free(d_tlay); call dev_free(d_coldry); call dev_free(d_x)
    if (error_msg /= '') return
    if (any(shape(toa_src) /= [ngpt, ncol])) then
      error_msg = "gas_optics(): array toa_src has wrong size"; return
    end if
    do icol = 1, ncol
      toa_src(:, icol) = this%solar_source(:)
    end do
  end function gas_optics_ext
end module mo_gas_optics_rrtmgp
