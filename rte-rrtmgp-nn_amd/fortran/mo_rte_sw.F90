! mo_rte_sw -- drop-in for rte/mo_rte_sw.F90 (rte_sw, :48-266; the fork passes surface albedos per
! g-point).  The optical properties are read from their device copies (mo_optical_props).  2str: the two-stream
! solver (sw_solver_2stream, rte/kernels/mo_rte_solver_kernels.F90:541-692) as one HIP kernel with the broadband
! reduction fused in; 1scl: apply_BC + sw_solver_noscat (:213-222), the direct beam only (flux_dn_dir; flux_up /
! flux_dn are left as they are, as in the reference).  ty_fluxes_flexible g-point fluxes on 2str properties
! (rrtmgpnn_sw_solver_2stream_gpt: up, total down, direct, :155-173, 228-234) and on 1scl properties the spectral
! direct beam into gpt_flux_dn_dir (rrtmgpnn_sw_solver_noscat_gpt, :155-163, 218-222).
module mo_rte_sw
  use, intrinsic :: iso_c_binding
  use mo_rte_kind,      only: wp
  use mo_optical_props, only: ty_optical_props_arry, ty_optical_props_2str
  use mo_fluxes,        only: ty_fluxes_flexible
  use mo_rte_rrtmgp_config, only: check_values
  use mo_rrtmgpnn_c
  implicit none
  private
  public :: rte_sw

contains

  function rte_sw(atmos, top_at_1, mu0, inc_flux, sfc_alb_dir_gpt, sfc_alb_dif_gpt, fluxes, inc_flux_dif) &
      result(error_msg)
    class(ty_optical_props_arry), intent(in) :: atmos
    logical,                      intent(in) :: top_at_1
    real(wp), dimension(:),       intent(in) :: mu0                 ! (ncol)
    real(wp), dimension(:,:),     intent(in) :: inc_flux, sfc_alb_dir_gpt, sfc_alb_dif_gpt   ! (ngpt, ncol)
    class(ty_fluxes_flexible), intent(inout) :: fluxes
    real(wp), dimension(:,:), optional, contiguous, target, intent(in) :: inc_flux_dif      ! (ngpt, ncol)
    character(len=128) :: error_msg
    integer :: ncol, nlay, ngpt
    integer(c_long_long) :: ng, nv, nsfc, ngv
    type(c_ptr) :: d_tau, d_ssa, d_g, d_mu0, d_inc, d_dif, d_adir, d_adif, d_up, d_dn, d_dir, d_gup, d_gdn, d_gdir
    real(wp), allocatable :: up(:,:), dn(:,:), dir(:,:)
    logical :: two_str, gpt, du, dd, dr

    ncol = atmos%get_ncol()
    nlay = atmos%get_nlay()
    ngpt = atmos%get_ngpt()
    error_msg = ""
    if (.not. fluxes%are_desired()) then
      error_msg = "rte_sw: no space allocated for fluxes"; return
    end if
    error_msg = fluxes%check_extents(nlay + 1, ncol)
    if (error_msg /= '') return
    if (associated(fluxes%gpt_flux_up)) then
      if (any(shape(fluxes%gpt_flux_up) /= [ngpt, nlay + 1, ncol])) then
        error_msg = "rte_sw: gpt_flux_up inconsistently sized"; return
      end if
    end if
    if (associated(fluxes%gpt_flux_dn)) then
      if (any(shape(fluxes%gpt_flux_dn) /= [ngpt, nlay + 1, ncol])) then
        error_msg = "rte_sw: gpt_flux_dn inconsistently sized"; return
      end if
    end if
    if (associated(fluxes%gpt_flux_dn_dir)) then
      if (any(shape(fluxes%gpt_flux_dn_dir) /= [ngpt, nlay + 1, ncol])) then
        error_msg = "rte_sw: gpt_flux_dn_dir inconsistently sized"; return
      end if
    end if
    if (size(mu0) /= ncol) then
      error_msg = "rte_sw: mu0 inconsistently sized"; return
    end if
    if (check_values) then
      if (any(mu0 < 0._wp .or. mu0 > 1._wp)) then
        error_msg = "rte_sw: one or more mu0 <= 0 or > 1"; return
      end if
    end if
    if (any(shape(inc_flux) /= [ngpt, ncol])) then
      error_msg = "rte_sw: inc_flux inconsistently sized"; return
    end if
    if (check_values) then
      if (any(inc_flux < 0._wp)) then
        error_msg = "rte_sw: one or more inc_flux < 0"; return
      end if
    end if
    if (present(inc_flux_dif)) then
      if (any(shape(inc_flux_dif) /= [ngpt, ncol])) then
        error_msg = "rte_sw: inc_flux_dif inconsistently sized"; return
      end if
      if (check_values) then
        if (any(inc_flux_dif < 0._wp)) then
          error_msg = "rte_sw: one or more inc_flux_dif < 0"; return
        end if
      end if
    end if
    if (any(shape(sfc_alb_dir_gpt) /= [ngpt, ncol])) then
      error_msg = "rte_sw: sfc_alb_dir inconsistently sized"; return
    end if
    if (check_values) then
      if (any(sfc_alb_dir_gpt < 0._wp .or. sfc_alb_dir_gpt > 1._wp)) then
        error_msg = "rte_sw: sfc_alb_dir out of bounds [0,1]"; return
      end if
    end if
    if (any(shape(sfc_alb_dif_gpt) /= [ngpt, ncol])) then
      error_msg = "rte_sw: sfc_alb_dif inconsistently sized"; return
    end if
    if (check_values) then
      if (any(sfc_alb_dif_gpt < 0._wp .or. sfc_alb_dif_gpt > 1._wp)) then
        error_msg = "rte_sw: sfc_alb_dif out of bounds [0,1]"; return
      end if
    end if

    ng = int(ngpt, c_long_long) * nlay * ncol
    nv = int(nlay + 1, c_long_long) * ncol
    nsfc = int(ngpt, c_long_long) * ncol
    d_tau = dev_present(atmos%tau, ng, PRESENT_READ)
    d_mu0 = dev_stage(mu0, int(ncol, c_long_long))
    d_inc = dev_stage(inc_flux, nsfc)
    d_adir = dev_stage(sfc_alb_dir_gpt, nsfc)
    if (same_array(sfc_alb_dir_gpt, sfc_alb_dif_gpt)) then  ! the drivers pass one array for both
      d_adif = d_adir
    else
      d_adif = dev_stage(sfc_alb_dif_gpt, nsfc)
    end if
    d_dif = c_null_ptr
    if (present(inc_flux_dif)) d_dif = dev_stage(inc_flux_dif, nsfc)
    d_up = dev_scratch(nv)
    d_dn = dev_scratch(nv)
    d_dir = dev_scratch(nv)
    gpt = fluxes%are_desired_gpt()
    ngv = int(ngpt, c_long_long) * (nlay + 1) * ncol
    d_gup = c_null_ptr
    d_gdn = c_null_ptr
    d_gdir = c_null_ptr
    two_str = .false.
    select type (atmos)
    class is (ty_optical_props_2str)
      two_str = .true.
      d_ssa = dev_present(atmos%ssa, ng, PRESENT_READ)
      d_g = c_null_ptr  ! NULL: g is identically zero (the solver takes it as a literal 0, same fluxes)
      if (.not. atmos%g_zero) d_g = dev_present(atmos%g, ng, PRESENT_READ)
      if (gpt) then
        d_gup = dev_scratch(ngv)
        d_gdn = dev_scratch(ngv)
        d_gdir = dev_scratch(ngv)
        error_msg = rrtmgpnn_check(c_rrtmgpnn_sw_solver_2stream_gpt(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                                   merge(1_c_int, 0_c_int, top_at_1), d_inc, d_dif, d_tau, d_ssa, d_g, d_mu0, &
                                   d_adir, d_adif, d_up, d_dn, d_dir, d_gup, d_gdn, d_gdir), "rte_sw: sw_solver_2stream")
      else
        error_msg = rrtmgpnn_check(c_rrtmgpnn_sw_solver_2stream(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                                   merge(1_c_int, 0_c_int, top_at_1), d_inc, d_dif, d_tau, d_ssa, d_g, d_mu0, &
                                   d_adir, d_adif, d_up, d_dn, d_dir), "rte_sw: sw_solver_2stream")
      end if
    class default
      ! 1scl: apply_BC(inc_flux, mu0) + sw_solver_noscat (:213-222): the direct beam only, no diffuse flux; with
      ! g-point outputs the spectral beam (the reference does not write gpt_flux_up / gpt_flux_dn here)
      if (gpt .and. associated(fluxes%gpt_flux_dn_dir)) d_gdir = dev_scratch(ngv)
      error_msg = rrtmgpnn_check(c_rrtmgpnn_sw_solver_noscat_gpt(rrtmgpnn_ctx(), ngpt, nlay, ncol, &
                                 merge(1_c_int, 0_c_int, top_at_1), d_inc, d_tau, d_mu0, d_dir, d_gdir), &
                                 "rte_sw: sw_solver_noscat")
    end select
    ! broadband fluxes go straight into the caller's arrays when they are contiguous (and no net flux is wanted from
    ! them); otherwise into temporaries copied after the sync
    du = .false.; dd = .false.; dr = .false.
    if (.not. associated(fluxes%flux_net)) then
      du = direct_ok(fluxes%flux_up, nv); dd = direct_ok(fluxes%flux_dn, nv); dr = direct_ok(fluxes%flux_dn_dir, nv)
    end if
    allocate(up(nlay + 1, ncol), dn(nlay + 1, ncol), dir(nlay + 1, ncol))
    if (error_msg == '') then
      if (two_str) then
        if (du) then
          call dev_copy_out(fluxes%flux_up, d_up, nv)
        else
          call dev_copy_out(up, d_up, nv)
        end if
        if (dd) then
          call dev_copy_out(fluxes%flux_dn, d_dn, nv)
        else
          call dev_copy_out(dn, d_dn, nv)
        end if
      end if
      if (dr) then
        call dev_copy_out(fluxes%flux_dn_dir, d_dir, nv)
      else
        call dev_copy_out(dir, d_dir, nv)
      end if
      if (gpt .and. two_str) then
        if (associated(fluxes%gpt_flux_up)) call dev_copy_out(fluxes%gpt_flux_up, d_gup, ngv)
        if (associated(fluxes%gpt_flux_dn)) call dev_copy_out(fluxes%gpt_flux_dn, d_gdn, ngv)
      end if
      if (gpt .and. associated(fluxes%gpt_flux_dn_dir)) call dev_copy_out(fluxes%gpt_flux_dn_dir, d_gdir, ngv)
    end if
    call rrtmgpnn_sync(error_msg, "rte_sw")
    if (error_msg == '') then
      if (associated(fluxes%flux_dn_dir) .and. .not. dr) fluxes%flux_dn_dir = dir
      if (two_str) then
        if (associated(fluxes%flux_up) .and. .not. du) fluxes%flux_up = up
        if (associated(fluxes%flux_dn) .and. .not. dd) fluxes%flux_dn = dn
        if (associated(fluxes%flux_net))  fluxes%flux_net = dn - up
      end if
    end if
    call dev_release(d_mu0); call dev_release(d_inc); call dev_release(d_dif); call dev_release(d_adir)
    if (.not. same_array(sfc_alb_dir_gpt, sfc_alb_dif_gpt)) call dev_release(d_adif)
    call dev_release(d_up); call dev_release(d_dn); call dev_release(d_dir)
    call dev_release(d_gup); call dev_release(d_gdn); call dev_release(d_gdir)
  end function rte_sw

  ! whether the device fluxes can be copied into f itself: associated, contiguous and n elements
  logical function direct_ok(f, n)
    real(wp), dimension(:,:), pointer, intent(in) :: f
    integer(c_long_long), intent(in) :: n
    direct_ok = .false.
    if (associated(f)) direct_ok = is_contiguous(f) .and. size(f, kind=c_long_long) == n
  end function direct_ok

  ! whether two dummy arrays are the same actual array (same first element, same shape)
  logical function same_array(a, b)
    real(wp), dimension(:,:), intent(in), target :: a, b
    same_array = c_associated(c_loc(a), c_loc(b)) .and. all(shape(a) == shape(b))
  end function same_array
end module mo_rte_sw
