! devstate.F90 -- exercises the Fortran drop-in's device data environment (tests/test_fortran.py):
! gas_optics leaves tau and the (deferred) Planck sources on the device; update_host() brings them back; a host write
! followed by update_device() is what the next rte_lw reads.
! usage: devstate <problem.rbin> <output.rbin> <data_dir>
!   output: tau, lay_source, lev_source, sfc_source (as gas_optics produced them), and the LW fluxes of rte_lw run
!   twice: on the gas-optics tau (flux_up/dn_a) and on 0.5 * tau written on the host (flux_up/dn_b); then, on that
!   tau, ty_fluxes_flexible g-point fluxes with rte_lw's lw_Ds (c: lw_Ds(icol, igpt) = 1 + 0.01 mod(7 icol + igpt, 100))
!   and with three Gauss angles (d), and rte_sw on two-stream properties tau = 0.1 tau_a, ssa = 0.5, g = 0.3 over the
!   same spectral discretisation with g-point fluxes (e: mu0 = 0.6, inc_flux = 1, albedos 0.2); rte_lw on those
!   two-stream properties with g-point fluxes, rescaled (f) and use_2stream (g); rte_sw on the 1scl tau of (b) with
!   gpt_flux_dn_dir (h: the spectral direct beam); rte_lw with flux_up_Jac / flux_dn_Jac (filled with -7) on the 1scl
!   tau of (b) (i) and on the two-stream properties, rescaled (j): '' returned, the Jacobian arrays untouched (written
!   out as jac_up_i/jac_dn_i/jac_up_j/jac_dn_j), the fluxes those of (b) and (f); with use_2stream the reference's
!   message for flux_up_Jac, and '' for a lone flux_dn_Jac (the reference tests flux_up_Jac twice, :252); (k) rte_lw
!   as (b) and (l) rte_sw as (e) with flux_net associated too (the fluxes through temporaries); (m) a flux_up of the
!   transposed shape (ncol, nlay+1) and a flux_dn_dir with one level too many are refused with reduce_broadband's
!   messages (exit status 4 / 5), the caller's array untouched.
program devstate
  use mo_rte_kind,           only: wp
  use mo_optical_props,      only: ty_optical_props_1scl, ty_optical_props_2str
  use mo_source_functions,   only: ty_source_func_lw
  use mo_fluxes,             only: ty_fluxes_flexible
  use mo_gas_concentrations, only: ty_gas_concs
  use mo_gas_optics_rrtmgp,  only: ty_gas_optics_rrtmgp
  use mod_network_rrtmgp,    only: rrtmgp_network_type
  use mo_rte_lw,             only: rte_lw
  use mo_rte_sw,             only: rte_sw
  use mo_rrtmgpnn_rbin
  implicit none
  character(len=512) :: pfile, ofile, ddir
  real(wp), allocatable :: play(:,:), plev(:,:), tlay(:,:), tlev(:,:), tsfc(:), sfc_emis(:), scal(:), vmr(:,:)
  real(wp), allocatable :: emis(:,:), tau0(:,:,:), lay0(:,:,:), lev0(:,:,:), sfc0(:,:)
  real(wp), allocatable, target :: up_a(:,:), dn_a(:,:), up_b(:,:), dn_b(:,:)
  real(wp), allocatable, target :: up_c(:,:), dn_c(:,:), gup_c(:,:,:), gdn_c(:,:,:), up_d(:,:), dn_d(:,:)
  real(wp), allocatable, target :: gup_d(:,:,:), gdn_d(:,:,:), up_e(:,:), dn_e(:,:), dir_e(:,:)
  real(wp), allocatable, target :: gup_e(:,:,:), gdn_e(:,:,:), gdir_e(:,:,:)
  real(wp), allocatable, target :: up_f(:,:), dn_f(:,:), gup_f(:,:,:), gdn_f(:,:,:)
  real(wp), allocatable, target :: up_g(:,:), dn_g(:,:), gup_g(:,:,:), gdn_g(:,:,:), dir_h(:,:), gdir_h(:,:,:)
  real(wp), allocatable, target :: up_i(:,:), dn_i(:,:), up_j(:,:), dn_j(:,:)
  real(wp), allocatable, target :: jup_i(:,:), jdn_i(:,:), jup_j(:,:), jdn_j(:,:)
  real(wp), allocatable, target :: up_k(:,:), dn_k(:,:), net_k(:,:), up_l(:,:), dn_l(:,:), dir_l(:,:), net_l(:,:)
  type(ty_fluxes_flexible) :: fl6, fl7
  real(wp), allocatable, target :: bad_t(:,:), bad_l(:,:)
  type(ty_fluxes_flexible) :: fl5
  type(ty_fluxes_flexible) :: fl3, fl4
  real(wp), allocatable :: lw_ds(:,:), inc(:,:), alb(:,:), mu0(:)
  type(ty_optical_props_2str) :: op2
  type(ty_fluxes_flexible) :: fl2
  integer :: ngpt
  character(len=32), allocatable :: gas_names(:)
  type(ty_gas_concs) :: gas_concs
  type(ty_gas_optics_rrtmgp) :: kdist
  type(rrtmgp_network_type), dimension(2) :: nets
  type(ty_optical_props_1scl) :: op
  type(ty_source_func_lw) :: src
  type(ty_fluxes_flexible) :: fl
  character(len=128) :: e
  integer :: ncol, nlay, ig, icol, u
  logical :: top_at_1

  call get_command_argument(1, pfile)
  call get_command_argument(2, ofile)
  call get_command_argument(3, ddir)
  call rbin_real2(pfile, "play", play, e); call chk(e)
  call rbin_real2(pfile, "plev", plev, e); call chk(e)
  call rbin_real2(pfile, "tlay", tlay, e); call chk(e)
  call rbin_real2(pfile, "tlev", tlev, e); call chk(e)
  call rbin_real1(pfile, "tsfc", tsfc, e); call chk(e)
  call rbin_real1(pfile, "sfc_emis", sfc_emis, e); call chk(e)
  call rbin_real1(pfile, "top_at_1", scal, e); call chk(e)
  top_at_1 = scal(1) /= 0._wp
  call rbin_strings(pfile, "gas_names", gas_names, e); call chk(e)
  nlay = size(play, 1)
  ncol = size(play, 2)
  call chk(gas_concs%init(gas_names))
  do ig = 1, size(gas_names)
    call rbin_real2(pfile, "vmr_" // trim(gas_names(ig)), vmr, e); call chk(e)
    call chk(gas_concs%set_vmr(gas_names(ig), vmr))
  end do
  call nets(1)%load_netcdf(trim(ddir) // "/nn_lw_g256_abs.rbin")
  call nets(2)%load_netcdf(trim(ddir) // "/nn_lw_g256_pfrac.rbin")
  call chk(kdist%load_rbin(trim(ddir) // "/kdist_lw_g256.rbin", gas_names))
  call chk(op%alloc_1scl(ncol, nlay, kdist))
  call chk(src%alloc(ncol, nlay, kdist))
  allocate(emis(kdist%get_nband(), ncol))
  do icol = 1, ncol
    emis(:, icol) = sfc_emis(icol)
  end do
  call chk(kdist%gas_optics(play, plev, tlay, tsfc, gas_concs, op, src, tlev=tlev, neural_nets=nets))
  ! the device results, copied back
  call op%update_host()
  call src%update_host()
  tau0 = op%tau
  lay0 = src%lay_source
  lev0 = src%lev_source
  sfc0 = src%sfc_source
  allocate(up_a(nlay + 1, ncol), dn_a(nlay + 1, ncol), up_b(nlay + 1, ncol), dn_b(nlay + 1, ncol))
  fl%flux_up => up_a
  fl%flux_dn => dn_a
  call chk(rte_lw(op, top_at_1, src, emis, fl))
  ! a host write, announced with update_device, is what the solver reads next
  op%tau = 0.5_wp * op%tau
  call op%update_device()
  fl%flux_up => up_b
  fl%flux_dn => dn_b
  call chk(rte_lw(op, top_at_1, src, emis, fl))
  ! (c) lw_Ds and g-point fluxes, (d) three angles and g-point fluxes -- on the tau of (b)
  ngpt = kdist%get_ngpt()
  allocate(lw_ds(ncol, ngpt))
  do ig = 1, ngpt
    do icol = 1, ncol
      lw_ds(icol, ig) = 1._wp + 0.01_wp * real(mod(7 * icol + ig, 100), wp)
    end do
  end do
  allocate(up_c(nlay + 1, ncol), dn_c(nlay + 1, ncol), gup_c(ngpt, nlay + 1, ncol), gdn_c(ngpt, nlay + 1, ncol))
  fl%flux_up => up_c
  fl%flux_dn => dn_c
  fl%gpt_flux_up => gup_c
  fl%gpt_flux_dn => gdn_c
  call chk(rte_lw(op, top_at_1, src, emis, fl, lw_Ds=lw_ds))
  allocate(up_d(nlay + 1, ncol), dn_d(nlay + 1, ncol), gup_d(ngpt, nlay + 1, ncol), gdn_d(ngpt, nlay + 1, ncol))
  fl%flux_up => up_d
  fl%flux_dn => dn_d
  fl%gpt_flux_up => gup_d
  fl%gpt_flux_dn => gdn_d
  call chk(rte_lw(op, top_at_1, src, emis, fl, n_gauss_angles=3))
  ! (e) rte_sw with g-point fluxes
  call chk(op2%alloc_2str(ncol, nlay, kdist))
  op2%tau = 0.1_wp * tau0
  op2%ssa = 0.5_wp
  op2%g = 0.3_wp
  allocate(inc(ngpt, ncol), alb(ngpt, ncol), mu0(ncol))
  inc = 1._wp
  alb = 0.2_wp
  mu0 = 0.6_wp
  allocate(up_e(nlay + 1, ncol), dn_e(nlay + 1, ncol), dir_e(nlay + 1, ncol))
  allocate(gup_e(ngpt, nlay + 1, ncol), gdn_e(ngpt, nlay + 1, ncol), gdir_e(ngpt, nlay + 1, ncol))
  fl2%flux_up => up_e
  fl2%flux_dn => dn_e
  fl2%flux_dn_dir => dir_e
  fl2%gpt_flux_up => gup_e
  fl2%gpt_flux_dn => gdn_e
  fl2%gpt_flux_dn_dir => gdir_e
  call chk(rte_sw(op2, top_at_1, mu0, inc, alb, alb, fl2))
  ! (f), (g) rte_lw on the two-stream properties with g-point fluxes
  allocate(up_f(nlay + 1, ncol), dn_f(nlay + 1, ncol), gup_f(ngpt, nlay + 1, ncol), gdn_f(ngpt, nlay + 1, ncol))
  fl3%flux_up => up_f
  fl3%flux_dn => dn_f
  fl3%gpt_flux_up => gup_f
  fl3%gpt_flux_dn => gdn_f
  call chk(rte_lw(op2, top_at_1, src, emis, fl3))
  allocate(up_g(nlay + 1, ncol), dn_g(nlay + 1, ncol), gup_g(ngpt, nlay + 1, ncol), gdn_g(ngpt, nlay + 1, ncol))
  fl3%flux_up => up_g
  fl3%flux_dn => dn_g
  fl3%gpt_flux_up => gup_g
  fl3%gpt_flux_dn => gdn_g
  call chk(rte_lw(op2, top_at_1, src, emis, fl3, use_2stream=.true.))
  ! (h) rte_sw on the 1scl properties with the spectral direct beam
  allocate(dir_h(nlay + 1, ncol), gdir_h(ngpt, nlay + 1, ncol))
  fl4%flux_dn_dir => dir_h
  fl4%gpt_flux_dn_dir => gdir_h
  call chk(rte_sw(op, top_at_1, mu0, inc, alb, alb, fl4))
  ! (i), (j) the Jacobian arguments: accepted, untouched (compute_Jac = .false., mo_rte_rrtmgp_config.F90:28)
  allocate(up_i(nlay + 1, ncol), dn_i(nlay + 1, ncol), up_j(nlay + 1, ncol), dn_j(nlay + 1, ncol))
  allocate(jup_i(nlay + 1, ncol), jdn_i(nlay + 1, ncol), jup_j(nlay + 1, ncol), jdn_j(nlay + 1, ncol))
  jup_i = -7._wp; jdn_i = -7._wp; jup_j = -7._wp; jdn_j = -7._wp
  fl5%flux_up => up_i
  fl5%flux_dn => dn_i
  call chk(rte_lw(op, top_at_1, src, emis, fl5, flux_up_Jac=jup_i, flux_dn_Jac=jdn_i))
  fl5%flux_up => up_j
  fl5%flux_dn => dn_j
  call chk(rte_lw(op2, top_at_1, src, emis, fl5, flux_up_Jac=jup_j, flux_dn_Jac=jdn_j))
  e = rte_lw(op2, top_at_1, src, emis, fl5, use_2stream=.true., flux_up_Jac=jup_j, flux_dn_Jac=jdn_j)
  if (e /= "rte_lw: can't provide Jacobian of fluxes w.r.t surface temperature with 2-stream") then
    write(*, '(a)') "use_2stream with flux_up_Jac returned: '" // trim(e) // "'"
    error stop 2
  end if
  e = rte_lw(op2, top_at_1, src, emis, fl5, use_2stream=.true., flux_dn_Jac=jdn_j)
  if (e /= "") then
    write(*, '(a)') "use_2stream with a lone flux_dn_Jac returned: '" // trim(e) // "'"
    error stop 3
  end if
  fl5%flux_up => up_j
  fl5%flux_dn => dn_j
  call chk(rte_lw(op2, top_at_1, src, emis, fl5, flux_up_Jac=jup_j, flux_dn_Jac=jdn_j))
  ! (k) rte_lw on the tau of (b) and (l) rte_sw on the properties of (e) with flux_net wanted too: the broadband
  ! fluxes then go through temporaries (net = dn - up on the host) instead of straight into the caller's arrays
  allocate(up_k(nlay + 1, ncol), dn_k(nlay + 1, ncol), net_k(nlay + 1, ncol))
  allocate(up_l(nlay + 1, ncol), dn_l(nlay + 1, ncol), dir_l(nlay + 1, ncol), net_l(nlay + 1, ncol))
  fl6%flux_up => up_k
  fl6%flux_dn => dn_k
  fl6%flux_net => net_k
  call chk(rte_lw(op, top_at_1, src, emis, fl6))
  fl6%flux_up => up_l
  fl6%flux_dn => dn_l
  fl6%flux_dn_dir => dir_l
  fl6%flux_net => net_l
  call chk(rte_sw(op2, top_at_1, mu0, inc, alb, alb, fl6))
  ! (m) broadband arrays of the wrong shape are refused before any device work, with reduce_broadband's messages
  ! (rte/mo_fluxes.F90:143-162): the same number of elements in the transposed shape, and one level too many
  allocate(bad_t(ncol, nlay + 1), bad_l(nlay + 2, ncol))
  bad_t = -3._wp
  fl7%flux_up => bad_t
  fl7%flux_dn => dn_k
  e = rte_lw(op, top_at_1, src, emis, fl7)
  if (e /= "reduce: flux_up array incorrectly sized" .or. any(bad_t /= -3._wp)) then
    write(*, '(a)') "rte_lw with a (ncol, nlay+1) flux_up returned: '" // trim(e) // "'"
    error stop 4
  end if
  fl7%flux_up => up_k
  fl7%flux_dn_dir => bad_l
  e = rte_sw(op2, top_at_1, mu0, inc, alb, alb, fl7)
  if (e /= "reduce: flux_dn_dir array incorrectly sized") then
    write(*, '(a)') "rte_sw with a (nlay+2, ncol) flux_dn_dir returned: '" // trim(e) // "'"
    error stop 5
  end if
  u = rbin_write_begin(ofile, 48)
  call rbin_write_real(u, "flux_up_k", up_k, shape(up_k))
  call rbin_write_real(u, "flux_dn_k", dn_k, shape(dn_k))
  call rbin_write_real(u, "flux_net_k", net_k, shape(net_k))
  call rbin_write_real(u, "flux_up_l", up_l, shape(up_l))
  call rbin_write_real(u, "flux_dn_l", dn_l, shape(dn_l))
  call rbin_write_real(u, "flux_dir_l", dir_l, shape(dir_l))
  call rbin_write_real(u, "flux_net_l", net_l, shape(net_l))
  call rbin_write_real(u, "tau", tau0, shape(tau0))
  call rbin_write_real(u, "lay_source", lay0, shape(lay0))
  call rbin_write_real(u, "lev_source", lev0, shape(lev0))
  call rbin_write_real(u, "sfc_source", sfc0, shape(sfc0))
  call rbin_write_real(u, "flux_up_a", up_a, shape(up_a))
  call rbin_write_real(u, "flux_dn_a", dn_a, shape(dn_a))
  call rbin_write_real(u, "flux_up_b", up_b, shape(up_b))
  call rbin_write_real(u, "flux_dn_b", dn_b, shape(dn_b))
  call rbin_write_real(u, "flux_up_c", up_c, shape(up_c))
  call rbin_write_real(u, "flux_dn_c", dn_c, shape(dn_c))
  call rbin_write_real(u, "gpt_up_c", gup_c, shape(gup_c))
  call rbin_write_real(u, "gpt_dn_c", gdn_c, shape(gdn_c))
  call rbin_write_real(u, "flux_up_d", up_d, shape(up_d))
  call rbin_write_real(u, "flux_dn_d", dn_d, shape(dn_d))
  call rbin_write_real(u, "gpt_up_d", gup_d, shape(gup_d))
  call rbin_write_real(u, "gpt_dn_d", gdn_d, shape(gdn_d))
  call rbin_write_real(u, "flux_up_e", up_e, shape(up_e))
  call rbin_write_real(u, "flux_dn_e", dn_e, shape(dn_e))
  call rbin_write_real(u, "flux_dir_e", dir_e, shape(dir_e))
  call rbin_write_real(u, "gpt_up_e", gup_e, shape(gup_e))
  call rbin_write_real(u, "gpt_dn_e", gdn_e, shape(gdn_e))
  call rbin_write_real(u, "gpt_dir_e", gdir_e, shape(gdir_e))
  call rbin_write_real(u, "lw_ds", lw_ds, shape(lw_ds))
  call rbin_write_real(u, "flux_up_f", up_f, shape(up_f))
  call rbin_write_real(u, "flux_dn_f", dn_f, shape(dn_f))
  call rbin_write_real(u, "gpt_up_f", gup_f, shape(gup_f))
  call rbin_write_real(u, "gpt_dn_f", gdn_f, shape(gdn_f))
  call rbin_write_real(u, "flux_up_g", up_g, shape(up_g))
  call rbin_write_real(u, "flux_dn_g", dn_g, shape(dn_g))
  call rbin_write_real(u, "gpt_up_g", gup_g, shape(gup_g))
  call rbin_write_real(u, "gpt_dn_g", gdn_g, shape(gdn_g))
  call rbin_write_real(u, "flux_dir_h", dir_h, shape(dir_h))
  call rbin_write_real(u, "gpt_dir_h", gdir_h, shape(gdir_h))
  call rbin_write_real(u, "flux_up_i", up_i, shape(up_i))
  call rbin_write_real(u, "flux_dn_i", dn_i, shape(dn_i))
  call rbin_write_real(u, "flux_up_j", up_j, shape(up_j))
  call rbin_write_real(u, "flux_dn_j", dn_j, shape(dn_j))
  call rbin_write_real(u, "jac_up_i", jup_i, shape(jup_i))
  call rbin_write_real(u, "jac_dn_i", jdn_i, shape(jdn_i))
  call rbin_write_real(u, "jac_up_j", jup_j, shape(jup_j))
  call rbin_write_real(u, "jac_dn_j", jdn_j, shape(jdn_j))
  call rbin_write_end(u)
contains
  subroutine chk(msg)
    character(len=*), intent(in) :: msg
    if (len_trim(msg) > 0) then
      write(*, '(a)') trim(msg)
      error stop 1
    end if
  end subroutine chk
end program devstate
