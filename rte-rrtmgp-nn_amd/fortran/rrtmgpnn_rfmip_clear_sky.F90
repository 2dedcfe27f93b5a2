! rrtmgpnn_rfmip_clear_sky -- example host program in the shape of the reference's RFMIP drivers
! (examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90 and rrtmgp_rfmip_sw.F90, NN configuration), written
! against the drop-in modules only: the same calls a reference user makes (ty_gas_concs%set_vmr,
! load_netcdf, gas_optics(..., neural_nets=...), rte_lw, rte_sw) now run on the GPU.
!
! As there, the gas concentrations are set per block before the loop (read_and_block_gases_ty) and the blocks run
! under OpenMP (`!$omp parallel do`, rrtmgp_rfmip_lw.F90:364-367): each thread owns its optical properties and
! sources, and its own device context and stream (mo_rrtmgpnn_c), so blocks run concurrently on the GPU.
!
! usage: rrtmgpnn_rfmip_clear_sky <problem.rbin> <output.rbin> <data_dir> [block_size] [nrepeat]
!   problem.rbin: play/tlay (ncol,nlay), plev/tlev (ncol,nlay+1), tsfc/sfc_emis/sfc_alb/mu0/tsi/usecol
!   (ncol), gas_names (ngas,32) + vmr_<gas> (ncol,nlay), top_at_1 and n_gauss_angles (1).
!   output.rbin:  lw_flux_up/dn, sw_flux_up/dn/dir (ncol,nlay+1), lw_heating_rate (ncol,nlay) [K/s].
!   nrepeat > 1: the block loop runs nrepeat times; the first is a warm-up, the others are timed together and
!   reported as "timing: <ms> ms per block loop" (system_clock, as the reference drivers time theirs).
program rrtmgpnn_rfmip_clear_sky
  use mo_rte_kind,           only: wp
  use mo_optical_props,      only: ty_optical_props_1scl, ty_optical_props_2str
  use mo_source_functions,   only: ty_source_func_lw
  use mo_fluxes,             only: ty_fluxes_broadband, ty_fluxes_flexible
  use mo_gas_concentrations, only: ty_gas_concs
  use mo_gas_optics_rrtmgp,  only: ty_gas_optics_rrtmgp
  use mod_network_rrtmgp,    only: rrtmgp_network_type
  use mo_rte_lw,             only: rte_lw
  use mo_rte_sw,             only: rte_sw
  use mo_rrtmgpnn_rbin
  use mo_heating_rates, only: compute_heating_rate
  use omp_lib
  implicit none

  character(len=512) :: problem_file, output_file, data_dir, arg
  real(wp), allocatable :: play(:,:), plev(:,:), tlay(:,:), tlev(:,:), tsfc(:), sfc_emis(:), sfc_alb(:)
  real(wp), allocatable :: mu0(:), tsi(:), usecol(:), scal(:), vmr(:,:)
  character(len=32), allocatable :: gas_names(:)
  real(wp), allocatable, target :: lw_up(:,:), lw_dn(:,:), sw_up(:,:), sw_dn(:,:), sw_dir(:,:)
  real(wp), allocatable :: sfc_emis_spec(:,:), toa_flux(:,:), sfc_alb_spec(:,:), def_tsi(:), lw_hr(:,:)
  type(ty_gas_concs), allocatable :: gas_concs(:)
  type(ty_gas_optics_rrtmgp) :: kdist_lw, kdist_sw
  type(rrtmgp_network_type), dimension(2) :: nets_lw, nets_sw
  type(ty_optical_props_1scl) :: op_lw
  type(ty_optical_props_2str) :: op_sw
  type(ty_source_func_lw) :: sources
  type(ty_fluxes_flexible) :: fluxes
  character(len=128) :: e
  logical :: top_at_1
  integer :: ncol, nlay, ngas, nmus, block_size, b0, b1, nb, icol, igpt, ig, u, nblocks, b, nrepeat, rep, nb_alloc
  integer(8) :: t0, t1, rate, ts(0:6)
  ! per-section host times of thread 0 over the timed loops (printed when RRTMGPNN_SECTION_TIMES is set)
  real(8) :: sect(6)
  integer :: env_len, c0, c1, ngpt_sw
  real(wp) :: s8(8)
  real(wp), allocatable :: vmr_all(:,:,:)

  if (command_argument_count() < 3) then
    write(*, '(a)') "usage: rrtmgpnn_rfmip_clear_sky <problem.rbin> <output.rbin> <data_dir> [block_size]"
    stop 2
  end if
  call get_command_argument(1, problem_file)
  call get_command_argument(2, output_file)
  call get_command_argument(3, data_dir)
  block_size = 0
  if (command_argument_count() >= 4) then
    call get_command_argument(4, arg)
    read(arg, *) block_size
  end if
  nrepeat = 1
  if (command_argument_count() >= 5) then
    call get_command_argument(5, arg)
    read(arg, *) nrepeat
  end if

  call rbin_real2(problem_file, "play", play, e); call stop_on_err(e)
  call rbin_real2(problem_file, "plev", plev, e); call stop_on_err(e)
  call rbin_real2(problem_file, "tlay", tlay, e); call stop_on_err(e)
  call rbin_real2(problem_file, "tlev", tlev, e); call stop_on_err(e)
  call rbin_real1(problem_file, "tsfc", tsfc, e); call stop_on_err(e)
  call rbin_real1(problem_file, "sfc_emis", sfc_emis, e); call stop_on_err(e)
  call rbin_real1(problem_file, "sfc_alb", sfc_alb, e); call stop_on_err(e)
  call rbin_real1(problem_file, "mu0", mu0, e); call stop_on_err(e)
  call rbin_real1(problem_file, "tsi", tsi, e); call stop_on_err(e)
  call rbin_real1(problem_file, "usecol", usecol, e); call stop_on_err(e)
  call rbin_real1(problem_file, "top_at_1", scal, e); call stop_on_err(e)
  top_at_1 = scal(1) /= 0._wp
  call rbin_real1(problem_file, "n_gauss_angles", scal, e); call stop_on_err(e)
  nmus = nint(scal(1))
  call rbin_strings(problem_file, "gas_names", gas_names, e); call stop_on_err(e)
  nlay = size(play, 1)
  ncol = size(play, 2)
  ngas = size(gas_names)
  if (block_size <= 0) block_size = ncol

  call nets_lw(1)%load_netcdf(trim(data_dir) // "/nn_lw_g256_abs.rbin")
  call nets_lw(2)%load_netcdf(trim(data_dir) // "/nn_lw_g256_pfrac.rbin")
  call nets_sw(1)%load_netcdf(trim(data_dir) // "/nn_sw_g224_abs.rbin")
  call nets_sw(2)%load_netcdf(trim(data_dir) // "/nn_sw_g224_ray.rbin")
  call stop_on_err(kdist_lw%load_rbin(trim(data_dir) // "/kdist_lw_g256.rbin", gas_names))
  call stop_on_err(kdist_sw%load_rbin(trim(data_dir) // "/kdist_sw_g224.rbin", gas_names))
  call stop_on_err(kdist_sw%set_tsi(1361.0_wp))                  ! rrtmgp_rfmip_sw.F90:317

  allocate(lw_up(nlay + 1, ncol), lw_dn(nlay + 1, ncol), sw_up(nlay + 1, ncol), sw_dn(nlay + 1, ncol), &
           sw_dir(nlay + 1, ncol))

  ! gas concentrations by block, set once (rrtmgp_rfmip_lw.F90:270, read_and_block_gases_ty)
  nblocks = (ncol + block_size - 1) / block_size
  allocate(gas_concs(nblocks), vmr_all(nlay, ncol, ngas))
  do ig = 1, ngas
    call rbin_real2(problem_file, "vmr_" // trim(gas_names(ig)), vmr, e); call stop_on_err(e)
    vmr_all(:, :, ig) = vmr
  end do
  do b = 1, nblocks
    b0 = (b - 1) * block_size + 1
    b1 = min(ncol, b0 + block_size - 1)
    call stop_on_err(gas_concs(b)%init(gas_names))
    do ig = 1, ngas
      call stop_on_err(gas_concs(b)%set_vmr(gas_names(ig), vmr_all(:, b0:b1, ig)))
    end do
  end do

  sect = 0
  call system_clock(count_rate=rate)
  ! One parallel region for every repetition: each thread allocates its optical properties, sources and spectral
  ! boundary arrays once, for a full block, as the reference drivers allocate theirs before the block loop
  ! (rrtmgp_rfmip_sw.F90:266-309); a shorter last block re-allocates.  (Allocated per block, the ~200 MB of host arrays
  ! per thread and block were mapped and unmapped every block, and the host time per block grew with the thread count.)
  !$omp parallel default(shared) &
  !$omp   private(b, b0, b1, nb, icol, igpt, c0, c1, ngpt_sw, s8, op_lw, op_sw, sources, fluxes, sfc_emis_spec, toa_flux, sfc_alb_spec, &
  !$omp           def_tsi, rep, nb_alloc, ts)
  nb_alloc = 0
  do rep = 1, nrepeat
    !$omp barrier
    !$omp masked
    if (rep == 2) call system_clock(t0)
    !$omp end masked
    !$omp do schedule(static)
    do b = 1, nblocks
      b0 = (b - 1) * block_size + 1
      b1 = min(ncol, b0 + block_size - 1)
      nb = b1 - b0 + 1
      if (nb /= nb_alloc) then
        if (nb_alloc > 0) then
          call op_lw%finalize()
          call sources%finalize()
          call op_sw%finalize()
          deallocate(sfc_emis_spec, toa_flux, sfc_alb_spec, def_tsi)
        end if
        call stop_on_err(op_lw%alloc_1scl(nb, nlay, kdist_lw))
        call stop_on_err(sources%alloc(nb, nlay, kdist_lw))
        call stop_on_err(op_sw%alloc_2str(nb, nlay, kdist_sw))
        allocate(sfc_emis_spec(kdist_lw%get_nband(), nb))
        allocate(toa_flux(kdist_sw%get_ngpt(), nb), sfc_alb_spec(kdist_sw%get_ngpt(), nb), def_tsi(nb))
        nb_alloc = nb
      end if

      ! ---- longwave (rrtmgp_rfmip_lw.F90:385-420) ----
      call system_clock(ts(0))
      do icol = 1, nb
        sfc_emis_spec(:, icol) = sfc_emis(b0 + icol - 1)
      end do
      call stop_on_err(kdist_lw%gas_optics(play(:, b0:b1), plev(:, b0:b1), tlay(:, b0:b1), tsfc(b0:b1), gas_concs(b), &
                                           op_lw, sources, tlev=tlev(:, b0:b1), neural_nets=nets_lw))
      call system_clock(ts(1))

      ! ---- shortwave gas optics (rrtmgp_rfmip_sw.F90:370-405), issued before either solver: the networks run while
      ! the host normalises the TSI ----
      call stop_on_err(kdist_sw%gas_optics(play(:, b0:b1), plev(:, b0:b1), tlay(:, b0:b1), gas_concs(b), op_sw, &
                                           toa_flux, neural_nets=nets_sw))
      call system_clock(ts(2))
      ! def_tsi(icol) sums toa_flux(:, icol) in g-point order (rrtmgp_sw_eval_nn_rfmip.F90:365-369); eight columns at
      ! a time keep eight independent sums in flight, each in its own column's order (so the same bits)
      ngpt_sw = kdist_sw%get_ngpt()
      c0 = 1
      do while (c0 + 7 <= nb)
        s8 = 0._wp
        do igpt = 1, ngpt_sw
          do c1 = 1, 8
            s8(c1) = s8(c1) + toa_flux(igpt, c0 + c1 - 1)
          end do
        end do
        def_tsi(c0:c0 + 7) = s8
        c0 = c0 + 8
      end do
      do icol = c0, nb
        def_tsi(icol) = 0._wp
        do igpt = 1, ngpt_sw
          def_tsi(icol) = def_tsi(icol) + toa_flux(igpt, icol)
        end do
      end do
      do icol = 1, nb
        do igpt = 1, ngpt_sw
          toa_flux(igpt, icol) = toa_flux(igpt, icol) * tsi(b0 + icol - 1) / def_tsi(icol)
        end do
        sfc_alb_spec(:, icol) = sfc_alb(b0 + icol - 1)
      end do
      call system_clock(ts(3))

      ! ---- rte_sw (rrtmgp_rfmip_sw.F90:420-470), then rte_lw (rrtmgp_rfmip_lw.F90:405-420): rte_sw's host staging
      ! overlaps the two networks, and rte_lw then waits for its solver alone ----
      fluxes%flux_up => sw_up(:, b0:b1)
      fluxes%flux_dn => sw_dn(:, b0:b1)
      fluxes%flux_dn_dir => sw_dir(:, b0:b1)
      call stop_on_err(rte_sw(op_sw, top_at_1, mu0(b0:b1), toa_flux, sfc_alb_spec, sfc_alb_spec, fluxes))
      call system_clock(ts(4))
      do icol = 1, nb
        if (usecol(b0 + icol - 1) == 0._wp) then
          sw_up(:, b0 + icol - 1) = 0._wp
          sw_dn(:, b0 + icol - 1) = 0._wp
        end if
      end do
      call system_clock(ts(5))
      fluxes%flux_up => lw_up(:, b0:b1)
      fluxes%flux_dn => lw_dn(:, b0:b1)
      fluxes%flux_dn_dir => NULL()
      call stop_on_err(rte_lw(op_lw, top_at_1, sources, sfc_emis_spec, fluxes, n_gauss_angles=nmus))
      call system_clock(ts(6))
      if (rep > 1 .and. b == 1) sect = sect + real(ts(1:6) - ts(0:5), 8)
    end do
    !$omp end do
  end do
  ! the thread's private objects give their device copies back to the context's pool (`!$acc exit data`): the
  ! compiler does not finalise OpenMP private copies
  if (nb_alloc > 0) then
    call op_lw%finalize()
    call sources%finalize()
    call op_sw%finalize()
    deallocate(sfc_emis_spec, toa_flux, sfc_alb_spec, def_tsi)
  end if
  !$omp end parallel
  if (nrepeat > 1) then
    call system_clock(t1)
    write(*, '(a,f12.4,a,i0,a,i0,a,i0,a)') "rrtmgpnn_rfmip_clear_sky: timing: ", &
      1000.0d0 * real(t1 - t0, 8) / real(rate, 8) / real(nrepeat - 1, 8), " ms per block loop (", nblocks, &
      " blocks of ", block_size, " columns, ", omp_get_max_threads(), " threads)"
    call get_environment_variable("RRTMGPNN_SECTION_TIMES", length=env_len)
    if (env_len > 0) write(*, '(a,6f10.1)') "rrtmgpnn_rfmip_clear_sky: block 1 us per loop (gas_optics_lw gas_optics_sw "// &
      "toa_norm rte_sw usecol rte_lw):", 1.0d6 * sect / real(rate, 8) / real(nrepeat - 1, 8)
  end if

  ! heating rates of the longwave fluxes (extensions/mo_heating_rates), K/s
  allocate(lw_hr(nlay, ncol))
  call stop_on_err(compute_heating_rate(lw_up, lw_dn, plev, lw_hr))

  u = rbin_write_begin(output_file, 6)
  call rbin_write_real(u, "lw_flux_up", lw_up, shape(lw_up))
  call rbin_write_real(u, "lw_flux_dn", lw_dn, shape(lw_dn))
  call rbin_write_real(u, "sw_flux_up", sw_up, shape(sw_up))
  call rbin_write_real(u, "sw_flux_dn", sw_dn, shape(sw_dn))
  call rbin_write_real(u, "sw_flux_dir", sw_dir, shape(sw_dir))
  call rbin_write_real(u, "lw_heating_rate", lw_hr, shape(lw_hr))
  call rbin_write_end(u)
  write(*, '(a,i0,a,i0,a)') "rrtmgpnn_rfmip_clear_sky: ", ncol, " columns x ", nlay, " layers done"

contains
  subroutine stop_on_err(msg)
    character(len=*), intent(in) :: msg
    if (len_trim(msg) > 0) then
      write(*, '(a)') trim(msg)
      error stop 1
    end if
  end subroutine stop_on_err
end program rrtmgpnn_rfmip_clear_sky
