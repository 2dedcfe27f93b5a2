! rrtmgpnn_allsky -- example host program in the shape of the reference's all-sky driver
! (examples/all-sky/rrtmgp_allsky.F90:329-446) with NN gas optics: clouds by the example's recipe, cloud
! optics by band (LUT, ice roughness 2), clouds%increment(atmos) for LW, clouds%delta_scale() then
! clouds%increment(atmos) for SW -- the same class calls a reference user makes, now on the GPU.
!
! usage: rrtmgpnn_allsky <problem.rbin> <output.rbin> <data_dir> [block_size] [nc]
!   problem.rbin / output.rbin as for rrtmgpnn_rfmip_clear_sky.  With "nc" the NN models and the cloud-optics
!   coefficients are the reference's own netCDF files, by their reference names, in data_dir (read by the
!   library's native readers: load_netcdf, load_cld_lutcoeff); otherwise their RBIN conversions.
program rrtmgpnn_allsky
  use mo_rte_kind,           only: wp
  use mo_optical_props,      only: ty_optical_props_1scl, ty_optical_props_2str
  use mo_source_functions,   only: ty_source_func_lw
  use mo_fluxes,             only: ty_fluxes_flexible
  use mo_gas_concentrations, only: ty_gas_concs
  use mo_gas_optics_rrtmgp,  only: ty_gas_optics_rrtmgp
  use mod_network_rrtmgp,    only: rrtmgp_network_type
  use mo_cloud_optics,       only: ty_cloud_optics
  use mo_load_cloud_coefficients, only: load_cld_lutcoeff
  use mo_rte_lw,             only: rte_lw
  use mo_rte_sw,             only: rte_sw
  use mo_rrtmgpnn_rbin
  implicit none

  character(len=512) :: problem_file, output_file, data_dir, arg
  real(wp), allocatable :: play(:,:), plev(:,:), tlay(:,:), tlev(:,:), tsfc(:), sfc_emis(:), sfc_alb(:)
  real(wp), allocatable :: mu0(:), tsi(:), usecol(:), scal(:), vmr(:,:)
  real(wp), allocatable :: lwp(:,:), iwp(:,:), rel(:,:), rei(:,:)
  character(len=32), allocatable :: gas_names(:)
  real(wp), allocatable, target :: lw_up(:,:), lw_dn(:,:), sw_up(:,:), sw_dn(:,:), sw_dir(:,:)
  real(wp), allocatable :: sfc_emis_spec(:,:), toa_flux(:,:), sfc_alb_spec(:,:), def_tsi(:)
  type(ty_gas_concs) :: gas_concs
  type(ty_gas_optics_rrtmgp) :: kdist_lw, kdist_sw
  type(rrtmgp_network_type), dimension(2) :: nets_lw, nets_sw
  type(ty_cloud_optics) :: cloud_optics_lw, cloud_optics_sw
  type(ty_optical_props_1scl) :: op_lw, clouds_lw
  type(ty_optical_props_2str) :: op_sw, clouds_sw
  type(ty_source_func_lw) :: sources
  type(ty_fluxes_flexible) :: fluxes
  character(len=128) :: e
  logical :: top_at_1, cloudy, nc
  real(wp) :: rel_val, rei_val
  integer :: ncol, nlay, ngas, nmus, block_size, b0, b1, nb, icol, ilay, igpt, ig, u

  if (command_argument_count() < 3) then
    write(*, '(a)') "usage: rrtmgpnn_allsky <problem.rbin> <output.rbin> <data_dir> [block_size] [nc]"
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
  nc = .false.
  if (command_argument_count() >= 5) then
    call get_command_argument(5, arg)
    nc = trim(arg) == "nc"
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

  if (nc) then  ! neural/data/ file names of the reference
    call nets_lw(1)%load_netcdf(trim(data_dir) // "/lw-g256-2018-12-04_absorption_58_58.nc")
    call nets_lw(2)%load_netcdf(trim(data_dir) // "/lw-g256-2018-12-04_planck_frac_16_16.nc")
    call nets_sw(1)%load_netcdf(trim(data_dir) // "/sw-g224-2018-12-04-absorption_16_16.nc")
    call nets_sw(2)%load_netcdf(trim(data_dir) // "/sw-g224-2018-12-04-rayleigh_16_16.nc")
  else
    call nets_lw(1)%load_netcdf(trim(data_dir) // "/nn_lw_g256_abs.rbin")
    call nets_lw(2)%load_netcdf(trim(data_dir) // "/nn_lw_g256_pfrac.rbin")
    call nets_sw(1)%load_netcdf(trim(data_dir) // "/nn_sw_g224_abs.rbin")
    call nets_sw(2)%load_netcdf(trim(data_dir) // "/nn_sw_g224_ray.rbin")
  end if
  call stop_on_err(kdist_lw%load_rbin(trim(data_dir) // "/kdist_lw_g256.rbin", gas_names))
  call stop_on_err(kdist_sw%load_rbin(trim(data_dir) // "/kdist_sw_g224.rbin", gas_names))
  call stop_on_err(kdist_sw%set_tsi(1361.0_wp))                  ! rrtmgp_rfmip_sw.F90:317
  if (nc) then  ! rrtmgp_allsky.F90:213-217
    call load_cld_lutcoeff(cloud_optics_lw, trim(data_dir) // "/rrtmgp-cloud-optics-coeffs-lw.nc")
    call load_cld_lutcoeff(cloud_optics_sw, trim(data_dir) // "/rrtmgp-cloud-optics-coeffs-sw.nc")
  else
    call stop_on_err(cloud_optics_lw%load_rbin(trim(data_dir) // "/cloud_optics_lw.rbin", .true.))
    call stop_on_err(cloud_optics_sw%load_rbin(trim(data_dir) // "/cloud_optics_sw.rbin", .true.))
  end if
  call stop_on_err(cloud_optics_lw%set_ice_roughness(2))         ! rrtmgp_allsky.F90:219
  call stop_on_err(cloud_optics_sw%set_ice_roughness(2))

  ! Clouds (rrtmgp_allsky.F90:329-350): between 100 and 900 hPa, in 2/3 of the columns
  allocate(lwp(nlay, ncol), iwp(nlay, ncol), rel(nlay, ncol), rei(nlay, ncol))
  rel_val = 0.5 * (cloud_optics_lw%get_min_radius_liq() + cloud_optics_lw%get_max_radius_liq())
  rei_val = 0.5 * (cloud_optics_lw%get_min_radius_ice() + cloud_optics_lw%get_max_radius_ice())
  do icol = 1, ncol
    do ilay = 1, nlay
      cloudy = play(ilay, icol) > 100._wp * 100._wp .and. play(ilay, icol) < 900._wp * 100._wp .and. &
               mod(icol, 3) /= 0
      lwp(ilay, icol) = merge(10._wp, 0._wp, cloudy .and. tlay(ilay, icol) > 263._wp)
      iwp(ilay, icol) = merge(10._wp, 0._wp, cloudy .and. tlay(ilay, icol) < 273._wp)
      rel(ilay, icol) = merge(rel_val, 0._wp, lwp(ilay, icol) > 0._wp)
      rei(ilay, icol) = merge(rei_val, 0._wp, iwp(ilay, icol) > 0._wp)
    end do
  end do

  allocate(lw_up(nlay + 1, ncol), lw_dn(nlay + 1, ncol), sw_up(nlay + 1, ncol), sw_dn(nlay + 1, ncol), &
           sw_dir(nlay + 1, ncol))

  do b0 = 1, ncol, block_size
    b1 = min(ncol, b0 + block_size - 1)
    nb = b1 - b0 + 1
    call stop_on_err(gas_concs%init(gas_names))
    do ig = 1, ngas
      call rbin_real2(problem_file, "vmr_" // trim(gas_names(ig)), vmr, e); call stop_on_err(e)
      call stop_on_err(gas_concs%set_vmr(gas_names(ig), vmr(:, b0:b1)))
    end do

    ! ---- longwave (rrtmgp_allsky.F90:366-404) ----
    call stop_on_err(clouds_lw%alloc_1scl(nb, nlay, cloud_optics_lw))
    call stop_on_err(cloud_optics_lw%cloud_optics(lwp(:, b0:b1), iwp(:, b0:b1), rel(:, b0:b1), rei(:, b0:b1), &
                                                  clouds_lw))
    call stop_on_err(op_lw%alloc_1scl(nb, nlay, kdist_lw))
    call stop_on_err(sources%alloc(nb, nlay, kdist_lw))
    allocate(sfc_emis_spec(kdist_lw%get_nband(), nb))
    do icol = 1, nb
      sfc_emis_spec(:, icol) = sfc_emis(b0 + icol - 1)
    end do
    call stop_on_err(kdist_lw%gas_optics(play(:, b0:b1), plev(:, b0:b1), tlay(:, b0:b1), tsfc(b0:b1), gas_concs, &
                                         op_lw, sources, tlev=tlev(:, b0:b1), neural_nets=nets_lw))
    call stop_on_err(clouds_lw%increment(op_lw))
    fluxes%flux_up => lw_up(:, b0:b1)
    fluxes%flux_dn => lw_dn(:, b0:b1)
    fluxes%flux_dn_dir => NULL()
    call stop_on_err(rte_lw(op_lw, top_at_1, sources, sfc_emis_spec, fluxes, n_gauss_angles=nmus))
    deallocate(sfc_emis_spec)

    ! ---- shortwave (rrtmgp_allsky.F90:405-446) ----
    call stop_on_err(clouds_sw%alloc_2str(nb, nlay, cloud_optics_sw))
    call stop_on_err(cloud_optics_sw%cloud_optics(lwp(:, b0:b1), iwp(:, b0:b1), rel(:, b0:b1), rei(:, b0:b1), &
                                                  clouds_sw))
    call stop_on_err(op_sw%alloc_2str(nb, nlay, kdist_sw))
    allocate(toa_flux(kdist_sw%get_ngpt(), nb), sfc_alb_spec(kdist_sw%get_ngpt(), nb), def_tsi(nb))
    call stop_on_err(kdist_sw%gas_optics(play(:, b0:b1), plev(:, b0:b1), tlay(:, b0:b1), gas_concs, op_sw, toa_flux, &
                                         neural_nets=nets_sw))
    call stop_on_err(clouds_sw%delta_scale())
    call stop_on_err(clouds_sw%increment(op_sw))
    do icol = 1, nb
      def_tsi(icol) = 0._wp
      do igpt = 1, kdist_sw%get_ngpt()
        def_tsi(icol) = def_tsi(icol) + toa_flux(igpt, icol)
      end do
      do igpt = 1, kdist_sw%get_ngpt()
        toa_flux(igpt, icol) = toa_flux(igpt, icol) * tsi(b0 + icol - 1) / def_tsi(icol)
      end do
      sfc_alb_spec(:, icol) = sfc_alb(b0 + icol - 1)
    end do
    fluxes%flux_up => sw_up(:, b0:b1)
    fluxes%flux_dn => sw_dn(:, b0:b1)
    fluxes%flux_dn_dir => sw_dir(:, b0:b1)
    call stop_on_err(rte_sw(op_sw, top_at_1, mu0(b0:b1), toa_flux, sfc_alb_spec, sfc_alb_spec, fluxes))
    do icol = 1, nb
      if (usecol(b0 + icol - 1) == 0._wp) then
        sw_up(:, b0 + icol - 1) = 0._wp
        sw_dn(:, b0 + icol - 1) = 0._wp
      end if
    end do
    deallocate(toa_flux, sfc_alb_spec, def_tsi)
  end do

  u = rbin_write_begin(output_file, 5)
  call rbin_write_real(u, "lw_flux_up", lw_up, shape(lw_up))
  call rbin_write_real(u, "lw_flux_dn", lw_dn, shape(lw_dn))
  call rbin_write_real(u, "sw_flux_up", sw_up, shape(sw_up))
  call rbin_write_real(u, "sw_flux_dn", sw_dn, shape(sw_dn))
  call rbin_write_real(u, "sw_flux_dir", sw_dir, shape(sw_dir))
  call rbin_write_end(u)
  write(*, '(a,i0,a,i0,a)') "rrtmgpnn_allsky: ", ncol, " columns x ", nlay, " layers done"

contains
  subroutine stop_on_err(msg)
    character(len=*), intent(in) :: msg
    if (len_trim(msg) > 0) then
      write(*, '(a)') trim(msg)
      error stop 1
    end if
  end subroutine stop_on_err
end program rrtmgpnn_allsky
