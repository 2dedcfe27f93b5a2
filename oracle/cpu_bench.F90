! cpu_bench.F90 -- BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg; never shipped, never linked by the product).
!
! The reference's CPU path timed the way its own RFMIP drivers run it: an OpenMP loop over blocks of columns
! (examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:364-446, `!$OMP PARALLEL firstprivate(...)` / `!$OMP DO`), each
! thread owning its optical-property, source and flux objects (allocated once per thread, :326-327), each block
! running gas optics -> rte_lw and gas optics -> rte_sw (rrtmgp_rfmip_sw.F90:370-470).  Built by
! oracle/Makefile.ref against the reference's own compiled modules:
!   rte_lw, rte_sw, ty_optical_props_*, ty_source_func_lw  (rte/, compiled from the reference's sources)
!   network_type%output_sgemm_flat + MKL sgemm (sequential)  (neural/mod_network.F90:273-354)
!   ty_cloud_optics%cloud_optics, %increment, %delta_scale  (extensions/cloud_optics, rte/mo_optical_props.F90)
! The NN gas-optics glue (compute_nn_inputs, get_col_dry, the output scaling, compute_Planck_source_nn) lives in
! mo_gas_optics_rrtmgp / mo_gas_optics_kernels, which need netcdf-fortran and cannot be built here: it is called from
! the C restatement (oracle/librrtmgpnn_oracle.so), bit-identical to the GPU path and < 5 % of the CPU time.
!
! usage: rrtmgp_cpu_bench <problem.rbin> <data_dir> <threads> <block> <columns per run> <sw 0|1> <reps>
!   problem.rbin: the Fortran example's problem format (play, plev, tlay, tlev, tsfc, sfc_emis, sfc_alb, mu0, tsi,
!   top_at_1, gas_names + vmr_<gas>), plus clwp, ciwp, rel, rei (nlay, ncol) for the all-sky step.
!   Blocks cycle through the problem's columns: block b covers columns mod(b*block, ncol) + 1 ... + block
!   (ncol must be a multiple of block, as the reference driver requires, rrtmgp_rfmip_lw.F90:213).
! After one untimed pass over the problem's columns, prints one JSON line: {"threads", "nproc", "block",
! "columns", "seconds": [one per rep]}.  With an 8th argument
! <fluxes.rbin>, the last rep also stores every block's broadband fluxes there (lw_flux_up/dn, sw_flux_up/dn/dir as
! (ncol, nlay+1)) so tests/test_cpu_bench.py can check the driver against the oracle.
module cpu_bench_glue
  use, intrinsic :: iso_c_binding
  implicit none
  interface
    ! oracle/rrtmgpnn_oracle.c (each cites the reference routine it restates)
    subroutine orc_compute_nn_inputs(ncol, nlay, nx, play, tlay, gas, gas_ndims, in_min, in_max, nn_inputs) &
        bind(C, name="orc_compute_nn_inputs")
      import :: c_int, c_ptr, c_float
      integer(c_int), value :: ncol, nlay, nx
      type(c_ptr), value :: play, tlay
      type(c_ptr), intent(in) :: gas(*)
      integer(c_int), intent(in) :: gas_ndims(*)
      real(c_float), intent(in) :: in_min(*), in_max(*)
      real(c_float), intent(out) :: nn_inputs(*)
    end subroutine
    subroutine orc_get_col_dry(ncol, nlay, vmr_h2o, plev, col_dry) bind(C, name="orc_get_col_dry")
      import :: c_int, c_ptr, c_float
      integer(c_int), value :: ncol, nlay
      type(c_ptr), value :: vmr_h2o, plev
      real(c_float), intent(out) :: col_dry(*)
    end subroutine
    subroutine orc_nn_tau_post(ngpt, nbatch, y, mean, std, coldry, tau_abs_to_tot) bind(C, name="orc_nn_tau_post")
      import :: c_int, c_long, c_ptr, c_float
      integer(c_int), value :: ngpt
      integer(c_long), value :: nbatch
      real(c_float), intent(inout) :: y(*)
      real(c_float), intent(in) :: mean(*), std(*), coldry(*)
      type(c_ptr), value :: tau_abs_to_tot
    end subroutine
    subroutine orc_square(n, y) bind(C, name="orc_square")
      import :: c_long, c_float
      integer(c_long), value :: n
      real(c_float), intent(inout) :: y(*)
    end subroutine
    subroutine orc_planck_source_nn(ncol, nlay, nbnd, ngpt, ntemp, tlay, tlev, tsfc, sfc_lay, band_lims_gpt, &
        temp_ref_min, totplnk_delta, totplnk, sfc_source, sfc_source_Jac, pfrac, lev_source) &
        bind(C, name="orc_planck_source_nn")
      import :: c_int, c_ptr, c_float
      integer(c_int), value :: ncol, nlay, nbnd, ngpt, ntemp, sfc_lay
      type(c_ptr), value :: tlay, tlev, tsfc
      integer(c_int), intent(in) :: band_lims_gpt(*)
      real(c_float), value :: temp_ref_min, totplnk_delta
      real(c_float), intent(in) :: totplnk(*)
      real(c_float), intent(out) :: sfc_source(*), sfc_source_Jac(*), lev_source(*)
      real(c_float), intent(inout) :: pfrac(*)
    end subroutine
  end interface
end module cpu_bench_glue

program rrtmgp_cpu_bench
  use, intrinsic :: iso_c_binding
  use omp_lib
  use mo_rte_kind,         only: wp
  use mo_optical_props,    only: ty_optical_props_1scl, ty_optical_props_2str
  use mo_source_functions, only: ty_source_func_lw
  use mo_fluxes,           only: ty_fluxes_flexible
  use mo_rte_lw,           only: rte_lw
  use mo_rte_sw,           only: rte_sw
  use mod_network,         only: network_type
  use mo_cloud_optics,     only: ty_cloud_optics
  use mo_rrtmgpnn_rbin
  use cpu_bench_glue
  implicit none

  character(len=512) :: pfile, ddir, arg
  integer :: nthreads, block, ncols_run, do_sw, nreps, rep, nblocks, ncol, nlay, ngas, k
  real(wp), allocatable, target :: play(:,:), plev(:,:), tlay(:,:), tlev(:,:), tsfc(:), sfc_emis(:), sfc_alb(:), &
                                   mu0(:), tsi(:), scal(:)
  real(wp), allocatable, target :: clwp(:,:), ciwp(:,:), rel(:,:), rei(:,:)
  character(len=32), allocatable :: gas_names(:)
  type :: gas_field
    real(wp), allocatable :: v(:,:)
  end type
  type(gas_field), allocatable, target :: vmr(:)
  ! one NN model: the network and compute_nn_inputs / output scaling data
  type :: nn_model
    type(network_type) :: net
    integer :: nx, ny
    real(wp), allocatable :: in_min(:), in_max(:), out_mean(:), out_std(:)
    integer, allocatable :: gas_idx(:)   ! index into vmr(:) of each input k >= 3, 0 = missing (ref_vmr = 0)
  end type
  type(nn_model) :: lw_abs, lw_pf, sw_abs, sw_ray
  integer, allocatable :: lims_lw(:,:), lims_sw(:,:)
  real(wp), allocatable :: wvn_lw(:,:), wvn_sw(:,:), totplnk(:,:), solar(:)
  real(wp) :: tmin_lw, tdelta_lw, def_tsi
  type(ty_cloud_optics) :: co_lw, co_sw
  logical :: top_at_1, allsky
  real(8), allocatable :: secs(:), starts(:)
  real(8) :: t0, tfirst
  character(len=128) :: e
  character(len=512) :: ofile
  character(len=32) :: num
  character(len=:), allocatable :: line
  logical :: keep
  real(wp), allocatable :: o_lwu(:,:), o_lwd(:,:), o_swu(:,:), o_swd(:,:), o_swr(:,:)
  integer :: u

  if (command_argument_count() < 7) then
    write(*, '(a)') "usage: rrtmgp_cpu_bench <problem.rbin> <data_dir> <threads> <block> <columns> <sw 0|1> <reps>"
    stop 2
  end if
  call get_command_argument(1, pfile)
  call get_command_argument(2, ddir)
  call get_command_argument(3, arg); read(arg, *) nthreads
  call get_command_argument(4, arg); read(arg, *) block
  call get_command_argument(5, arg); read(arg, *) ncols_run
  call get_command_argument(6, arg); read(arg, *) do_sw
  call get_command_argument(7, arg); read(arg, *) nreps
  ofile = ''
  if (command_argument_count() >= 8) call get_command_argument(8, ofile)

  call rbin_real2(pfile, "play", play, e); call chk(e)
  call rbin_real2(pfile, "plev", plev, e); call chk(e)
  call rbin_real2(pfile, "tlay", tlay, e); call chk(e)
  call rbin_real2(pfile, "tlev", tlev, e); call chk(e)
  call rbin_real1(pfile, "tsfc", tsfc, e); call chk(e)
  call rbin_real1(pfile, "sfc_emis", sfc_emis, e); call chk(e)
  call rbin_real1(pfile, "sfc_alb", sfc_alb, e); call chk(e)
  call rbin_real1(pfile, "mu0", mu0, e); call chk(e)
  call rbin_real1(pfile, "tsi", tsi, e); call chk(e)
  call rbin_real1(pfile, "top_at_1", scal, e); call chk(e)
  top_at_1 = scal(1) /= 0._wp
  call rbin_strings(pfile, "gas_names", gas_names, e); call chk(e)
  nlay = size(play, 1)
  ncol = size(play, 2)
  ngas = size(gas_names)
  allocate(vmr(ngas))
  do k = 1, ngas
    call rbin_real2(pfile, "vmr_" // trim(gas_names(k)), vmr(k)%v, e); call chk(e)
  end do
  call rbin_real2(pfile, "clwp", clwp, e)
  allsky = e == ''
  if (allsky) then
    call rbin_real2(pfile, "ciwp", ciwp, e); call chk(e)
    call rbin_real2(pfile, "rel", rel, e); call chk(e)
    call rbin_real2(pfile, "rei", rei, e); call chk(e)
  end if
  if (mod(ncol, block) /= 0) call chk("rrtmgp_cpu_bench: number of columns doesn't fit evenly into blocks")
  nblocks = max(1, ncols_run / block)

  call load_model(trim(ddir) // "/nn_lw_g256_abs.rbin", lw_abs)
  call load_model(trim(ddir) // "/nn_lw_g256_pfrac.rbin", lw_pf)
  call load_model(trim(ddir) // "/nn_sw_g224_abs.rbin", sw_abs)
  call load_model(trim(ddir) // "/nn_sw_g224_ray.rbin", sw_ray)
  call rbin_int2(trim(ddir) // "/kdist_lw_g256.rbin", "band_lims_gpt", lims_lw, e); call chk(e)
  call rbin_real2(trim(ddir) // "/kdist_lw_g256.rbin", "band_lims_wvn", wvn_lw, e); call chk(e)
  call rbin_real2(trim(ddir) // "/kdist_lw_g256.rbin", "totplnk", totplnk, e); call chk(e)
  call rbin_real1(trim(ddir) // "/kdist_lw_g256.rbin", "temp_ref_min", scal, e); call chk(e)
  tmin_lw = scal(1)
  call rbin_real1(trim(ddir) // "/kdist_lw_g256.rbin", "temp_ref_max", scal, e); call chk(e)
  ! totplnk_delta = (temp_ref_max - temp_ref_min) / (nPlanckTemp - 1)   (rrtmgp/mo_gas_optics_rrtmgp.F90:1218)
  tdelta_lw = (scal(1) - tmin_lw) / real(size(totplnk, 1) - 1, wp)
  call rbin_int2(trim(ddir) // "/kdist_sw_g224.rbin", "band_lims_gpt", lims_sw, e); call chk(e)
  call rbin_real2(trim(ddir) // "/kdist_sw_g224.rbin", "band_lims_wvn", wvn_sw, e); call chk(e)
  call rbin_real1(trim(ddir) // "/kdist_sw_g224.rbin", "solar_source", solar, e); call chk(e)
  ! set_tsi(1361) (rrtmgp_rfmip_sw.F90:317; mo_gas_optics_rrtmgp.F90:1097-1120), then the default TSI the driver
  ! renormalises each column by (:408-427)
  def_tsi = 1._wp / sum_seq(solar)
  solar = solar * 1361.0_wp * def_tsi
  def_tsi = sum_seq(solar)
  if (allsky) then
    call load_clouds(trim(ddir) // "/cloud_optics_lw.rbin", wvn_lw, co_lw)
    call load_clouds(trim(ddir) // "/cloud_optics_sw.rbin", wvn_sw, co_sw)
  end if

  allocate(secs(nreps), starts(nreps))
  keep = .false.
  ! one untimed pass first (thread creation, MKL initialisation, first touch of every array)
  rep = nblocks
  nblocks = max(1, ncol / block)
  call run_blocks()
  nblocks = rep
  do rep = 1, nreps
    if (rep == nreps .and. len_trim(ofile) > 0) then
      keep = .true.
      allocate(o_lwu(nlay + 1, ncol), o_lwd(nlay + 1, ncol), o_swu(nlay + 1, ncol), o_swd(nlay + 1, ncol), &
               o_swr(nlay + 1, ncol))
      o_lwu = 0._wp; o_lwd = 0._wp; o_swu = 0._wp; o_swd = 0._wp; o_swr = 0._wp
    end if
    t0 = omp_get_wtime()
    if (rep == 1) tfirst = t0
    starts(rep) = t0 - tfirst
    call run_blocks()
    secs(rep) = omp_get_wtime() - t0
  end do
  if (keep) then
    u = rbin_write_begin(ofile, 5)
    call rbin_write_real(u, "lw_flux_up", o_lwu, shape(o_lwu))
    call rbin_write_real(u, "lw_flux_dn", o_lwd, shape(o_lwd))
    call rbin_write_real(u, "sw_flux_up", o_swu, shape(o_swu))
    call rbin_write_real(u, "sw_flux_dn", o_swd, shape(o_swd))
    call rbin_write_real(u, "sw_flux_dir", o_swr, shape(o_swr))
    call rbin_write_end(u)
  end if
  write(num, '(i0)') nthreads
  line = '{"threads": ' // trim(num)
  write(num, '(i0)') omp_get_num_procs()
  line = line // ', "nproc": ' // trim(num)
  write(num, '(i0)') block
  line = line // ', "block": ' // trim(num)
  write(num, '(i0)') nblocks * block
  line = line // ', "columns": ' // trim(num) // ', "seconds": ['
  do rep = 1, nreps
    write(num, '(f0.6)') secs(rep)
    if (num(1:1) == '.') num = '0' // num
    line = line // trim(num)
    if (rep < nreps) line = line // ', '
  end do
  ! each run's start, seconds after the first timed run's (a slow run can then be tied to the host's load over time)
  line = line // '], "starts": ['
  do rep = 1, nreps
    write(num, '(f0.6)') starts(rep)
    if (num(1:1) == '.') num = '0' // num
    line = line // trim(num)
    if (rep < nreps) line = line // ', '
  end do
  write(*, '(a)') line // ']}'

contains

  subroutine chk(msg)
    character(len=*), intent(in) :: msg
    if (len_trim(msg) > 0) then
      write(*, '(a)') trim(msg)
      error stop 1
    end if
  end subroutine chk

  ! float32 sum in index order (a Fortran DO loop)
  function sum_seq(a) result(s)
    real(wp), intent(in) :: a(:)
    real(wp) :: s
    integer :: i
    s = 0._wp
    do i = 1, size(a)
      s = s + a(i)
    end do
  end function sum_seq

  ! network_type from an RBIN model file (the reference's load reads the same numbers from netCDF,
  ! neural/mod_network_rrtmgp.F90:58-122): w<n> is w_transposed(n_out, n_in), activations by name
  subroutine load_model(path, m)
    character(len=*), intent(in) :: path
    type(nn_model), intent(inout) :: m
    integer, allocatable :: dims(:), acts(:)
    real(wp), allocatable :: w(:,:), b(:)
    character(len=32), allocatable :: names(:)
    character(len=16), dimension(0:6) :: an = [character(len=16) :: 'linear', 'softsign', 'relu', 'sigmoid', &
                                               'hard_sigmoid', 'tanh', 'gaussian']
    character(len=8) :: lname
    integer :: n, k, g
    call rbin_int1(path, "dims", dims, e); call chk(e)
    call rbin_int1(path, "activation", acts, e); call chk(e)
    call m%net%init(dims)
    do n = 1, size(dims) - 1
      write(lname, '(i0)') n
      call rbin_real2(path, "w" // trim(lname), w, e); call chk(e)
      call rbin_real1(path, "b" // trim(lname), b, e); call chk(e)
      m%net%layers(n)%w_transposed = w
      m%net%layers(n)%w = transpose(w)
      m%net%layers(n)%b = b
      call m%net%layers(n)%set_activation(trim(an(acts(n))))
    end do
    m%nx = dims(1)
    m%ny = dims(size(dims))
    call rbin_real1(path, "input_min", m%in_min, e); call chk(e)
    call rbin_real1(path, "input_max", m%in_max, e); call chk(e)
    call rbin_real1(path, "output_mean", m%out_mean, e)   ! absent for the Planck-fraction model (pfrac = y**2)
    if (e /= '') allocate(m%out_mean(0))
    call rbin_real1(path, "output_std", m%out_std, e)
    if (e /= '') allocate(m%out_std(0))
    call rbin_strings(path, "input_names", names, e); call chk(e)
    allocate(m%gas_idx(m%nx))
    m%gas_idx = 0
    do k = 3, m%nx
      do g = 1, ngas
        if (trim(gas_names(g)) == trim(names(k))) m%gas_idx(k) = g
      end do
    end do
  end subroutine load_model

  ! ty_cloud_optics%load_lut + set_ice_roughness(2), as the all-sky example (examples/all-sky/rrtmgp_allsky.F90)
  subroutine load_clouds(path, wvn, co)
    character(len=*), intent(in) :: path
    real(wp), intent(in) :: wvn(:,:)
    type(ty_cloud_optics), intent(inout) :: co
    real(wp), allocatable :: rl(:), ru(:), rf(:), il(:), iu(:), ifc(:)
    real(wp), allocatable :: el(:,:), sl(:,:), al(:,:), ei(:,:,:), si(:,:,:), ai(:,:,:)
    call rbin_real1(path, "radliq_lwr", rl, e); call chk(e)
    call rbin_real1(path, "radliq_upr", ru, e); call chk(e)
    call rbin_real1(path, "radliq_fac", rf, e); call chk(e)
    call rbin_real1(path, "radice_lwr", il, e); call chk(e)
    call rbin_real1(path, "radice_upr", iu, e); call chk(e)
    call rbin_real1(path, "radice_fac", ifc, e); call chk(e)
    call rbin_real2(path, "lut_extliq", el, e); call chk(e)
    call rbin_real2(path, "lut_ssaliq", sl, e); call chk(e)
    call rbin_real2(path, "lut_asyliq", al, e); call chk(e)
    call rbin_real3(path, "lut_extice", ei, e); call chk(e)
    call rbin_real3(path, "lut_ssaice", si, e); call chk(e)
    call rbin_real3(path, "lut_asyice", ai, e); call chk(e)
    call chk(co%load(wvn, rl(1), ru(1), rf(1), il(1), iu(1), ifc(1), el, sl, al, ei, si, ai))
    call chk(co%set_ice_roughness(2))
  end subroutine load_clouds

  ! compute_nn_inputs (rrtmgp/mo_gas_optics_rrtmgp.F90:618-798) for columns c0+1 .. c0+nb
  subroutine nn_inputs(m, c0, nb, x)
    type(nn_model), intent(in) :: m
    integer, intent(in) :: c0, nb
    real(wp), intent(out) :: x(*)
    type(c_ptr) :: gp(64)
    integer(c_int) :: nd(64)
    integer :: k
    gp = c_null_ptr
    nd = 2
    do k = 3, m%nx
      if (m%gas_idx(k) > 0) gp(k) = c_loc(vmr(m%gas_idx(k))%v(1, c0 + 1))
    end do
    call orc_compute_nn_inputs(nb, nlay, m%nx, c_loc(play(1, c0 + 1)), c_loc(tlay(1, c0 + 1)), gp, nd, &
                               m%in_min, m%in_max, x)
  end subroutine nn_inputs

  subroutine run_blocks()
    type(ty_optical_props_1scl) :: op_lw, cl_lw
    type(ty_optical_props_2str), target :: op_sw
    type(ty_optical_props_2str) :: cl_sw
    type(ty_source_func_lw) :: src
    type(ty_fluxes_flexible) :: fl_lw, fl_sw
    real(wp), allocatable, target :: x(:), cd(:), emis(:,:), toa(:,:), alb(:,:)
    real(wp), allocatable, target :: up(:,:), dn(:,:), sup(:,:), sdn(:,:), sdir(:,:)
    integer :: b, c0, icol, sfc_lay, nbt
    integer(c_long) :: nbatch
    character(len=128) :: err

    !$omp parallel num_threads(nthreads) default(shared) &
    !$omp   private(op_lw, cl_lw, op_sw, cl_sw, src, fl_lw, fl_sw, x, cd, emis, toa, alb, up, dn, sup, sdn, sdir, &
    !$omp           b, c0, icol, sfc_lay, nbt, nbatch, err)
    ! per-thread objects, allocated once (rrtmgp_rfmip_lw.F90:326-327, firstprivate into the block loop)
    call chk(op_lw%alloc_1scl(block, nlay, wvn_lw, lims_lw))
    call chk(src%alloc(block, nlay, op_lw))
    call chk(op_sw%alloc_2str(block, nlay, wvn_sw, lims_sw))
    if (allsky) then
      call chk(cl_lw%alloc_1scl(block, nlay, wvn_lw))
      call chk(cl_sw%alloc_2str(block, nlay, wvn_sw))
    end if
    allocate(x(max(lw_abs%nx, sw_abs%nx) * nlay * block), cd(nlay * block))
    allocate(emis(size(lims_lw, 2), block), toa(size(solar), block), alb(size(solar), block))
    allocate(up(nlay + 1, block), dn(nlay + 1, block), sup(nlay + 1, block), sdn(nlay + 1, block), &
             sdir(nlay + 1, block))
    fl_lw%flux_up => up
    fl_lw%flux_dn => dn
    fl_sw%flux_up => sup
    fl_sw%flux_dn => sdn
    fl_sw%flux_dn_dir => sdir
    nbatch = int(nlay, c_long) * block
    !$omp do schedule(static)
    do b = 0, nblocks - 1
      c0 = mod(b * block, ncol)
      ! ---- longwave: gas_optics (NN) -> [clouds%increment] -> rte_lw (rrtmgp_rfmip_lw.F90:385-446) ----
      call nn_inputs(lw_abs, c0, block, x)
      call orc_get_col_dry(block, nlay, c_loc(vmr(lw_abs%gas_idx(3))%v(1, c0 + 1)), c_loc(plev(1, c0 + 1)), cd)
      call lw_abs%net%output_sgemm_flat(lw_abs%nx, lw_abs%ny, int(nbatch), x, op_lw%tau)
      call orc_nn_tau_post(lw_abs%ny, nbatch, op_lw%tau, lw_abs%out_mean, lw_abs%out_std, cd, c_null_ptr)
      call lw_pf%net%output_sgemm_flat(lw_pf%nx, lw_pf%ny, int(nbatch), x, src%lay_source)
      call orc_square(int(lw_pf%ny, c_long) * nbatch, src%lay_source)
      sfc_lay = merge(1, nlay, play(1, c0 + 1) > play(nlay, c0 + 1))
      call orc_planck_source_nn(block, nlay, size(lims_lw, 2), lw_abs%ny, size(totplnk, 1), &
                                c_loc(tlay(1, c0 + 1)), c_loc(tlev(1, c0 + 1)), c_loc(tsfc(c0 + 1)), sfc_lay, &
                                lims_lw, tmin_lw, tdelta_lw, totplnk, src%sfc_source, src%sfc_source_Jac, &
                                src%lay_source, src%lev_source)
      do icol = 1, block
        emis(:, icol) = sfc_emis(c0 + icol)
      end do
      if (allsky) then
        call chk(co_lw%cloud_optics(clwp(:, c0 + 1:c0 + block), ciwp(:, c0 + 1:c0 + block), &
                                    rel(:, c0 + 1:c0 + block), rei(:, c0 + 1:c0 + block), cl_lw))
        call chk(cl_lw%increment(op_lw))
      end if
      call chk(rte_lw(op_lw, top_at_1, src, emis, fl_lw, n_gauss_angles=1, use_2stream=.false.))
      if (keep) then
        o_lwu(:, c0 + 1:c0 + block) = up
        o_lwd(:, c0 + 1:c0 + block) = dn
      end if
      if (do_sw == 0) cycle
      ! ---- shortwave: gas_optics (NN) -> [delta_scale, increment] -> rte_sw (rrtmgp_rfmip_sw.F90:370-470) ----
      call nn_inputs(sw_abs, c0, block, x)
      call sw_abs%net%output_sgemm_flat(sw_abs%nx, sw_abs%ny, int(nbatch), x, op_sw%tau)
      call orc_nn_tau_post(sw_abs%ny, nbatch, op_sw%tau, sw_abs%out_mean, sw_abs%out_std, cd, c_null_ptr)
      call sw_ray%net%output_sgemm_flat(sw_ray%nx, sw_ray%ny, int(nbatch), x, op_sw%ssa)
      call orc_nn_tau_post(sw_ray%ny, nbatch, op_sw%ssa, sw_ray%out_mean, sw_ray%out_std, cd, c_loc(op_sw%tau))
      op_sw%g = 0._wp
      do icol = 1, block
        toa(:, icol) = solar(:) * tsi(c0 + icol) / def_tsi
        alb(:, icol) = sfc_alb(c0 + icol)
      end do
      if (allsky) then
        call chk(co_sw%cloud_optics(clwp(:, c0 + 1:c0 + block), ciwp(:, c0 + 1:c0 + block), &
                                    rel(:, c0 + 1:c0 + block), rei(:, c0 + 1:c0 + block), cl_sw))
        call chk(cl_sw%delta_scale())
        call chk(cl_sw%increment(op_sw))
      end if
      call chk(rte_sw(op_sw, top_at_1, mu0(c0 + 1:c0 + block), toa, alb, alb, fl_sw))
      if (keep) then
        o_swu(:, c0 + 1:c0 + block) = sup
        o_swd(:, c0 + 1:c0 + block) = sdn
        o_swr(:, c0 + 1:c0 + block) = sdir
      end if
    end do
    !$omp end do
    !$omp end parallel
  end subroutine run_blocks
end program rrtmgp_cpu_bench
