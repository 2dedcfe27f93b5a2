! reset_vmr.F90 -- a gas re-set between two parallel block loops (tests/test_fortran.py): the device data environment's
! invalidations are process-wide (csrc/present.cpp), so worker threads whose contexts cached a block's concentrations
! in loop 1 read the values set_vmr stored from the serial region before loop 2 (drop, deallocate, allocate: usually
! the same address and size), as the reference's single OpenACC data environment would.
! usage: reset_vmr <problem.rbin> <output.rbin> <data_dir> <block_size>
!   output: LW fluxes of loop 1 (flux_up_1 / flux_dn_1, the problem's gases) and of loop 2 (flux_up_2 / flux_dn_2,
!   h2o scaled by 0.5 and o3 by 0.25 in every block), (nlay+1, ncol) each.
program reset_vmr
  use mo_rte_kind,           only: wp
  use mo_optical_props,      only: ty_optical_props_1scl
  use mo_source_functions,   only: ty_source_func_lw
  use mo_fluxes,             only: ty_fluxes_flexible
  use mo_gas_concentrations, only: ty_gas_concs
  use mo_gas_optics_rrtmgp,  only: ty_gas_optics_rrtmgp
  use mod_network_rrtmgp,    only: rrtmgp_network_type
  use mo_rte_lw,             only: rte_lw
  use mo_rrtmgpnn_rbin
  implicit none
  character(len=512) :: pfile, ofile, ddir, arg
  real(wp), allocatable :: play(:,:), plev(:,:), tlay(:,:), tlev(:,:), tsfc(:), sfc_emis(:), scal(:), vmr(:,:)
  real(wp), allocatable :: vmr_all(:,:,:), emis(:,:)
  real(wp), allocatable, target :: up(:,:,:), dn(:,:,:)
  character(len=32), allocatable :: gas_names(:)
  type(ty_gas_concs), allocatable :: gas_concs(:)
  type(ty_gas_optics_rrtmgp) :: kdist
  type(rrtmgp_network_type), dimension(2) :: nets
  type(ty_optical_props_1scl) :: op
  type(ty_source_func_lw) :: src
  type(ty_fluxes_flexible) :: fl
  character(len=128) :: e
  integer :: ncol, nlay, ngas, ig, icol, u, bs, nblocks, b, b0, b1, nb, loop
  logical :: top_at_1

  call get_command_argument(1, pfile)
  call get_command_argument(2, ofile)
  call get_command_argument(3, ddir)
  call get_command_argument(4, arg)
  read(arg, *) bs
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
  ngas = size(gas_names)
  call nets(1)%load_netcdf(trim(ddir) // "/nn_lw_g256_abs.rbin")
  call nets(2)%load_netcdf(trim(ddir) // "/nn_lw_g256_pfrac.rbin")
  call chk(kdist%load_rbin(trim(ddir) // "/kdist_lw_g256.rbin", gas_names))
  nblocks = (ncol + bs - 1) / bs
  allocate(gas_concs(nblocks), vmr_all(nlay, ncol, ngas), up(nlay + 1, ncol, 2), dn(nlay + 1, ncol, 2))
  do ig = 1, ngas
    call rbin_real2(pfile, "vmr_" // trim(gas_names(ig)), vmr, e); call chk(e)
    vmr_all(:, :, ig) = vmr
  end do
  do b = 1, nblocks
    b0 = (b - 1) * bs + 1
    b1 = min(ncol, b0 + bs - 1)
    call chk(gas_concs(b)%init(gas_names))
    do ig = 1, ngas
      call chk(gas_concs(b)%set_vmr(gas_names(ig), vmr_all(:, b0:b1, ig)))
    end do
  end do
  do loop = 1, 2
    if (loop == 2) then
      ! serial region, as a GCM's next step: new values for two gases of every block
      do ig = 1, ngas
        if (trim(gas_names(ig)) == "h2o") vmr_all(:, :, ig) = 0.5_wp * vmr_all(:, :, ig)
        if (trim(gas_names(ig)) == "o3") vmr_all(:, :, ig) = 0.25_wp * vmr_all(:, :, ig)
      end do
      do b = 1, nblocks
        b0 = (b - 1) * bs + 1
        b1 = min(ncol, b0 + bs - 1)
        do ig = 1, ngas
          if (trim(gas_names(ig)) == "h2o" .or. trim(gas_names(ig)) == "o3") &
            call chk(gas_concs(b)%set_vmr(gas_names(ig), vmr_all(:, b0:b1, ig)))
        end do
      end do
    end if
    !$omp parallel do schedule(static) default(shared) private(b, b0, b1, nb, icol, op, src, fl, emis)
    do b = 1, nblocks
      b0 = (b - 1) * bs + 1
      b1 = min(ncol, b0 + bs - 1)
      nb = b1 - b0 + 1
      call chk(op%alloc_1scl(nb, nlay, kdist))
      call chk(src%alloc(nb, nlay, kdist))
      allocate(emis(kdist%get_nband(), nb))
      do icol = 1, nb
        emis(:, icol) = sfc_emis(b0 + icol - 1)
      end do
      call chk(kdist%gas_optics(play(:, b0:b1), plev(:, b0:b1), tlay(:, b0:b1), tsfc(b0:b1), gas_concs(b), op, src, &
                                tlev=tlev(:, b0:b1), neural_nets=nets))
      fl%flux_up => up(:, b0:b1, loop)
      fl%flux_dn => dn(:, b0:b1, loop)
      call chk(rte_lw(op, top_at_1, src, emis, fl))
      deallocate(emis)
      call op%finalize()
      call src%finalize()
    end do
    !$omp end parallel do
  end do
  u = rbin_write_begin(ofile, 4)
  call rbin_write_real(u, "flux_up_1", up(:, :, 1), [nlay + 1, ncol])
  call rbin_write_real(u, "flux_dn_1", dn(:, :, 1), [nlay + 1, ncol])
  call rbin_write_real(u, "flux_up_2", up(:, :, 2), [nlay + 1, ncol])
  call rbin_write_real(u, "flux_dn_2", dn(:, :, 2), [nlay + 1, ncol])
  call rbin_write_end(u)
contains
  subroutine chk(msg)
    character(len=*), intent(in) :: msg
    if (len_trim(msg) > 0) then
      write(*, '(a)') trim(msg)
      error stop 1
    end if
  end subroutine chk
end program reset_vmr
