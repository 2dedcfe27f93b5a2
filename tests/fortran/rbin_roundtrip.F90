! CPU-only check of the Fortran RBIN reader/writer and ty_gas_concs (no device calls):
! reads play, tsfc and gas_names from argv(1), writes play, tsfc and the h2o vmr read back through
! ty_gas_concs into argv(2).
program rbin_roundtrip
  use mo_rte_kind,           only: wp
  use mo_rrtmgpnn_rbin
  use mo_gas_concentrations, only: ty_gas_concs
  implicit none
  character(len=512) :: fin, fout
  real(wp), allocatable :: play(:,:), tsfc(:), vmr(:,:)
  character(len=32), allocatable :: names(:)
  character(len=128) :: e
  type(ty_gas_concs) :: gc
  integer :: u, nd, igas
  call get_command_argument(1, fin)
  call get_command_argument(2, fout)
  call rbin_real2(fin, "play", play, e); if (e /= '') error stop 1
  call rbin_real1(fin, "tsfc", tsfc, e); if (e /= '') error stop 2
  call rbin_strings(fin, "gas_names", names, e); if (e /= '') error stop 3
  call rbin_real2(fin, "vmr_h2o", vmr, e); if (e /= '') error stop 4
  e = gc%init(names); if (e /= '') error stop 5
  e = gc%set_vmr("H2O", vmr); if (e /= '') error stop 6
  e = gc%get_conc_dims_and_igas("h2o", nd, igas); if (e /= '' .or. nd /= 2) error stop 7
  e = gc%set_vmr("bogus", 0.5_wp); if (e == '') error stop 8
  u = rbin_write_begin(fout, 3)
  call rbin_write_real(u, "play", play, shape(play))
  call rbin_write_real(u, "tsfc", tsfc, shape(tsfc))
  call rbin_write_real(u, "h2o", gc%concs(igas)%conc, shape(gc%concs(igas)%conc))
  call rbin_write_end(u)
end program rbin_roundtrip
