! stop_on_err -- the caller-provided error hook the reference's class layer calls
! (e.g. rte/mo_rte_lw.F90 "class default" branch); the reference drivers define it in the
! program unit (examples/rfmip-clear-sky/rrtmgp_rfmip_lw.F90:25-35).  TEST INFRASTRUCTURE.
subroutine stop_on_err(msg)
  use iso_fortran_env, only: error_unit
  character(len=*), intent(in) :: msg
  if (len_trim(msg) > 0) then
    write(error_unit, *) trim(msg)
    error stop 1
  end if
end subroutine stop_on_err
