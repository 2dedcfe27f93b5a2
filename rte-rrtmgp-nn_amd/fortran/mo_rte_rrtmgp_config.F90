! mo_rte_rrtmgp_config -- drop-in for rte/mo_rte_rrtmgp_config.F90: run-time switches for argument checks.
! Extent checks always run in this build (a mis-sized array would be an out-of-bounds device access);
! check_values gates the value-range checks exactly as in the reference (default .false., :7-8).
module mo_rte_rrtmgp_config
  use mo_rte_kind, only: wl
  implicit none
  private
  logical(wl), protected, public :: check_extents = .false.
  logical(wl), protected, public :: check_values  = .false.
  logical(wl), parameter, public :: compute_Jac = .false.
  logical(wl), parameter, public :: use_Pade_source = .false.
  integer, protected, public :: nn_scenario_index = 0

  interface rte_rrtmgp_config_checks
    module procedure config_checks_each, config_checks_all
  end interface
  public :: rte_rrtmgp_config_checks
contains
  subroutine config_checks_each(extents, values)
    logical(wl), intent(in) :: extents, values
    check_extents = extents
    check_values  = values
  end subroutine config_checks_each

  subroutine config_checks_all(do_checks)
    logical(wl), intent(in) :: do_checks
    check_extents = do_checks
    check_values  = do_checks
  end subroutine config_checks_all
end module mo_rte_rrtmgp_config
