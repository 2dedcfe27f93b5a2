! mo_rte_kind -- kinds of the reference (rte/mo_rte_kind.F90:29-33): single precision working kind.
module mo_rte_kind
  use, intrinsic :: iso_c_binding, only: c_float, c_double, c_bool
  implicit none
  public
  integer, parameter :: sp = c_float, dp = c_double, wp = sp, wl = c_bool
end module mo_rte_kind
