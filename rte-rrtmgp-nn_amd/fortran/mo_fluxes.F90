! mo_fluxes -- drop-in for rte/mo_fluxes.F90 (ty_fluxes_broadband / ty_fluxes_flexible, :35-67):
! broadband outputs are pointers into caller memory, (nlay+1, ncol) each; g-point outputs (ngpt, nlay+1, ncol).
module mo_fluxes
  use mo_rte_kind, only: wp
  implicit none
  private

  type, public :: ty_fluxes_broadband
    real(wp), dimension(:,:), contiguous, pointer :: flux_up => NULL(), flux_dn => NULL()
    real(wp), dimension(:,:), contiguous, pointer :: flux_net => NULL()
    real(wp), dimension(:,:), contiguous, pointer :: flux_dn_dir => NULL()
  contains
    procedure, public :: are_desired => are_desired_broadband
    procedure, public :: check_extents => check_extents_broadband
  end type ty_fluxes_broadband

  type, extends(ty_fluxes_broadband), public :: ty_fluxes_flexible
    real(wp), dimension(:,:,:), contiguous, pointer :: gpt_flux_up => NULL(), gpt_flux_dn => NULL()
    real(wp), dimension(:,:,:), contiguous, pointer :: gpt_flux_net => NULL(), gpt_flux_dn_dir => NULL()
    real(wp), dimension(:,:,:), contiguous, pointer :: gpt_flux_up_Jac => NULL()
  contains
    procedure, public :: are_desired_gpt
  end type ty_fluxes_flexible

contains

  logical function are_desired_broadband(this)
    class(ty_fluxes_broadband), intent(in) :: this
    are_desired_broadband = any([associated(this%flux_up), associated(this%flux_dn), associated(this%flux_dn_dir), &
                                 associated(this%flux_net)])
  end function are_desired_broadband

  ! The output extents reduce_broadband checks (rte/mo_fluxes.F90:143-162): every associated broadband array must be
  ! (nlev, ncol); the last failing array's message is returned, as there.  rte_lw / rte_sw call it before any
  ! device work, so a mis-shaped caller array is reported instead of written in the wrong layout.
  function check_extents_broadband(this, nlev, ncol) result(error_msg)
    class(ty_fluxes_broadband), intent(in) :: this
    integer,                    intent(in) :: nlev, ncol
    character(len=128) :: error_msg
    error_msg = ""
    if (associated(this%flux_up)) then
      if (any(shape(this%flux_up) /= [nlev, ncol])) error_msg = "reduce: flux_up array incorrectly sized"
    end if
    if (associated(this%flux_dn)) then
      if (any(shape(this%flux_dn) /= [nlev, ncol])) error_msg = "reduce: flux_dn array incorrectly sized"
    end if
    if (associated(this%flux_net)) then
      if (any(shape(this%flux_net) /= [nlev, ncol])) error_msg = "reduce: flux_net array incorrectly sized"
    end if
    if (associated(this%flux_dn_dir)) then
      if (any(shape(this%flux_dn_dir) /= [nlev, ncol])) error_msg = "reduce: flux_dn_dir array incorrectly sized"
    end if
  end function check_extents_broadband

  logical function are_desired_gpt(this)
    class(ty_fluxes_flexible), intent(in) :: this
    are_desired_gpt = any([associated(this%gpt_flux_up), associated(this%gpt_flux_dn), &
                           associated(this%gpt_flux_dn_dir), associated(this%gpt_flux_net)])
  end function are_desired_gpt
end module mo_fluxes
