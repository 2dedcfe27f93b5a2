! mo_fluxes -- drop-in for rte/mo_fluxes.F90 (ty_fluxes_broadband / ty_fluxes_flexible, :35-67):
! broadband outputs are pointers into caller memory.  g-point fluxes are not produced by this build.
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

  logical function are_desired_gpt(this)
    class(ty_fluxes_flexible), intent(in) :: this
    are_desired_gpt = any([associated(this%gpt_flux_up), associated(this%gpt_flux_dn), &
                           associated(this%gpt_flux_dn_dir), associated(this%gpt_flux_net)])
  end function are_desired_gpt
end module mo_fluxes
