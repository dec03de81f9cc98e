! compton2d_mod.f90 -- Fortran 2003 (iso_c_binding) interface to include/compton2d.h.
!
! This is the binding a maintainer adds to the reference's Fortran host
! (bbw7561135/Compton2d src/) so that the worker-side calls
!     call imcfield2d ; call imcvol2d ; call imcsurf2d      (src/xec2d.f:167-176)
! become one c2d_transport_step() per GPU, with the COMMON tables passed in
! place through (c_loc, strides).  See INTEGRATION.md.
module compton2d
  use iso_c_binding
  implicit none

  integer(c_int), parameter :: C2D_OK = 0, C2D_E_ARG = -1, C2D_E_HIP = -2, &
       C2D_E_CENSUS_OVERFLOW = -3, C2D_E_EVENT_OVERFLOW = -4, C2D_E_QUEUE_OVERFLOW = -5
  integer(c_int32_t), parameter :: C2D_COMTOT_EXACT = 0, C2D_COMTOT_TABLE = 1
  integer, parameter :: C2D_NCOUNTERS = 16, C2D_CNT_STEPS = 0, C2D_CNT_ESCAPES = 1, &
       C2D_CNT_CENSUS = 2

  type, bind(C) :: c2d_array3
     type(c_ptr) :: data = c_null_ptr
     integer(c_int64_t) :: s_i = 0, s_j = 0, s_k = 0
  end type c2d_array3

  type, bind(C) :: c2d_array2
     type(c_ptr) :: data = c_null_ptr
     integer(c_int64_t) :: s_j = 0, s_k = 0
  end type c2d_array2

  type, bind(C) :: c2d_spectrum
     integer(c_int32_t) :: nfile = 0
     type(c_ptr) :: E_file = c_null_ptr, a1 = c_null_ptr, I_file = c_null_ptr, &
          F_file = c_null_ptr, P_file = c_null_ptr
  end type c2d_spectrum

  type, bind(C) :: c2d_config
     integer(c_int32_t) :: nz = 0, nr = 0
     real(c_double) :: rmin = 0, zmin = 0
     type(c_ptr) :: z = c_null_ptr, r = c_null_ptr, E_ph = c_null_ptr, &
          E_field = c_null_ptr, gnt = c_null_ptr
     integer(c_int32_t) :: nphtotal = 0
     type(c_ptr) :: hu = c_null_ptr
     integer(c_int32_t) :: nph_lc = 0
     type(c_ptr) :: Elcmin = c_null_ptr, Elcmax = c_null_ptr
     integer(c_int32_t) :: nmu = 0
     type(c_ptr) :: mu = c_null_ptr
     integer(c_int32_t) :: split1 = 10, split2 = 10, split3 = 3, spl3_trg = 10
     integer(c_int32_t) :: spec_switch = 0, cr_sent = 0, pair_switch = 0, kappa_lag = 1
     integer(c_int32_t) :: comtot_mode = C2D_COMTOT_TABLE, device = 0
     integer(c_int64_t) :: seed = 99999
     integer(c_int32_t) :: rank = 0, world = 1
     integer(c_int64_t) :: census_capacity = 5000000, event_capacity = 5000000, &
          queue_capacity = 262144
  end type c2d_config

  type, bind(C) :: c2d_step_in
     integer(c_int32_t) :: ncycle = 0
     real(c_double) :: time = 0, dt = 0
     type(c2d_array3) :: kappa_tot, eps_tot, eps_th, f_nt, Pnt
     type(c2d_array2) :: n_e, Eloss_th, Eloss_tot, zsurf, ewsv
     type(c2d_array2) :: nsv                     ! int32 data (c2d_iarray2)
     type(c_ptr) :: nsurfi = c_null_ptr, nsurfo = c_null_ptr, ewsurfi = c_null_ptr, &
          ewsurfo = c_null_ptr, nsurfu = c_null_ptr, nsurfl = c_null_ptr, &
          ewsurfu = c_null_ptr, ewsurfl = c_null_ptr
     type(c_ptr) :: tbbi = c_null_ptr, tbbo = c_null_ptr, tbbu = c_null_ptr, tbbl = c_null_ptr
     type(c_ptr) :: spec_i = c_null_ptr, spec_o = c_null_ptr, spec_u = c_null_ptr, &
          spec_l = c_null_ptr
     integer(c_int32_t) :: n_spectra = 0
     type(c_ptr) :: spectra = c_null_ptr
  end type c2d_step_in

  type, bind(C) :: c2d_tally_layout
     integer(c_int64_t) :: edep, prdep, ecens, npcen, n_field, E_IC, nelectron, fout, &
          edout, erlki, erlko, erlku, erlkl, Ed_in, counters, total
  end type c2d_tally_layout

  interface
     integer(c_int) function c2d_init(cfg, ctx) bind(C, name='c2d_init')
       import :: c_int, c_ptr, c2d_config
       type(c2d_config), intent(in) :: cfg
       type(c_ptr), intent(out) :: ctx
     end function c2d_init

     subroutine c2d_finalize(ctx) bind(C, name='c2d_finalize')
       import :: c_ptr
       type(c_ptr), value :: ctx
     end subroutine c2d_finalize

     type(c_ptr) function c2d_last_error(ctx) bind(C, name='c2d_last_error')
       import :: c_ptr
       type(c_ptr), value :: ctx
     end function c2d_last_error

     integer(c_int) function c2d_transport_step(ctx, sin) bind(C, name='c2d_transport_step')
       import :: c_int, c_ptr, c2d_step_in
       type(c_ptr), value :: ctx
       type(c2d_step_in), intent(in) :: sin
     end function c2d_transport_step

     integer(c_int) function c2d_set_step(ctx, sin) bind(C, name='c2d_set_step')
       import :: c_int, c_ptr, c2d_step_in
       type(c_ptr), value :: ctx
       type(c2d_step_in), intent(in) :: sin
     end function c2d_set_step

     integer(c_int) function c2d_set_clock(ctx, ncycle, time, dt) bind(C, name='c2d_set_clock')
       import :: c_int, c_ptr, c_int32_t, c_double
       type(c_ptr), value :: ctx
       integer(c_int32_t), value :: ncycle
       real(c_double), value :: time, dt
     end function c2d_set_clock

     integer(c_int) function c2d_run_step(ctx) bind(C, name='c2d_run_step')
       import :: c_int, c_ptr
       type(c_ptr), value :: ctx
     end function c2d_run_step

     integer(c_int) function c2d_tally_layout_get(ctx, lay) bind(C, name='c2d_tally_layout_get')
       import :: c_int, c_ptr, c2d_tally_layout
       type(c_ptr), value :: ctx
       type(c2d_tally_layout), intent(out) :: lay
     end function c2d_tally_layout_get

     integer(c_int) function c2d_tally_download(ctx, host, n) bind(C, name='c2d_tally_download')
       import :: c_int, c_ptr, c_double, c_int64_t
       type(c_ptr), value :: ctx
       real(c_double), intent(out) :: host(*)
       integer(c_int64_t), value :: n
     end function c2d_tally_download

     integer(c_int) function c2d_events(ctx, buf, cap, n) bind(C, name='c2d_events')
       import :: c_int, c_ptr, c_double, c_int64_t
       type(c_ptr), value :: ctx
       real(c_double), intent(out) :: buf(7, *)
       integer(c_int64_t), value :: cap
       integer(c_int64_t), intent(out) :: n
     end function c2d_events

     integer(c_int) function c2d_census_count(ctx, n) bind(C, name='c2d_census_count')
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: ctx
       integer(c_int64_t), intent(out) :: n
     end function c2d_census_count

     integer(c_int) function c2d_census_export(ctx, d6, i5, keys, cap, n) &
          bind(C, name='c2d_census_export')
       import :: c_int, c_ptr, c_double, c_int32_t, c_int64_t
       type(c_ptr), value :: ctx
       real(c_double), intent(out) :: d6(6, *)
       integer(c_int32_t), intent(out) :: i5(5, *)
       integer(c_int64_t), intent(out) :: keys(*)
       integer(c_int64_t), value :: cap
       integer(c_int64_t), intent(out) :: n
     end function c2d_census_export

     integer(c_int) function c2d_census_import(ctx, d6, i5, keys, n) &
          bind(C, name='c2d_census_import')
       import :: c_int, c_ptr, c_double, c_int32_t, c_int64_t
       type(c_ptr), value :: ctx
       real(c_double), intent(in) :: d6(6, *)
       integer(c_int32_t), intent(in) :: i5(5, *)
       integer(c_int64_t), intent(in) :: keys(*)
       integer(c_int64_t), value :: n
     end function c2d_census_import
  end interface
end module compton2d
