! compton2d_mod.f90 -- Fortran 2003 (iso_c_binding) interface to include/compton2d.h.
!
! This is the binding a maintainer adds to the reference's Fortran host
! (bbw7561135/Compton2d src/) so that the worker-side calls
!     call imcfield2d ; call imcvol2d ; call imcsurf2d      (src/xec2d.f:167-176)
! become one c2d_transport_step() per GPU, and `call update`
! (src/xec2d.f:86-87, src/update2d.f:7-327) one c2d_fp_step(), with the COMMON
! tables passed in place through (c_loc, strides).  See INTEGRATION.md.
module compton2d
  use iso_c_binding
  implicit none

  integer(c_int), parameter :: C2D_OK = 0, C2D_E_ARG = -1, C2D_E_HIP = -2, &
       C2D_E_CENSUS_OVERFLOW = -3, C2D_E_EVENT_OVERFLOW = -4, C2D_E_QUEUE_OVERFLOW = -5, &
       C2D_E_NOMEM = -6, C2D_E_STATE = -7, C2D_E_FP = -8, C2D_E_RCCL = -9, C2D_E_IO = -10, &
       C2D_E_NONFINITE = -11
  ! c2d_step_in%device_tables flags; RCCL unique-id size (c2d_comm_unique_id)
  integer(c_int32_t), parameter :: C2D_DEV_EMISSION = 1, C2D_DEV_ELECTRONS = 2
  integer(c_int32_t), parameter :: C2D_FP_EXACT = 0, C2D_FP_FAST = 1, C2D_FP_AUTO = 2
  integer, parameter :: C2D_COMM_ID_BYTES = 128
  integer(c_int32_t), parameter :: C2D_COMTOT_EXACT = 0, C2D_COMTOT_TABLE = 1
  integer(c_int32_t), parameter :: C2D_TRK_SRC = 0, C2D_TRK_2012_11 = 1
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
     integer(c_int32_t) :: census_inplace = 0
     integer(c_int32_t) :: trk_variant = 0
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
     integer(c_int32_t) :: device_tables = 0     ! C2D_DEV_* flags
  end type c2d_step_in

  ! ---- Fokker-Planck update (c2d_fp_set_config / c2d_fp_step) ----
  integer, parameter :: C2D_FP_NDIAG = 8, C2D_FP_STEPS = 5, C2D_FP_SKIPPED = 6

  type, bind(C) :: c2d_marray3
     type(c_ptr) :: data = c_null_ptr
     integer(c_int64_t) :: s_i = 0, s_j = 0, s_k = 0
  end type c2d_marray3

  type, bind(C) :: c2d_marray2
     type(c_ptr) :: data = c_null_ptr
     integer(c_int64_t) :: s_j = 0, s_k = 0
  end type c2d_marray2

  type, bind(C) :: c2d_fp_config              ! reader.f:512-559, general.pa:27-28
     integer(c_int32_t) :: pair_switch = 0
     real(c_double) :: df_implicit = 1.d-2, df_T = 2.5d-1, r_esc = 0.3d0, r_acc = 1.d0
     integer(c_int32_t) :: cf_sentinel = 0
     real(c_double) :: r_flare = 0, z_flare = 0, t_flare = 0, sigma_r = 1, sigma_z = 1, &
          sigma_t = 1, flare_amp = 0
     integer(c_int32_t) :: inj_switch = 0, inj_dis = 2, g2var_switch = 0, pick_sw = 0
     real(c_double) :: inj_g1 = 0, inj_g2 = 0, inj_p = 0, inj_t = 0, inj_L = 0, &
          pick_rate = 0, inj_gg = 0, inj_sigma = 1, inj_v = 0
     type(c_ptr) :: F_IC = c_null_ptr             ! F_IC(num_nt, nphfield), COMMON /fic/
     integer(c_int64_t) :: F_IC_s_i = 1, F_IC_s_ph = 200
  end type c2d_fp_config

  type, bind(C) :: c2d_fp_step_in              ! what FP_send_job packs (fp_mpi.f:632-686)
     integer(c_int32_t) :: ncycle = 0
     real(c_double) :: time = 0, dt = 0
     type(c2d_array2) :: tea, tna, n_e, B_field, Eloss_sy, ec_old, turb_lev, vol
     type(c2d_array2) :: f_pair, ecens           ! ecens: null data = device tallies
     type(c2d_array3) :: n_field                 ! null data = device tallies
  end type c2d_fp_step_in

  type, bind(C) :: c2d_fp_step_out             ! updated in place (fp_mpi.f:972-1003)
     type(c2d_marray3) :: f_nt, Pnt
     type(c2d_marray2) :: Te_new, tea, n_e, gmin, gmax, amxwl, p_nth
     type(c_ptr) :: zone_diag = c_null_ptr
     real(c_double) :: E_tot_old = 0, E_tot_new = 0, hr_total = 0, hr_st_total = 0, dT_max = 0
  end type c2d_fp_step_out

  ! ---- emission / absorption tables (c2d_volume_em; imcgen2d.f:209-333) ----
  type, bind(C) :: c2d_iarray2
     type(c_ptr) :: data = c_null_ptr
     integer(c_int64_t) :: s_j = 0, s_k = 0
  end type c2d_iarray2

  type, bind(C) :: c2d_vem_in
     real(c_double) :: dt = 0
     type(c2d_array2) :: tea, tna, n_e, B_field, f_pair, zsurf, vol
     type(c2d_iarray2) :: ep_switch              ! null data: all 0
     type(c2d_array3) :: f_nt
  end type c2d_vem_in

  type, bind(C) :: c2d_vem_out
     type(c2d_marray3) :: kappa_tot, eps_tot, eps_th
     type(c2d_marray2) :: B_field, Eloss_sy, Eloss_cy, Eloss_th, Eloss_tot
     type(c_ptr) :: E_ph = c_null_ptr
  end type c2d_vem_out

  ! ---- observer-frame binning (c2d_obs_*; postprocessing/pspt.c, plcm.c) ----
  integer, parameter :: C2D_OBS_SED = 0, C2D_OBS_LC = 1

  type, bind(C) :: c2d_obs_bins
     integer(c_int32_t) :: mode = 0
     real(c_double) :: gam_bulk = 33.d0, rmax = 1.d16, t_offset = 0.d0
     integer(c_int32_t) :: n_t = 0
     type(c_ptr) :: t0 = c_null_ptr, t1 = c_null_ptr
     integer(c_int32_t) :: n_mu = 0
     type(c_ptr) :: mu0 = c_null_ptr, mu1 = c_null_ptr
     integer(c_int32_t) :: n_e = 0
     type(c_ptr) :: E0 = c_null_ptr, E1 = c_null_ptr
  end type c2d_obs_bins

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

     integer(c_int) function c2d_tally_download_range(ctx, host, offset, n) &
         bind(C, name='c2d_tally_download_range')
       import :: c_int, c_ptr, c_double, c_int64_t
       type(c_ptr), value :: ctx
       real(c_double), intent(out) :: host(*)
       integer(c_int64_t), value :: offset, n
     end function c2d_tally_download_range

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

     integer(c_int) function c2d_fp_set_config(ctx, fcfg) bind(C, name='c2d_fp_set_config')
       import :: c_int, c_ptr, c2d_fp_config
       type(c_ptr), value :: ctx
       type(c2d_fp_config), intent(in) :: fcfg
     end function c2d_fp_set_config

     ! C2D_FP_EXACT (default, bit for bit the reference order) | C2D_FP_FAST
     ! | C2D_FP_AUTO (per update: exact on the tea clamp, fast off it)
     integer(c_int) function c2d_fp_set_mode(ctx, mode) bind(C, name='c2d_fp_set_mode')
       import :: c_int, c_ptr, c_int32_t
       type(c_ptr), value :: ctx
       integer(c_int32_t), value :: mode
     end function c2d_fp_set_mode

     integer(c_int) function c2d_last_fp_mode(ctx, mode) bind(C, name='c2d_last_fp_mode')
       import :: c_int, c_ptr, c_int32_t
       type(c_ptr), value :: ctx
       integer(c_int32_t), intent(out) :: mode
     end function c2d_last_fp_mode

     integer(c_int) function c2d_fp_step(ctx, fin, fout) bind(C, name='c2d_fp_step')
       import :: c_int, c_ptr, c2d_fp_step_in, c2d_fp_step_out
       type(c_ptr), value :: ctx
       type(c2d_fp_step_in), intent(in) :: fin
       type(c2d_fp_step_out), intent(inout) :: fout
     end function c2d_fp_step

     integer(c_int) function c2d_volume_em(ctx, vin, vout) bind(C, name='c2d_volume_em')
       import :: c_int, c_ptr, c2d_vem_in, c2d_vem_out
       type(c_ptr), value :: ctx
       type(c2d_vem_in), intent(in) :: vin
       type(c2d_vem_out), intent(inout) :: vout
     end function c2d_volume_em

     integer(c_int) function c2d_obs_begin(ctx, bins) bind(C, name='c2d_obs_begin')
       import :: c_int, c_ptr, c2d_obs_bins
       type(c_ptr), value :: ctx
       type(c2d_obs_bins), intent(in) :: bins
     end function c2d_obs_begin

     integer(c_int) function c2d_obs_accumulate(ctx, events, n) bind(C, name='c2d_obs_accumulate')
       import :: c_int, c_ptr, c_int64_t
       type(c_ptr), value :: ctx, events           ! c_null_ptr: device events of the last step
       integer(c_int64_t), value :: n
     end function c2d_obs_accumulate

     integer(c_int) function c2d_obs_result(ctx, F, F2, cnt, kernel_ms) bind(C, name='c2d_obs_result')
       import :: c_int, c_ptr, c_double
       type(c_ptr), value :: ctx, F, F2, cnt       ! [n_e, n_mu, n_t] in Fortran order
       real(c_double), intent(out) :: kernel_ms
     end function c2d_obs_result

     ! pspt's dialogue (one answer a line, C string) -> the SED binning
     integer(c_int) function c2d_obs_begin_pspt(ctx, deck) bind(C, name='c2d_obs_begin_pspt')
       import :: c_int, c_ptr, c_char
       type(c_ptr), value :: ctx
       character(kind=c_char), intent(in) :: deck(*)   ! NUL-terminated
     end function c2d_obs_begin_pspt

     ! pspt's output file from the histogram so far (path NUL-terminated,
     ! empty = the deck's name); world_sum: summed over the communicator
     integer(c_int) function c2d_obs_write_pspt(ctx, path, factor, world_sum) &
          bind(C, name='c2d_obs_write_pspt')
       import :: c_int, c_ptr, c_char, c_int32_t
       type(c_ptr), value :: ctx
       character(kind=c_char), intent(in) :: path(*)
       integer(c_int32_t), value :: factor, world_sum
     end function c2d_obs_write_pspt

     ! ---- RCCL tally all-reduce (replaces xec_add / graphics_collect,
     !      src/xec2d.f:325-399, and cens_add_up / E_add_up,
     !      src/update2d.f:1929-2078): rank 0 makes the id, the host
     !      broadcasts it (MPI_Bcast of C2D_COMM_ID_BYTES bytes) ----
     integer(c_int) function c2d_comm_unique_id(id, cap) bind(C, name='c2d_comm_unique_id')
       import :: c_int, c_int8_t, c_int64_t
       integer(c_int8_t), intent(out) :: id(*)
       integer(c_int64_t), value :: cap
     end function c2d_comm_unique_id

     integer(c_int) function c2d_comm_init(ctx, id, rank, world) bind(C, name='c2d_comm_init')
       import :: c_int, c_ptr, c_int8_t, c_int32_t
       type(c_ptr), value :: ctx
       integer(c_int8_t), intent(in) :: id(*)
       integer(c_int32_t), value :: rank, world
     end function c2d_comm_init

     integer(c_int) function c2d_allreduce_tallies(ctx) bind(C, name='c2d_allreduce_tallies')
       import :: c_int, c_ptr
       type(c_ptr), value :: ctx
     end function c2d_allreduce_tallies

     integer(c_int) function c2d_device_count(n) bind(C, name='c2d_device_count')
       import :: c_int, c_int32_t
       integer(c_int32_t), intent(out) :: n
     end function c2d_device_count

     integer(c_int) function c2d_electron_state(ctx, f_nt, Pnt) bind(C, name='c2d_electron_state')
       import :: c_int, c_ptr, c2d_marray3
       type(c_ptr), value :: ctx
       type(c2d_marray3), value :: f_nt, Pnt
     end function c2d_electron_state

     integer(c_int) function c2d_census_export_range(ctx, first, stride, d6, i5, keys, cap, n) &
          bind(C, name='c2d_census_export_range')
       import :: c_int, c_ptr, c_double, c_int32_t, c_int64_t
       type(c_ptr), value :: ctx
       integer(c_int64_t), value :: first, stride
       real(c_double), intent(out) :: d6(6, *)
       integer(c_int32_t), intent(out) :: i5(5, *)
       integer(c_int64_t), intent(out) :: keys(*)
       integer(c_int64_t), value :: cap
       integer(c_int64_t), intent(out) :: n
     end function c2d_census_export_range
  end interface
end module compton2d
