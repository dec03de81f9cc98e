! fortran_fp_driver.f90 -- the reference's `call update` (src/xec2d.f:86-87,
! src/update2d.f:7-327) replaced by c2d_fp_step on the MI355X.
!
! The electron state lives in arrays with the reference's COMMON extents and
! layouts (src/general.pa: jmax=kmax=99, num_nt=200, nphfield=400;
! f_nt(jmax,kmax,num_nt), Pnt(...), n_field(nphfield,jmax,kmax),
! F_IC(num_nt,nphfield), zone arrays (jmax,kmax)) and is handed to the
! library in place via (c_loc, strides); the library updates f_nt, Pnt, n_e,
! tea, gmin, gmax, amxwl, p_nth and Te_new where FP_recv_result/update
! would.  Inputs: a stream file written by tests/test_fortran_binding.py (the
! reference's FP inputs of a golden case); output: the updated arrays.
!
! usage: fortran_fp_driver CASE.bin OUT.bin
program fortran_fp_driver
  use compton2d
  implicit none
  integer, parameter :: jmax = 99, kmax = 99, n_vol = 400, num_nt = 200, nphfield = 400
  real(c_double), target, save :: f_nt(jmax, kmax, num_nt), Pnt(jmax, kmax, num_nt)
  real(c_double), target, save :: n_field(nphfield, jmax, kmax), F_IC(num_nt, nphfield)
  real(c_double), target, save :: tea(jmax, kmax), tna(jmax, kmax), n_e(jmax, kmax), &
       B_field(jmax, kmax), Eloss_sy(jmax, kmax), ecens(jmax, kmax), ec_old(jmax, kmax), &
       turb_lev(jmax, kmax), vol(jmax, kmax), f_pair(jmax, kmax), gmin(jmax, kmax), &
       gmax(jmax, kmax), amxwl(jmax, kmax), p_nth(jmax, kmax), Te_new(jmax, kmax)
  real(c_double), target :: z(jmax), r(kmax), E_ph(n_vol), E_field(nphfield), gnt(num_nt)
  real(c_double), target :: hu(129), Elcmin(10), Elcmax(10), mu(32)
  real(c_double) :: consts(22)
  integer(c_int32_t) :: ints(6)
  type(c2d_config) :: cfg
  type(c2d_fp_config) :: fcfg
  type(c2d_fp_step_in) :: fin
  type(c2d_fp_step_out) :: fout
  type(c_ptr) :: ctx
  integer(c_int32_t) :: nz, nr, nphtotal, nph_lc, nmu, nsteps, ncycle
  real(c_double) :: rmin, zmin, time, dt
  integer :: i, j, k, n, u, v, rc
  integer(c_int64_t), parameter :: one = 1, jm = jmax, jk = jmax * kmax
  character(len=512) :: cin, cout
  character(kind=c_char), pointer :: msg(:)

  call get_command_argument(1, cin)
  call get_command_argument(2, cout)
  open(newunit=u, file=trim(cin), access='stream', form='unformatted', status='old')
  read(u) nz, nr, nphtotal, nph_lc, nmu, nsteps
  read(u) rmin, zmin
  read(u) (z(j), j = 1, nz), (r(k), k = 1, nr)
  read(u) E_ph, E_field, gnt
  read(u) (hu(i), i = 1, nphtotal + 1), (Elcmin(i), i = 1, nph_lc), (Elcmax(i), i = 1, nph_lc), &
       (mu(i), i = 1, nmu)
  read(u) ints, consts
  read(u) F_IC

  cfg%nz = nz; cfg%nr = nr; cfg%rmin = rmin; cfg%zmin = zmin
  cfg%z = c_loc(z); cfg%r = c_loc(r); cfg%E_ph = c_loc(E_ph); cfg%E_field = c_loc(E_field)
  cfg%gnt = c_loc(gnt); cfg%nphtotal = nphtotal; cfg%hu = c_loc(hu)
  cfg%nph_lc = nph_lc; cfg%Elcmin = c_loc(Elcmin); cfg%Elcmax = c_loc(Elcmax)
  cfg%nmu = nmu; cfg%mu = c_loc(mu)
  cfg%census_capacity = 1024; cfg%event_capacity = 1024; cfg%queue_capacity = 1024
  rc = c2d_init(cfg, ctx)
  if (rc /= C2D_OK) then
     write(*, '(a,i0)') 'c2d_init failed: ', rc
     if (c_associated(ctx)) call print_error(ctx)
     stop 3
  end if

  ! setup_bcast / FP_bcast once: run constants and the IC loss kernel
  fcfg%pair_switch = 0
  fcfg%cf_sentinel = ints(1); fcfg%inj_switch = ints(2); fcfg%inj_dis = ints(3)
  fcfg%g2var_switch = ints(4); fcfg%pick_sw = ints(5)
  fcfg%df_implicit = consts(1); fcfg%df_T = consts(2); fcfg%r_esc = consts(3)
  fcfg%r_acc = consts(4); fcfg%r_flare = consts(5); fcfg%z_flare = consts(6)
  fcfg%t_flare = consts(7); fcfg%sigma_r = consts(8); fcfg%sigma_z = consts(9)
  fcfg%sigma_t = consts(10); fcfg%flare_amp = consts(11); fcfg%inj_g1 = consts(12)
  fcfg%inj_g2 = consts(13); fcfg%inj_p = consts(14); fcfg%inj_t = consts(15)
  fcfg%inj_L = consts(16); fcfg%pick_rate = consts(17); fcfg%inj_gg = consts(18)
  fcfg%inj_sigma = consts(19); fcfg%inj_v = consts(20)
  fcfg%F_IC = c_loc(F_IC); fcfg%F_IC_s_i = 1; fcfg%F_IC_s_ph = num_nt
  rc = c2d_fp_set_config(ctx, fcfg)
  if (rc /= C2D_OK) then
     call print_error(ctx)
     stop 4
  end if

  ! the COMMON arrays in place: (i,j,k) 0-based at data[i*s_i + j*s_j + k*s_k]
  fin%tea = c2d_array2(c_loc(tea), one, jm);  fin%tna = c2d_array2(c_loc(tna), one, jm)
  fin%n_e = c2d_array2(c_loc(n_e), one, jm);  fin%B_field = c2d_array2(c_loc(B_field), one, jm)
  fin%Eloss_sy = c2d_array2(c_loc(Eloss_sy), one, jm)
  fin%ec_old = c2d_array2(c_loc(ec_old), one, jm)
  fin%turb_lev = c2d_array2(c_loc(turb_lev), one, jm)
  fin%vol = c2d_array2(c_loc(vol), one, jm);  fin%f_pair = c2d_array2(c_loc(f_pair), one, jm)
  fin%ecens = c2d_array2(c_loc(ecens), one, jm)
  fin%n_field = c2d_array3(c_loc(n_field), one, int(nphfield, c_int64_t), int(nphfield, c_int64_t) * jm)
  fout%f_nt = c2d_marray3(c_loc(f_nt), jk, one, jm)
  fout%Pnt = c2d_marray3(c_loc(Pnt), jk, one, jm)
  fout%Te_new = c2d_marray2(c_loc(Te_new), one, jm); fout%tea = c2d_marray2(c_loc(tea), one, jm)
  fout%n_e = c2d_marray2(c_loc(n_e), one, jm);   fout%gmin = c2d_marray2(c_loc(gmin), one, jm)
  fout%gmax = c2d_marray2(c_loc(gmax), one, jm); fout%amxwl = c2d_marray2(c_loc(amxwl), one, jm)
  fout%p_nth = c2d_marray2(c_loc(p_nth), one, jm)

  open(newunit=v, file=trim(cout), access='stream', form='unformatted', status='replace')
  do n = 1, nsteps
     read(u) ncycle, time, dt
     read(u) ((tea(j, k), k = 1, nr), j = 1, nz), ((tna(j, k), k = 1, nr), j = 1, nz), &
          ((n_e(j, k), k = 1, nr), j = 1, nz), ((B_field(j, k), k = 1, nr), j = 1, nz), &
          ((Eloss_sy(j, k), k = 1, nr), j = 1, nz), ((ecens(j, k), k = 1, nr), j = 1, nz), &
          ((ec_old(j, k), k = 1, nr), j = 1, nz), ((turb_lev(j, k), k = 1, nr), j = 1, nz), &
          ((vol(j, k), k = 1, nr), j = 1, nz), ((f_pair(j, k), k = 1, nr), j = 1, nz), &
          ((gmin(j, k), k = 1, nr), j = 1, nz), ((gmax(j, k), k = 1, nr), j = 1, nz), &
          ((amxwl(j, k), k = 1, nr), j = 1, nz), ((p_nth(j, k), k = 1, nr), j = 1, nz)
     read(u) (((f_nt(j, k, i), i = 1, num_nt), k = 1, nr), j = 1, nz)
     read(u) (((Pnt(j, k, i), i = 1, num_nt), k = 1, nr), j = 1, nz)
     read(u) (((n_field(i, j, k), i = 1, nphfield), k = 1, nr), j = 1, nz)
     fin%ncycle = ncycle; fin%time = time; fin%dt = dt
     ! call update  (src/xec2d.f:86-87)
     rc = c2d_fp_step(ctx, fin, fout)
     if (rc /= C2D_OK) then
        write(*, '(a,i0)') 'c2d_fp_step failed: ', rc
        call print_error(ctx)
        stop 5
     end if
     write(v) fout%E_tot_old, fout%E_tot_new, fout%hr_total, fout%hr_st_total, fout%dT_max
     write(v) ((Te_new(j, k), k = 1, nr), j = 1, nz), ((tea(j, k), k = 1, nr), j = 1, nz), &
          ((n_e(j, k), k = 1, nr), j = 1, nz), ((gmin(j, k), k = 1, nr), j = 1, nz), &
          ((gmax(j, k), k = 1, nr), j = 1, nz), ((amxwl(j, k), k = 1, nr), j = 1, nz), &
          ((p_nth(j, k), k = 1, nr), j = 1, nz)
     write(v) (((f_nt(j, k, i), i = 1, num_nt), k = 1, nr), j = 1, nz)
     write(v) (((Pnt(j, k, i), i = 1, num_nt), k = 1, nr), j = 1, nz)
     write(*, '(a,i0,a,es14.7)') 'update ', ncycle, ': dT_max ', fout%dT_max
  end do
  close(u)
  close(v)
  call c2d_finalize(ctx)

contains
  subroutine print_error(c)
    type(c_ptr), intent(in) :: c
    type(c_ptr) :: p
    integer :: m
    p = c2d_last_error(c)
    call c_f_pointer(p, msg, [512])
    do m = 1, 512
       if (msg(m) == c_null_char) exit
       write(*, '(a)', advance='no') msg(m)
    end do
    write(*, *)
  end subroutine print_error
end program fortran_fp_driver
