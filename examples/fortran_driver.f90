! fortran_driver.f90 -- the reference's Fortran host calling the MI355X engine.
!
! Holds the transport tables in arrays with the reference's COMMON extents
! (src/general.pa: n_vol=400, jmax=kmax=99, num_nt=200; layouts of
! src/commonblock.f:53-70), passes them to c2d_transport_step in place via
! (c_loc, strides), and runs NSTEPS steps.  Inputs: a stream file written by
! tests/test_fortran_binding.py (the golden case's step tables, only the
! [1:nz,1:nr] block); output: the fused tally buffer of every step after
! the RCCL all-reduce that replaces xec_add / cens_add_up (one rank here: an
! MPI host broadcasts the id from rank 0 and passes its own rank / size).
!
! usage: fortran_driver CASE.bin OUT.bin
program fortran_driver
  use compton2d
  implicit none
  integer, parameter :: jmax = 99, kmax = 99, n_vol = 400, num_nt = 200, nphfield = 400
  real(c_double), target, save :: kappa_tot(n_vol, jmax, kmax), eps_tot(n_vol, jmax, kmax), &
       eps_th(n_vol, jmax, kmax), f_nt(jmax, kmax, num_nt), Pnt(jmax, kmax, num_nt)
  real(c_double), target, save :: n_e(jmax, kmax), Eloss_th(jmax, kmax), Eloss_tot(jmax, kmax), &
       zsurf(jmax, kmax), ewsv(jmax, kmax)
  integer(c_int32_t), target, save :: nsv(jmax, kmax)
  real(c_double), target :: z(jmax), r(kmax), E_ph(n_vol), E_field(nphfield), gnt(num_nt)
  real(c_double), target :: hu(129), Elcmin(10), Elcmax(10), mu(32)
  integer(c_int32_t), target :: nsurfi(jmax), nsurfo(jmax), nsurfu(kmax), nsurfl(kmax)
  real(c_double), target :: ewsurfi(jmax), ewsurfo(jmax), ewsurfu(kmax), ewsurfl(kmax)
  real(c_double), target :: tbbi(jmax), tbbo(jmax), tbbu(kmax), tbbl(kmax)
  real(c_double), allocatable :: tal(:), tal_raw(:)
  integer(c_int8_t) :: comm_id(C2D_COMM_ID_BYTES)
  type(c2d_config) :: cfg
  type(c2d_step_in) :: sin
  type(c2d_tally_layout) :: lay
  type(c_ptr) :: ctx
  integer(c_int32_t) :: nz, nr, nphtotal, nph_lc, nmu, nsteps, s1, s2, s3, s4, ncycle, mode
  real(c_double) :: rmin, zmin, time, dt
  integer :: i, j, k, n, u, v, rc
  character(len=512) :: fin, fout
  character(kind=c_char), pointer :: msg(:)

  call get_command_argument(1, fin)
  call get_command_argument(2, fout)
  open(newunit=u, file=trim(fin), access='stream', form='unformatted', status='old')
  read(u) nz, nr, nphtotal, nph_lc, nmu, nsteps, s1, s2, s3, s4, mode
  read(u) rmin, zmin
  read(u) (z(j), j = 1, nz), (r(k), k = 1, nr)
  read(u) E_ph, E_field, gnt
  read(u) (hu(i), i = 1, nphtotal + 1), (Elcmin(i), i = 1, nph_lc), (Elcmax(i), i = 1, nph_lc), &
       (mu(i), i = 1, nmu)

  cfg%nz = nz; cfg%nr = nr; cfg%rmin = rmin; cfg%zmin = zmin
  cfg%z = c_loc(z); cfg%r = c_loc(r); cfg%E_ph = c_loc(E_ph); cfg%E_field = c_loc(E_field)
  cfg%gnt = c_loc(gnt); cfg%nphtotal = nphtotal; cfg%hu = c_loc(hu)
  cfg%nph_lc = nph_lc; cfg%Elcmin = c_loc(Elcmin); cfg%Elcmax = c_loc(Elcmax)
  cfg%nmu = nmu; cfg%mu = c_loc(mu)
  cfg%split1 = s1; cfg%split2 = s2; cfg%split3 = s3; cfg%spl3_trg = s4
  cfg%comtot_mode = mode; cfg%seed = int(z'5EEDC2D', c_int64_t)
  cfg%census_capacity = 1048576; cfg%event_capacity = 1048576; cfg%queue_capacity = 262144
  rc = c2d_init(cfg, ctx)
  if (rc /= C2D_OK) then
     write(*, '(a,i0)') 'c2d_init failed: ', rc
     if (c_associated(ctx)) call print_error(ctx)
     stop 3
  end if
  rc = c2d_tally_layout_get(ctx, lay)
  allocate(tal(lay%total), tal_raw(lay%total))
  ! RCCL communicator for the per-step tally all-reduce: rank 0 of 1 here;
  ! under MPI: if (myid == 0) c2d_comm_unique_id, MPI_Bcast(comm_id), then
  ! c2d_comm_init(ctx, comm_id, myid, numprocs)
  rc = c2d_comm_unique_id(comm_id, int(C2D_COMM_ID_BYTES, c_int64_t))
  if (rc == C2D_OK) rc = c2d_comm_init(ctx, comm_id, 0_c_int32_t, 1_c_int32_t)
  if (rc /= C2D_OK) then
     write(*, '(a,i0)') 'c2d_comm_init failed: ', rc
     call print_error(ctx)
     stop 5
  end if
  open(newunit=v, file=trim(fout), access='stream', form='unformatted', status='replace')

  ! the COMMON arrays, described in place: element (i,j,k) 0-based at
  ! data[i*s_i + j*s_j + k*s_k]
  sin%kappa_tot = c2d_array3(c_loc(kappa_tot), 1_c_int64_t, int(n_vol, c_int64_t), &
       int(n_vol * jmax, c_int64_t))
  sin%eps_tot = c2d_array3(c_loc(eps_tot), 1_c_int64_t, int(n_vol, c_int64_t), &
       int(n_vol * jmax, c_int64_t))
  sin%eps_th = c2d_array3(c_loc(eps_th), 1_c_int64_t, int(n_vol, c_int64_t), &
       int(n_vol * jmax, c_int64_t))
  sin%f_nt = c2d_array3(c_loc(f_nt), int(jmax * kmax, c_int64_t), 1_c_int64_t, &
       int(jmax, c_int64_t))
  sin%Pnt = c2d_array3(c_loc(Pnt), int(jmax * kmax, c_int64_t), 1_c_int64_t, &
       int(jmax, c_int64_t))
  sin%n_e = c2d_array2(c_loc(n_e), 1_c_int64_t, int(jmax, c_int64_t))
  sin%Eloss_th = c2d_array2(c_loc(Eloss_th), 1_c_int64_t, int(jmax, c_int64_t))
  sin%Eloss_tot = c2d_array2(c_loc(Eloss_tot), 1_c_int64_t, int(jmax, c_int64_t))
  sin%zsurf = c2d_array2(c_loc(zsurf), 1_c_int64_t, int(jmax, c_int64_t))
  sin%ewsv = c2d_array2(c_loc(ewsv), 1_c_int64_t, int(jmax, c_int64_t))
  sin%nsv = c2d_array2(c_loc(nsv), 1_c_int64_t, int(jmax, c_int64_t))
  sin%nsurfi = c_loc(nsurfi); sin%nsurfo = c_loc(nsurfo)
  sin%nsurfu = c_loc(nsurfu); sin%nsurfl = c_loc(nsurfl)
  sin%ewsurfi = c_loc(ewsurfi); sin%ewsurfo = c_loc(ewsurfo)
  sin%ewsurfu = c_loc(ewsurfu); sin%ewsurfl = c_loc(ewsurfl)
  sin%tbbi = c_loc(tbbi); sin%tbbo = c_loc(tbbo); sin%tbbu = c_loc(tbbu); sin%tbbl = c_loc(tbbl)

  do n = 1, nsteps
     read(u) ncycle, time, dt
     read(u) (((kappa_tot(i, j, k), i = 1, n_vol), k = 1, nr), j = 1, nz)
     read(u) (((eps_tot(i, j, k), i = 1, n_vol), k = 1, nr), j = 1, nz)
     read(u) (((eps_th(i, j, k), i = 1, n_vol), k = 1, nr), j = 1, nz)
     read(u) (((f_nt(j, k, i), i = 1, num_nt), k = 1, nr), j = 1, nz)
     read(u) (((Pnt(j, k, i), i = 1, num_nt), k = 1, nr), j = 1, nz)
     read(u) ((n_e(j, k), k = 1, nr), j = 1, nz), ((Eloss_th(j, k), k = 1, nr), j = 1, nz), &
          ((Eloss_tot(j, k), k = 1, nr), j = 1, nz), ((zsurf(j, k), k = 1, nr), j = 1, nz), &
          ((ewsv(j, k), k = 1, nr), j = 1, nz)
     read(u) ((nsv(j, k), k = 1, nr), j = 1, nz)
     read(u) (nsurfi(j), j = 1, nz), (nsurfo(j), j = 1, nz), (nsurfu(k), k = 1, nr), &
          (nsurfl(k), k = 1, nr)
     read(u) (ewsurfi(j), j = 1, nz), (ewsurfo(j), j = 1, nz), (ewsurfu(k), k = 1, nr), &
          (ewsurfl(k), k = 1, nr)
     read(u) (tbbi(j), j = 1, nz), (tbbo(j), j = 1, nz), (tbbu(k), k = 1, nr), (tbbl(k), k = 1, nr)
     sin%ncycle = ncycle; sin%time = time; sin%dt = dt
     ! imcfield2d + imcvol2d + imcsurf2d of this step (src/xec2d.f:167-176)
     rc = c2d_transport_step(ctx, sin)
     if (rc /= C2D_OK) then
        write(*, '(a,i0)') 'c2d_transport_step failed: ', rc
        call print_error(ctx)
        stop 4
     end if
     rc = c2d_tally_download(ctx, tal_raw, lay%total)
     ! xec_add + graphics_collect + cens_add_up: one all-reduce of the fused buffer
     rc = c2d_allreduce_tallies(ctx)
     if (rc /= C2D_OK) then
        write(*, '(a,i0)') 'c2d_allreduce_tallies failed: ', rc
        call print_error(ctx)
        stop 6
     end if
     rc = c2d_tally_download(ctx, tal, lay%total)
     if (all(transfer(tal, 0_c_int64_t, size(tal)) == transfer(tal_raw, 0_c_int64_t, size(tal_raw)))) then
        write(*, '(a)') 'allreduce: bitwise identical (1 rank)'
     else
        write(*, '(a)') 'allreduce: MISMATCH'
     end if
     write(v) tal
     write(*, '(a,i0,a,f0.0,a,f0.0)') 'step ', ncycle, ': packet-steps ', &
          tal(lay%counters + C2D_CNT_STEPS + 1), ' census ', tal(lay%counters + C2D_CNT_CENSUS + 1)
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
end program fortran_driver
