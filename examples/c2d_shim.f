c     c2d_shim.f -- drop-in replacements of the reference's per-step
c     transport and Fokker-Planck entry points over the MI355X
c     engine's C-ABI (include/compton2d.h via include/compton2d_mod.f90).
c
c     The reference's master/worker loop (src/xec2d.f:41-193) calls five
c     argument-less subroutines that talk through COMMON
c     (src/commonblock.f).  This file defines the same five names; link
c     it ahead of the reference's own objects with those five entry
c     points weakened (oracle/ref/build_shim.sh: objcopy
c     --weaken-symbol), together with the reference's main program
c     (src/compton2d.f), reader, setup, xec, imcgen2d, graphics,
c     write_record ... unchanged:
c
c       src/imcfield2d.f:5      imcfield2d  one c2d_transport_step per
c                                           worker GPU: census + volume +
c                                           surface sources of the step
c       src/imcvol2d_para.f:1   imcvol2d    (done in imcfield2d)
c       src/imcsurf2d_para.f:1  imcsurf2d   (done in imcfield2d)
c       src/imcredist.f:5       imcredist   (census stays on its GPU)
c       src/update2d.f:7        update      cens_add_up, c2d_fp_step for
c                                           every zone on the master,
c                                           E_add_up, FP_end_bcast
c
c     Ranks as in the reference: rank 0 (master) schedules and runs no
c     transport; ranks 1..numprocs-1 are workers, one GPU each (device
c     mod(myid-1, GPUs visible)), with the step's sources sharded over
c     them by lineage (c2d_config rank/world).  Each worker's step
c     tallies are ADDED into its COMMON exactly where the reference's
c     workers accumulate them (edep, prdep, ecens, npcen, n_field, E_IC,
c     nelectron, fout, edout, erlk*, Ed_in), so xec_add,
c     graphics_collect, cens_add_up and E_add_up reduce them unchanged;
c     escape events are binned on the GPU into the time-resolved SED of
c     the post-processing tool pspt (postprocessing/pspt.c: its binning
c     from its own input deck, its output file, rewritten every step;
c     N workers: summed over them inside the C-ABI) instead of being
c     written as text -- or, opted in, written to the worker's event file
c     (unit nunit_evt, the reference's format, src/imcleak2d.f:171,181)
c     for the stand-alone tools; the census is mirrored
c     into dbufout/ibufout/ndxout for write_record (src/census2d.f) when
c     it fits ucens, and imported from them after read_record.
c
c     Environment: C2D_SHIM_EXACT=1 (exact comtot build),
c     C2D_SHIM_CENSUS_CAPACITY=n,
c     C2D_SHIM_SED_DECK=path (pspt's input deck, e.g.
c     postprocessing/mrk421_sed.input; unset: pspt's defaults),
c     C2D_SHIM_SED=0 (no on-device SED),
c     C2D_SHIM_EVENTS=1 (also write the event file),
c     C2D_SHIM_CENSUS_MIRROR=1|0 (dbufout mirror every step | never;
c     default: only near write_record's elapsed-time mark),
c     C2D_SHIM_FP_MODE=0|1|2 (exact | fast | auto FP, default auto,
c     c2d_fp_set_mode), C2D_SHIM_FP_FAST=1 (= C2D_SHIM_FP_MODE=1),
c     C2D_SHIM_ALLREDUCE=0 (N workers: no all-reduce inside the C-ABI;
c     every worker deposits its own tallies into COMMON instead).
c     Errors print the library's message and MPI_ABORT (the reference
c     `stop`s, src/imctrk2d.f:573-577).
c
      module c2d_shim_state
      use iso_c_binding
      use compton2d
      implicit none
c     worker transport context / master FP context
      type(c_ptr), save :: tctx = c_null_ptr, fctx = c_null_ptr
      logical, save :: tready = .false., fready = .false.
      type(c2d_tally_layout), save :: lay
      real(c_double), allocatable, target, save :: tal(:)
c     file_sp tables of this step's file-spectrum surface slots
c     (2*jmax + 2*kmax slots x 5 tables of nfmax)
      integer, parameter :: shm_nslot = 396, shm_nf = 500
      type(c2d_spectrum), target, save :: spec(shm_nslot)
      real(c_double), target, save :: sptab(shm_nf, 5, shm_nslot)
      integer(c_int32_t), target, save :: sidx_i(99), sidx_o(99),
     1     sidx_u(99), sidx_l(99)
      integer, save :: ev_on = 0, mirror_on = 2, warned = 0
c     census mirror (mode 2): write_record's mark in seconds of etotal
c     (C2D_SHIM_MIRROR_MARK overrides it, a test hook) and the latch that
c     keeps the mirror on every step once it has started
      double precision, save :: mirror_mark = (0.95d0*480.d0-3.d0)*60.d0
      logical, save :: mir_latch = .false.
c     test hook (C2D_SHIM_WRITE_CENS=1): after every mirror, write the
c     mirrored census as write_record would (write_record.f:433-437)
      integer, save :: wcens_on = 0
c     the on-device SED (c2d_obs_begin_pspt / c2d_obs_write_pspt)
      integer, save :: sed_on = 1
      logical, save :: static_done = .false.
c     the run's lineage seed: the master's rseed, the same on every
c     worker (setup_bcast leaves each worker rseed + myid*84725,
c     src/fp_mpi.f:66-68)
      integer, save :: seed0 = 0
c     N workers: the step's tallies all-reduced over the workers inside
c     the C-ABI (c2d_comm_init / c2d_allreduce_tallies: one RCCL
c     all-reduce of the fused buffer), deposited into COMMON by worker 1
c     only (C2D_SHIM_ALLREDUCE=0: every worker deposits its own share)
      integer, save :: ar_on = 0
      integer(c_int8_t), save :: commid(C2D_COMM_ID_BYTES)
      end module c2d_shim_state
c
c
c     print the engine's last error and abort every rank
      subroutine c2d_shim_fail(ctx, where, rc)
      use iso_c_binding
      use compton2d
      implicit none
      include 'mpif.h'
      type(c_ptr) ctx
      character*(*) where
      integer(c_int) rc
      character(kind=c_char), pointer :: msg(:)
      character*512 line
      integer i, ierr2
      line = ' '
      if (c_associated(ctx)) then
         call c_f_pointer(c2d_last_error(ctx), msg, [512])
         do 10 i = 1, 512
            if (msg(i) .eq. c_null_char) goto 11
            line(i:i) = msg(i)
 10      continue
 11      continue
      endif
      write(*,'(a,a,a,i0,a,a)') 'c2d_shim: ', where, ' failed: ', rc,
     1     ' ', trim(line)
      flush(6)
      call MPI_ABORT(MPI_COMM_WORLD, 3, ierr2)
      stop 3
      end
c
c
c     integer environment knob (default dflt)
      integer*8 function c2d_shim_env(name, dflt)
      implicit none
      character*(*) name
      integer*8 dflt
      character*32 v
      integer st
      c2d_shim_env = dflt
      call get_environment_variable(name, v, status=st)
      if (st .eq. 0) read(v, *) c2d_shim_env
      end
c
c
c     one engine context from the setup COMMON (src/setup2d.f): the
c     workers' transport context, or the master's FP-only context
      subroutine c2d_shim_init(ctx, rank, world, device, ccap, ecap,
     1                         qcap)
      use iso_c_binding
      use compton2d
      use c2d_shim_state, only: seed0
      implicit none
      include 'mpif.h'
      include 'general.pa'
      include 'commonblock.f'
      target :: z, r, E_ph, E_field, gnt, hu, Elcmin, Elcmax, mu
      type(c_ptr) ctx
      integer rank, world, device
      integer*8 ccap, ecap, qcap, c2d_shim_env
      type(c2d_config) :: cfg
      integer(c_int) rc
      cfg%nz = nz
      cfg%nr = nr
      cfg%rmin = rmin
      cfg%zmin = zmin
      cfg%z = c_loc(z)
      cfg%r = c_loc(r)
      cfg%E_ph = c_loc(E_ph)
      cfg%E_field = c_loc(E_field)
      cfg%gnt = c_loc(gnt)
      cfg%nphtotal = nphtotal
      cfg%hu = c_loc(hu)
      cfg%nph_lc = nph_lc
      cfg%Elcmin = c_loc(Elcmin)
      cfg%Elcmax = c_loc(Elcmax)
      cfg%nmu = nmu
      cfg%mu = c_loc(mu)
      cfg%split1 = split1
      cfg%split2 = split2
      cfg%split3 = split3
      cfg%spl3_trg = spl3_trg
      cfg%spec_switch = spec_switch
      cfg%cr_sent = cr_sent
      cfg%pair_switch = pair_switch
c     hazard H3: census + volume transport see the previous kappa_tot
      cfg%kappa_lag = 1
      cfg%comtot_mode = C2D_COMTOT_TABLE
      if (c2d_shim_env('C2D_SHIM_EXACT', 0_8) .eq. 1)
     1     cfg%comtot_mode = C2D_COMTOT_EXACT
      cfg%device = device
      cfg%seed = seed0
      cfg%rank = rank
      cfg%world = world
      cfg%census_capacity = ccap
      cfg%event_capacity = ecap
      cfg%queue_capacity = qcap
c     the tracker of the host's snapshot: src/ (0, default) or
c     src_20121113/ (1: the azimuth fix of hazard H1, compton2d.h)
      cfg%trk_variant = int(c2d_shim_env('C2D_SHIM_TRK_VARIANT', 0_8))
      rc = c2d_init(cfg, ctx)
      if (rc .ne. C2D_OK) call c2d_shim_fail(ctx, 'c2d_init', rc)
      end
c
c
      subroutine imcfield2d
      use iso_c_binding
      use compton2d
      use c2d_shim_state, only: tctx, tready, lay, tal, spec, sptab,
     1     sidx_i, sidx_o, sidx_u, sidx_l, ev_on, mirror_on, warned,
     2     static_done, seed0, ar_on, commid, sed_on, mirror_mark,
     3     mir_latch, wcens_on
      implicit none
      include 'mpif.h'
      include 'general.pa'
      include 'commonblock.f'
      target :: kappa_tot, eps_tot, eps_th, f_nt, Pnt, n_e, Eloss_th,
     1     Eloss_tot, zsurf, ewsv, nsv, nsurfi, nsurfo, ewsurfi,
     2     ewsurfo, nsurfu, nsurfl, ewsurfu, ewsurfl, dbufout
      double precision, allocatable :: pk(:), evb(:,:)
      integer(c_int32_t), allocatable :: i5(:,:)
      integer(c_int64_t), allocatable :: keys(:)
      double precision t_average
      double precision, target :: tbi(jmax), tbo(jmax), tbu(kmax),
     1     tbl(kmax)
      type(c2d_step_in) :: stin
      integer(c_int) rc
      integer(c_int32_t) ngpu
      integer(c_int64_t) nev, ncs, m
      integer*8 npk, ccap, ecap, qcap, c2d_shim_env
      integer i, j, k, n, l, nw, cell, nsp, ucf
      logical mir
      character*40 cfname
c
c     the time-window index of this step (imcsurf2d_para.f:55-64)
      if (myid .eq. master) then
         if (ncycle .eq. 0) then
            ti = 1
         else
            t_average = time + 5.d-1*dt(1)
            do 10 ti = 1, ntime
               if (t1(ti) .gt. t_average) goto 11
 10         continue
 11         continue
         endif
      endif
c
c     run constants the reference's workers receive with their surface
c     and volume jobs (reader.f; z_surf_bcast, vol_bcast), once
      if (.not. static_done) then
         call MPI_BCAST(nphtotal, 1, MPI_INTEGER, master,
     1        MPI_COMM_WORLD, ierr)
         call MPI_BCAST(nph_lc, 1, MPI_INTEGER, master,
     1        MPI_COMM_WORLD, ierr)
         call MPI_BCAST(spec_switch, 1, MPI_INTEGER, master,
     1        MPI_COMM_WORLD, ierr)
         call MPI_BCAST(ntime, 1, MPI_INTEGER, master,
     1        MPI_COMM_WORLD, ierr)
         call MPI_BCAST(nst, 1, MPI_INTEGER, master,
     1        MPI_COMM_WORLD, ierr)
         call MPI_BCAST(hu, nphomax+1, MPI_DOUBLE_PRECISION, master,
     1        MPI_COMM_WORLD, ierr)
         call MPI_BCAST(Elcmin, nphlcmax, MPI_DOUBLE_PRECISION,
     1        master, MPI_COMM_WORLD, ierr)
         call MPI_BCAST(Elcmax, nphlcmax, MPI_DOUBLE_PRECISION,
     1        master, MPI_COMM_WORLD, ierr)
         call MPI_BCAST(t0, ntmax, MPI_DOUBLE_PRECISION, master,
     1        MPI_COMM_WORLD, ierr)
         call MPI_BCAST(t1, ntmax, MPI_DOUBLE_PRECISION, master,
     1        MPI_COMM_WORLD, ierr)
         seed0 = rseed
         call MPI_BCAST(seed0, 1, MPI_INTEGER, master, MPI_COMM_WORLD,
     1        ierr)
c        the workers' exchange: worker 1 makes the unique id, every rank
c        takes part in its broadcast (128 bytes, once per run)
         if (numprocs .gt. 2) ar_on =
     1        int(c2d_shim_env('C2D_SHIM_ALLREDUCE', 1_8))
         if (ar_on .eq. 1) then
            if (myid .eq. 1) then
               rc = c2d_comm_unique_id(commid,
     1              int(C2D_COMM_ID_BYTES, c_int64_t))
               if (rc .ne. C2D_OK) call c2d_shim_fail(c_null_ptr,
     1              'c2d_comm_unique_id', rc)
            endif
            call MPI_BCAST(commid, C2D_COMM_ID_BYTES, MPI_BYTE, 1,
     1           MPI_COMM_WORLD, ierr)
         endif
         static_done = .true.
      endif
c
c     what the workers' jobs carry in the reference (vol_bcast,
c     z_surf_bcast, r_surf_bcast and the job messages): this step's
c     tables and budgets, packed to the [1:nz,1:nr] zones
      call MPI_BCAST(ti, 1, MPI_INTEGER, master, MPI_COMM_WORLD, ierr)
      call MPI_BCAST(dt, 2, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      npk = 3*n_vol*nz*nr
      allocate(pk(npk))
      if (myid .eq. master) then
         l = 0
         do 22 k = 1, nr
            do 21 j = 1, nz
               do 20 i = 1, n_vol
                  pk(l+1) = kappa_tot(i,j,k)
                  pk(l+2) = eps_tot(i,j,k)
                  pk(l+3) = eps_th(i,j,k)
                  l = l + 3
 20            continue
 21         continue
 22      continue
      endif
      call MPI_BCAST(pk, int(npk), MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      if (myid .ne. master) then
         l = 0
         do 25 k = 1, nr
            do 24 j = 1, nz
               do 23 i = 1, n_vol
                  kappa_tot(i,j,k) = pk(l+1)
                  eps_tot(i,j,k) = pk(l+2)
                  eps_th(i,j,k) = pk(l+3)
                  l = l + 3
 23            continue
 24         continue
 25      continue
      endif
      deallocate(pk)
      call MPI_BCAST(E_ph, n_vol, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(Eloss_th, jmax*kmax, MPI_DOUBLE_PRECISION,
     1     master, MPI_COMM_WORLD, ierr)
      call MPI_BCAST(Eloss_tot, jmax*kmax, MPI_DOUBLE_PRECISION,
     1     master, MPI_COMM_WORLD, ierr)
      call MPI_BCAST(ewsv, jmax*kmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(nsv, jmax*kmax, MPI_INTEGER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(nsurfi, jmax, MPI_INTEGER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(nsurfo, jmax, MPI_INTEGER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(nsurfu, kmax, MPI_INTEGER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(nsurfl, kmax, MPI_INTEGER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(ewsurfi, jmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(ewsurfo, jmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(ewsurfu, kmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(ewsurfl, kmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(tbbi, jmax*ntmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(tbbo, jmax*ntmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(tbbu, kmax*ntmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(tbbl, kmax*ntmax, MPI_DOUBLE_PRECISION, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(i_fname, 30*jmax*ntmax, MPI_CHARACTER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(o_fname, 30*jmax*ntmax, MPI_CHARACTER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(u_fname, 30*kmax*ntmax, MPI_CHARACTER, master,
     1     MPI_COMM_WORLD, ierr)
      call MPI_BCAST(l_fname, 30*kmax*ntmax, MPI_CHARACTER, master,
     1     MPI_COMM_WORLD, ierr)
c     the master schedules only (src/xec2d.f:70-83)
      if (myid .eq. master) return
c
c     ---- worker: one GPU context, lineage shard myid-1 of numprocs-1
      nw = numprocs - 1
      if (.not. tready) then
         rc = c2d_device_count(ngpu)
         if (rc .ne. C2D_OK .or. ngpu .lt. 1) ngpu = 1
         ccap = c2d_shim_env('C2D_SHIM_CENSUS_CAPACITY',
     1        max(int(ucens, 8), 10_8*int(nst, 8)/nw))
         ecap = max(1048576_8, 8_8*int(nst, 8)/nw)
         qcap = max(1048576_8, int(nst, 8)/nw)
         call c2d_shim_init(tctx, myid - 1, nw, mod(myid - 1, ngpu),
     1        ccap, ecap, qcap)
         rc = c2d_tally_layout_get(tctx, lay)
         allocate(tal(lay%total))
         ev_on = int(c2d_shim_env('C2D_SHIM_EVENTS', 0_8))
         mirror_on = int(c2d_shim_env('C2D_SHIM_CENSUS_MIRROR', 2_8))
         mirror_mark = dble(c2d_shim_env('C2D_SHIM_MIRROR_MARK',
     1        int(mirror_mark, 8)))
         wcens_on = int(c2d_shim_env('C2D_SHIM_WRITE_CENS', 0_8))
         sed_on = int(c2d_shim_env('C2D_SHIM_SED', 1_8))
c        N workers without the all-reduce cannot sum one SED: events
         if (sed_on .eq. 1 .and. nw .gt. 1 .and. ar_on .ne. 1) then
            sed_on = 0
            ev_on = 1
         endif
         if (sed_on .eq. 1) call c2d_shim_sed_begin(tctx)
c        restart: census records read by read_record (census2d.f)
         if (ndxout .gt. 0) then
            allocate(i5(5, ndxout), keys(ndxout))
            do 30 n = 1, ndxout
               do 29 i = 1, 5
                  i5(i, n) = ibufout(6*(n-1) + i)
 29            continue
               keys(n) = ibufout(6*n)
 30         continue
            rc = c2d_census_import(tctx, dbufout, i5, keys,
     1           int(ndxout, c_int64_t))
            if (rc .ne. C2D_OK) call c2d_shim_fail(tctx,
     1           'c2d_census_import', rc)
            deallocate(i5, keys)
         endif
         if (ar_on .eq. 1) then
            rc = c2d_comm_init(tctx, commid, int(myid - 1, c_int32_t),
     1           int(nw, c_int32_t))
            if (rc .ne. C2D_OK) call c2d_shim_fail(tctx,
     1           'c2d_comm_init', rc)
         endif
         tready = .true.
      endif
c
c     the step's inputs, COMMON arrays passed in place (pointer,
c     strides of the (n_vol|num_nt, jmax, kmax) extents)
      stin%ncycle = ncycle
      stin%time = time
      stin%dt = dt(1)
      stin%kappa_tot = c2d_array3(c_loc(kappa_tot), 1_c_int64_t,
     1     int(n_vol, c_int64_t), int(n_vol*jmax, c_int64_t))
      stin%eps_tot = c2d_array3(c_loc(eps_tot), 1_c_int64_t,
     1     int(n_vol, c_int64_t), int(n_vol*jmax, c_int64_t))
      stin%eps_th = c2d_array3(c_loc(eps_th), 1_c_int64_t,
     1     int(n_vol, c_int64_t), int(n_vol*jmax, c_int64_t))
      stin%f_nt = c2d_array3(c_loc(f_nt), int(jmax*kmax, c_int64_t),
     1     1_c_int64_t, int(jmax, c_int64_t))
      stin%Pnt = c2d_array3(c_loc(Pnt), int(jmax*kmax, c_int64_t),
     1     1_c_int64_t, int(jmax, c_int64_t))
      stin%n_e = c2d_array2(c_loc(n_e), 1_c_int64_t,
     1     int(jmax, c_int64_t))
      stin%Eloss_th = c2d_array2(c_loc(Eloss_th), 1_c_int64_t,
     1     int(jmax, c_int64_t))
      stin%Eloss_tot = c2d_array2(c_loc(Eloss_tot), 1_c_int64_t,
     1     int(jmax, c_int64_t))
      stin%zsurf = c2d_array2(c_loc(zsurf), 1_c_int64_t,
     1     int(jmax, c_int64_t))
      stin%ewsv = c2d_array2(c_loc(ewsv), 1_c_int64_t,
     1     int(jmax, c_int64_t))
      stin%nsv = c2d_array2(c_loc(nsv), 1_c_int64_t,
     1     int(jmax, c_int64_t))
      stin%nsurfi = c_loc(nsurfi)
      stin%nsurfo = c_loc(nsurfo)
      stin%nsurfu = c_loc(nsurfu)
      stin%nsurfl = c_loc(nsurfl)
      stin%ewsurfi = c_loc(ewsurfi)
      stin%ewsurfo = c_loc(ewsurfo)
      stin%ewsurfu = c_loc(ewsurfu)
      stin%ewsurfl = c_loc(ewsurfl)
c     boundary temperatures of time window ti; every surface slot that
c     emits with a file spectrum (tbb <= 0) gets file_sp's tables of
c     its file (imcsurf2d_para.f:544-685; the reference's workers call
c     file_sp per surface job)
      nsp = 0
      do 40 j = 1, nz
         tbi(j) = tbbi(j, ti)
         tbo(j) = tbbo(j, ti)
         sidx_i(j) = -1
         sidx_o(j) = -1
         if (nsurfi(j) .gt. 0 .and. tbi(j) .le. 0.d0) then
            call c2d_shim_spectrum(i_fname(j, ti), nsp)
            sidx_i(j) = nsp - 1
         endif
         if (nsurfo(j) .gt. 0 .and. tbo(j) .le. 0.d0) then
            call c2d_shim_spectrum(o_fname(j, ti), nsp)
            sidx_o(j) = nsp - 1
         endif
 40   continue
      do 41 k = 1, nr
         tbu(k) = tbbu(k, ti)
         tbl(k) = tbbl(k, ti)
         sidx_u(k) = -1
         sidx_l(k) = -1
         if (nsurfu(k) .gt. 0 .and. tbu(k) .le. 0.d0) then
            call c2d_shim_spectrum(u_fname(k, ti), nsp)
            sidx_u(k) = nsp - 1
         endif
         if (nsurfl(k) .gt. 0 .and. tbl(k) .le. 0.d0) then
            call c2d_shim_spectrum(l_fname(k, ti), nsp)
            sidx_l(k) = nsp - 1
         endif
 41   continue
      stin%tbbi = c_loc(tbi)
      stin%tbbo = c_loc(tbo)
      stin%tbbu = c_loc(tbu)
      stin%tbbl = c_loc(tbl)
      stin%spec_i = c_loc(sidx_i)
      stin%spec_o = c_loc(sidx_o)
      stin%spec_u = c_loc(sidx_u)
      stin%spec_l = c_loc(sidx_l)
      stin%n_spectra = nsp
      stin%spectra = c_loc(spec)
      stin%device_tables = 0
c
      rc = c2d_transport_step(tctx, stin)
      if (rc .ne. C2D_OK) call c2d_shim_fail(tctx,
     1     'c2d_transport_step', rc)
c
c     this worker's tallies (N workers: all workers', summed by one
c     all-reduce over the workers inside the C-ABI), added where the
c     reference's workers accumulate them (imctrk2d.f, compb_2d.f,
c     imcleak2d.f).  With the all-reduce only worker 1 deposits: the
c     reference's own reductions (xec_add, graphics_collect,
c     cens_add_up -- the latter 400 x nz x nr doubles per step) then
c     carry zeros from every other worker.
      if (ar_on .eq. 1) then
         rc = c2d_allreduce_tallies(tctx)
         if (rc .ne. C2D_OK) call c2d_shim_fail(tctx,
     1        'c2d_allreduce_tallies', rc)
      endif
      rc = c2d_tally_download(tctx, tal, lay%total)
      if (rc .ne. C2D_OK) call c2d_shim_fail(tctx,
     1     'c2d_tally_download', rc)
      if (ar_on .eq. 1 .and. myid .ne. 1) tal = 0.d0
      do 52 j = 1, nz
         do 51 k = 1, nr
            cell = (j-1)*nr + (k-1)
            edep(j,k) = edep(j,k) + tal(lay%edep + cell + 1)
            prdep(j,k) = prdep(j,k) + tal(lay%prdep + cell + 1)
            ecens(j,k) = ecens(j,k) + tal(lay%ecens + cell + 1)
            npcen(j,k) = npcen(j,k) + nint(tal(lay%npcen + cell + 1))
            do 50 i = 1, nphfield
               n_field(i,j,k) = n_field(i,j,k)
     1              + tal(lay%n_field + cell*nphfield + i)
 50         continue
 51      continue
 52   continue
      do 53 i = 1, num_nt
         E_IC(i) = E_IC(i) + tal(lay%E_IC + i + 1)
         nelectron(i) = nelectron(i)
     1        + nint(tal(lay%nelectron + i + 1))
 53   continue
      do 55 n = 1, nmu
         do 54 i = 1, nphomax
            fout(n,i) = fout(n,i) + tal(lay%fout + (n-1)*nphomax + i)
 54      continue
         do 56 i = 1, nph_lc
            edout(n,i) = edout(n,i)
     1           + tal(lay%edout + (n-1)*nphlcmax + i)
 56      continue
 55   continue
      do 57 j = 1, nz
         erlki(j) = erlki(j) + tal(lay%erlki + j)
         erlko(j) = erlko(j) + tal(lay%erlko + j)
 57   continue
      do 58 k = 1, nr
         erlku(k) = erlku(k) + tal(lay%erlku + k)
         erlkl(k) = erlkl(k) + tal(lay%erlkl + k)
         Ed_in(k) = Ed_in(k) + tal(lay%Ed_in + k)
 58   continue
c
c     escape events -> the SED on the device, rewritten every step (N
c     workers: summed over them; worker 1 writes)
      if (sed_on .eq. 1 .and. ncycle .gt. 0) then
         rc = c2d_obs_accumulate(tctx, c_null_ptr, 0_c_int64_t)
         if (rc .ne. C2D_OK) call c2d_shim_fail(tctx,
     1        'c2d_obs_accumulate', rc)
c        factor 1: what pspt prints for one series p001..pNNN_evb.dat
c        (pspt.c:222-238 counts the series end that is not p001)
         rc = c2d_obs_write_pspt(tctx, c_null_char, 1_c_int32_t,
     1        int(ar_on, c_int32_t))
         if (rc .ne. C2D_OK) call c2d_shim_fail(tctx,
     1        'c2d_obs_write_pspt', rc)
      endif
c     escape events -> this worker's event file (imcleak2d.f:171,181)
      if (ev_on .eq. 1 .and. ncycle .gt. 0) then
         rc = c2d_events(tctx, tal, 0_c_int64_t, nev)
         if (nev .gt. 0) then
            allocate(evb(7, nev))
            rc = c2d_events(tctx, evb, nev, m)
            do 60 n = 1, int(nev)
               write(nunit_evt, 105) (evb(i, n), i = 1, 7)
 60         continue
            deallocate(evb)
         endif
      endif
 105  format(6(e14.7,1x),e14.7)
c
c     census mirror for write_record (imctrk2d.f:558-572 layout:
c     6 f64 + 6 i32 per record, the 6th the record's seed), which is
c     the mirror's only reader: write_record runs once, at the start of
c     the step whose etotal (the master's elapsed time, COMMON, broadcast
c     by xec_bcast) passes the mark (0.95*wallm-3)*60 s, wallm = 480
c     minutes (xec2d.f:24,50,150).  That etotal is not known here, so
c     C2D_SHIM_CENSUS_MIRROR=2 (default) starts mirroring once etotal
c     plus two of its last increments passes 0.8 of the mark and then
c     mirrors every step to the end of the run (a step would have to
c     take ~90 minutes to jump the margin); 1: every step; 0: never (the
c     census stays on the GPU)
      rc = c2d_census_count(tctx, ncs)
      mir = mirror_on .eq. 1
      if (mirror_on .eq. 2) then
         if (.not. mir_latch .and. dble(etotal) + 2.d0 *
     1        max(dble(etotal) - dble(etotal_old), 0.d0) .gt.
     2        0.8d0*mirror_mark) then
            mir_latch = .true.
            write(*,*) 'c2d_shim: census mirror on from ncycle', ncycle
         endif
         mir = mir_latch
      endif
      if (mir .and. ncs .le. ucens) then
         allocate(i5(5, max(ncs, 1_8)), keys(max(ncs, 1_8)))
         rc = c2d_census_export(tctx, dbufout, i5, keys, ncs, m)
         do 70 n = 1, int(ncs)
            do 69 i = 1, 5
               ibufout(6*(n-1) + i) = i5(i, n)
 69         continue
            ibufout(6*n) = int(modulo(keys(n), 100000_8))
 70      continue
         ndxout = int(ncs)
         deallocate(i5, keys)
         if (wcens_on .eq. 1) then
            write(cfname, '(a,i3.3,a)') 'p', myid, '_census_mirror.dat'
            open(newunit=ucf, file=trim(cfname), status='replace')
            call write_cens(ndxout, ucf)
            close(ucf)
         endif
      else
         if (ndxout .gt. 0) write(*,*) 'c2d_shim: census mirror of',
     1        ndxout, ' records dropped at ncycle', ncycle,
     2        ': write_record would see no census'
         ndxout = 0
         if (warned .eq. 0 .and. mir) then
            write(*,*) 'c2d_shim: census of', ncs, ' records exceeds',
     1           ' ucens: kept on the GPU only (c2d_census_export)'
            warned = 1
         endif
      endif
      end
c
c
c     the SED binning from pspt's input deck (C2D_SHIM_SED_DECK: a file
c     with one answer a line; unset: every default of pspt)
      subroutine c2d_shim_sed_begin(ctx)
      use iso_c_binding
      use compton2d
      implicit none
      type(c_ptr) ctx
      character(kind=c_char, len=4096) :: deck
      character*512 fname, line
      integer st, u, ios, n, l
      integer(c_int) rc
      deck = ' '
      n = 0
      call get_environment_variable('C2D_SHIM_SED_DECK', fname,
     1     status=st)
      if (st .eq. 0 .and. len_trim(fname) .gt. 0) then
         open(newunit=u, file=trim(fname), status='old', iostat=ios)
         if (ios .ne. 0) then
            write(*,*) 'c2d_shim: cannot open ', trim(fname)
            call c2d_shim_fail(c_null_ptr, 'C2D_SHIM_SED_DECK', -1)
         endif
 10      read(u, '(a)', iostat=ios) line
         if (ios .eq. 0) then
            l = len_trim(line)
            if (n + l + 1 .lt. len(deck)) then
               if (l .gt. 0) deck(n+1:n+l) = line(1:l)
               deck(n+l+1:n+l+1) = char(10)
               n = n + l + 1
            endif
            goto 10
         endif
         close(u)
      endif
      deck(n+1:n+1) = c_null_char
      rc = c2d_obs_begin_pspt(ctx, deck)
      if (rc .ne. C2D_OK) call c2d_shim_fail(ctx, 'c2d_obs_begin_pspt',
     1     rc)
      end
c
c
c     file_sp (imcsurf2d_para.f:544-685) of one file into the next
c     spectrum slot
      subroutine c2d_shim_spectrum(fname, nsp)
      use iso_c_binding
      use c2d_shim_state, only: spec, sptab, shm_nslot
      implicit none
      include 'general.pa'
      include 'commonblock.f'
      character*30 fname
      integer nsp, i
      call file_sp(fname)
      nsp = nsp + 1
      if (nsp .gt. shm_nslot) stop 'c2d_shim: too many spectra'
      do 10 i = 1, nfmax
         sptab(i, 1, nsp) = E_file(i)
         sptab(i, 2, nsp) = a1(i)
         sptab(i, 3, nsp) = I_file(i)
         sptab(i, 4, nsp) = F_file(i)
         sptab(i, 5, nsp) = P_file(i)
 10   continue
      spec(nsp)%nfile = nfile
      spec(nsp)%E_file = c_loc(sptab(1, 1, nsp))
      spec(nsp)%a1 = c_loc(sptab(1, 2, nsp))
      spec(nsp)%I_file = c_loc(sptab(1, 3, nsp))
      spec(nsp)%F_file = c_loc(sptab(1, 4, nsp))
      spec(nsp)%P_file = c_loc(sptab(1, 5, nsp))
      end
c
c
c     volume and surface sources ran with the census in imcfield2d's
c     c2d_transport_step (one generation-0 launch per step)
      subroutine imcvol2d
      end
c
      subroutine imcsurf2d
      end
c
c     census balance (imcredist.f:5-133): each worker's census stays on
c     its GPU; the sources of the next step are re-sharded by lineage
      subroutine imcredist
      end
c
c
c     update (src/update2d.f:7-327) with FP_calc of every zone on the
c     master's GPU; the reference's own reductions and broadcasts
c     around it (cens_add_up, E_add_up, FP_end_bcast) are kept
      subroutine update
      use iso_c_binding
      use compton2d
      use c2d_shim_state, only: fctx, fready
      implicit none
      include 'mpif.h'
      include 'general.pa'
      include 'commonblock.f'
      target :: tea, tna, n_e, B_field, Eloss_sy, ec_old, turb_lev,
     1     vol, f_pair, ecens, n_field, f_nt, Pnt, Te_new, gmin, gmax,
     2     amxwl, p_nth, F_IC
      type(c2d_fp_config) :: fcfg
      type(c2d_fp_step_in) :: fpi
      type(c2d_fp_step_out) :: fpo
      integer(c_int) rc
      integer(c_int32_t) fpmode
      integer(c_int64_t) s1, sj, sk
      integer*8 c2d_shim_env

c
      lnL = 20.d0
c     edep, ecens, n_field of all workers -> master (update2d.f:1929)
      call cens_add_up
      hr_st_total = 0.d0
      hr_total = 0.d0
      E_tot_old = 0.d0
      E_tot_new = 0.d0
      dT_max = 0.d0
      if (myid .eq. master) then
         f_t_implicit = 2.d-1
         if (.not. fready) then

            call c2d_shim_init(fctx, 0, 1, 0, 65536_8, 65536_8,
     1           65536_8)
            fcfg%pair_switch = pair_switch
            fcfg%df_implicit = df_implicit
            fcfg%df_T = df_T
            fcfg%r_esc = r_esc
            fcfg%r_acc = r_acc
            fcfg%cf_sentinel = cf_sentinel
            fcfg%r_flare = r_flare
            fcfg%z_flare = z_flare
            fcfg%t_flare = t_flare
            fcfg%sigma_r = sigma_r
            fcfg%sigma_z = sigma_z
            fcfg%sigma_t = sigma_t
            fcfg%flare_amp = flare_amp
            fcfg%inj_switch = inj_switch
            fcfg%inj_dis = inj_dis
            fcfg%g2var_switch = g2var_switch
            fcfg%pick_sw = pick_sw
            fcfg%inj_g1 = inj_g1
            fcfg%inj_g2 = inj_g2
            fcfg%inj_p = inj_p
            fcfg%inj_t = inj_t
            fcfg%inj_L = inj_L
            fcfg%pick_rate = pick_rate
            fcfg%inj_gg = inj_gg
            fcfg%inj_sigma = inj_sigma
            fcfg%inj_v = inj_v
            fcfg%F_IC = c_loc(F_IC)
            fcfg%F_IC_s_i = 1
            fcfg%F_IC_s_ph = num_nt
            rc = c2d_fp_set_config(fctx, fcfg)
            if (rc .ne. C2D_OK) call c2d_shim_fail(fctx,
     1           'c2d_fp_set_config', rc)
c           FP arithmetic: C2D_FP_AUTO by default (exact while every
c           zone sits on the tea clamp, the block-parallel fast mode off
c           it, include/compton2d.h); C2D_SHIM_FP_MODE=0|1|2 picks exact,
c           fast or auto; C2D_SHIM_FP_FAST=1 is fast
            fpmode = int(c2d_shim_env('C2D_SHIM_FP_MODE',
     1           int(C2D_FP_AUTO, 8)), c_int32_t)
            if (c2d_shim_env('C2D_SHIM_FP_FAST', 0_8) .eq. 1)
     1           fpmode = C2D_FP_FAST
            rc = c2d_fp_set_mode(fctx, fpmode)
            if (rc .ne. C2D_OK) call c2d_shim_fail(fctx,
     1           'c2d_fp_set_mode', rc)
            fready = .true.
         endif
c        zone arrays in place: (j, k) of (jmax, kmax); the electron
c        spectra (jmax, kmax, num_nt); n_field (nphfield, jmax, kmax)
         s1 = 1
         sj = jmax
         sk = jmax*kmax
         fpi%ncycle = ncycle
         fpi%time = time
         fpi%dt = dt(1)
         fpi%tea = c2d_array2(c_loc(tea), s1, sj)
         fpi%tna = c2d_array2(c_loc(tna), s1, sj)
         fpi%n_e = c2d_array2(c_loc(n_e), s1, sj)
         fpi%B_field = c2d_array2(c_loc(B_field), s1, sj)
         fpi%Eloss_sy = c2d_array2(c_loc(Eloss_sy), s1, sj)
         fpi%ec_old = c2d_array2(c_loc(ec_old), s1, sj)
         fpi%turb_lev = c2d_array2(c_loc(turb_lev), s1, sj)
         fpi%vol = c2d_array2(c_loc(vol), s1, sj)
         fpi%f_pair = c2d_array2(c_loc(f_pair), s1, sj)
         fpi%ecens = c2d_array2(c_loc(ecens), s1, sj)
         fpi%n_field = c2d_array3(c_loc(n_field), s1,
     1        int(nphfield, c_int64_t), int(nphfield*jmax, c_int64_t))
         fpo%f_nt = c2d_marray3(c_loc(f_nt), sk, s1, sj)
         fpo%Pnt = c2d_marray3(c_loc(Pnt), sk, s1, sj)
         fpo%Te_new = c2d_marray2(c_loc(Te_new), s1, sj)
         fpo%tea = c2d_marray2(c_loc(tea), s1, sj)
         fpo%n_e = c2d_marray2(c_loc(n_e), s1, sj)
         fpo%gmin = c2d_marray2(c_loc(gmin), s1, sj)
         fpo%gmax = c2d_marray2(c_loc(gmax), s1, sj)
         fpo%amxwl = c2d_marray2(c_loc(amxwl), s1, sj)
         fpo%p_nth = c2d_marray2(c_loc(p_nth), s1, sj)
         fpo%zone_diag = c_null_ptr
c        FP_calc of every zone, its energy sums and dT_max, and the
c        tea update with its clamp (update2d.f:190-214, :266-276)
         rc = c2d_fp_step(fctx, fpi, fpo)
         if (rc .ne. C2D_OK) call c2d_shim_fail(fctx, 'c2d_fp_step',
     1        rc)
         E_tot_old = fpo%E_tot_old
         E_tot_new = fpo%E_tot_new
         hr_total = fpo%hr_total
         hr_st_total = fpo%hr_st_total
         dT_max = fpo%dT_max
      endif
c     energy and leakage sums, dT_max (update2d.f:1993-2078)
      call E_add_up
      if (myid .eq. master) then
c        time-step advice (update2d.f:233-243; dt(1) itself is kept)
         if (dT_max .lt. (0.2*df_T)) then
            dt_new = 3.d0*dt(1)
         else if (dT_max .lt. (.75*df_T)) then
            dt_new = 1.1d0*dt(1)
         else if (dT_max .gt. (5.*df_T)) then
            dt_new = 0.33d0*dt(1)
         else if (dT_max .gt. (1.25*df_T)) then
            dt_new = 7.5d-1*dt(1)
         else
            dt_new = dt(1)
         endif
         dt(2) = dt(1)
      endif
c     the new electron state to every rank (fp_mpi.f:1017-1084)
      call FP_end_bcast
      end
