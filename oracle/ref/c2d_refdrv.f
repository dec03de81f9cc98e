c     c2d_refdrv.f -- TEST INFRASTRUCTURE ONLY (oracle/ref).
c
c     Serial driver for the REFERENCE Fortran (built from
c     /root/reference/src by oracle/ref/build_ref.sh into
c     oracle/_ref/).  It runs, in one process, the same per-step
c     sequence a master + worker pair runs under MPI
c     (src/xec2d.f:41-110 master, :141-193 worker):
c        imcgen2d (master part)              src/imcgen2d.f:1-553
c        worker tally reset                  src/imcgen2d.f:557-601
c        field_calc (census)                 src/imcfield2d.f:57
c        vol_calc for every zone             src/imcvol2d_para.f:90
c        z_surf_calc / r_surf_calc           src/imcsurf2d_para.f:228,353
c     emulating the worker's lagged kappa_tot (hazard H3: workers
c     receive kappa_tot only in z_surf_bcast, src/surf_mpi.f:97) and
c     restoring the master's seeds after field_calc overwrites them
c     (src/imcfield2d.f:115; volume jobs carry the master's seed,
c     src/vol_mpi.f:107).  After every step it dumps the transport
c     inputs and the worker tallies in full precision (stream files)
c     so tests can compare the C oracle against the reference itself.
c
c     usage: c2d_refdrv NSTEPS KLAG [NFORCEU]   (run inside a prepared
c            case directory holding input/input.dat + input_JJ_KK.dat)
c
c     NFORCEU > 0 gives every upper ring with a blackbody temperature
c     (tbbu > 0) NFORCEU packets of weight erinu/NFORCEU after imcgen2d.
c     In src/ such a ring gets its energy erinu (imcgen2d.f:155-163) but
c     no packets (nsurfu is set only for tbbu < 0, imcgen2d.f:436-437),
c     so r_surf_calc's planck branch (imcsurf2d_para.f:399-401,
c     planck2d.f) is unreachable from input.dat; this exercises the
c     reference's own r_surf_calc + planck on such packets.
c
      program c2d_refdrv
      implicit none
      include 'mpif.h'
      include 'general.pa'
      include 'commonblock.f'
c
      integer nsteps, klag, n, j, k, zone, js, ks, u, nforceu
      integer iargc
      integer seeds_sv(jmax,kmax)
      double precision kap_cur(n_vol,jmax,kmax)
      double precision kap_prev(n_vol,jmax,kmax)
      double precision t_average, tw0, tw1, tw2, tw3
      character*32 arg
      character*40 fn
      save kap_cur, kap_prev, seeds_sv
c
      call MPI_INIT(ierr)
      call MPI_COMM_RANK(MPI_COMM_WORLD, myid, ierr)
      call MPI_COMM_SIZE(MPI_COMM_WORLD, numprocs, ierr)
      master = 0
      call getarg(1, arg)
      read(arg, *) nsteps
      call getarg(2, arg)
      read(arg, *) klag
      nforceu = 0
      if (iargc().ge.3) then
         call getarg(3, arg)
         read(arg, *) nforceu
      endif
c
      open(unit=4, file='log.txt')
      call reader
      call setup
c
      nunit_evt = 1001
      kap_prev = 0.d0
      ndxout = 0
      u = 31
c
c     static configuration (after setup)
      open(unit=u, file='config.bin', access='stream',
     1     form='unformatted', status='replace')
      write(u) nz, nr, nphtotal, nph_lc, nmu
      write(u) split1, split2, split3, spl3_trg
      write(u) spec_switch, cr_sent, pair_switch, rand_switch
      write(u) rseed, T_const, ntime
      write(u) rmin, zmin
      write(u) (z(j), j=1,nz)
      write(u) (r(k), k=1,nr)
      write(u) (E_field(j), j=1,nphfield)
      write(u) (gnt(j), j=1,num_nt)
      write(u) (hu(j), j=1,nphtotal+1)
      write(u) (Elcmin(j), j=1,nph_lc)
      write(u) (Elcmax(j), j=1,nph_lc)
      write(u) (mu(j), j=1,nmu)
      close(u)
c     IC loss kernel of setup (icloss2d.f:1-64), input of FP_calc
      open(unit=u, file='fic.bin', access='stream',
     1     form='unformatted', status='replace')
      write(u) ((F_IC(j,k), j=1,num_nt), k=1,nphfield)
      close(u)
c
      do 500 n = 0, nsteps-1
c        H6: the master's n_ph never receives the workers' tallies (no
c        reduce of it, src/update2d.f:1958-1973) and stays 0, so pairprod
c        (dn_pp) and kgg_calc (k_gg) see no photons under MPI
         if (pair_switch.eq.1) n_ph = 0.d0
c        master part of the step
         call imcgen2d
c        worker-side resets (src/imcgen2d.f:559-601)
         do 10 j = 1, nz
            erlko(j) = 0.d0
            erlki(j) = 0.d0
 10      continue
         do 12 k = 1, nr
            erlku(k) = 0.d0
            erlkl(k) = 0.d0
 12      continue
         do 14 j = 1, num_nt
            nelectron(j) = 0
 14      continue
c        time-window index (src/imcsurf2d_para.f:55-64)
         if (ncycle.eq.0) then
            ti = 1
         else
            t_average = time + 5.d-1*dt(1)
            do 20 ti = 1, ntime
               if (t1(ti).gt.t_average) goto 21
 20         continue
 21         continue
         endif
         if (nforceu.gt.0) then
            do 22 k = 1, nr
               if (tbbu(k,ti).gt.0.d0) then
                  nsurfu(k) = nforceu
                  ewsurfu(k) = erinu(k)/dble(nforceu)
               endif
 22         continue
         endif
c        transport inputs of this step
         write(fn, '(a,i3.3,a)') 'in_', n, '.bin'
         open(unit=u, file=fn, access='stream',
     1        form='unformatted', status='replace')
         write(u) ncycle, ti
         write(u) time, dt(1)
         write(u) (E_ph(j), j=1,n_vol)
         write(u) (((kappa_tot(j,js,ks), j=1,n_vol), ks=1,nr),
     1             js=1,nz)
         write(u) (((eps_tot(j,js,ks), j=1,n_vol), ks=1,nr), js=1,nz)
         write(u) (((eps_th(j,js,ks), j=1,n_vol), ks=1,nr), js=1,nz)
         write(u) (((f_nt(js,ks,j), j=1,num_nt), ks=1,nr), js=1,nz)
         write(u) (((Pnt(js,ks,j), j=1,num_nt), ks=1,nr), js=1,nz)
         write(u) ((n_e(js,ks), ks=1,nr), js=1,nz)
         write(u) ((Eloss_th(js,ks), ks=1,nr), js=1,nz)
         write(u) ((Eloss_tot(js,ks), ks=1,nr), js=1,nz)
         write(u) ((zsurf(js,ks), ks=1,nr), js=1,nz)
         write(u) ((ewsv(js,ks), ks=1,nr), js=1,nz)
         write(u) ((nsv(js,ks), ks=1,nr), js=1,nz)
         write(u) (nsurfi(j), j=1,nz), (nsurfo(j), j=1,nz)
         write(u) (ewsurfi(j), j=1,nz), (ewsurfo(j), j=1,nz)
         write(u) (nsurfu(k), k=1,nr), (nsurfl(k), k=1,nr)
         write(u) (ewsurfu(k), k=1,nr), (ewsurfl(k), k=1,nr)
         write(u) (tbbi(j,ti), j=1,nz), (tbbo(j,ti), j=1,nz)
         write(u) (tbbu(k,ti), k=1,nr), (tbbl(k,ti), k=1,nr)
         write(u) rseed
         close(u)
c
c        per-step event file (the reference appends to p###_evb.dat)
         write(fn, '(a,i3.3,a)') 'ev_', n, '.dat'
         open(unit=nunit_evt, file=fn, status='replace')
c        census transport with the worker's previous kappa_tot (H3)
         seeds_sv = seeds
         kap_cur = kappa_tot
         if (klag.eq.1) kappa_tot = kap_prev
         tw0 = MPI_WTIME()
         call field_calc
         tw1 = MPI_WTIME()
         seeds = seeds_sv
         do 30 zone = 1, nz*nr
            call vol_calc(zone)
 30      continue
         tw2 = MPI_WTIME()
         kappa_tot = kap_cur
         do 40 js = 1, nz
            call z_surf_calc(js)
 40      continue
         do 50 ks = 1, nr
            call r_surf_calc(ks)
 50      continue
         tw3 = MPI_WTIME()
         kap_prev = kap_cur
c        wall time of this step's transport legs (census, volume,
c        surfaces; tools/fortran_vs_port.py)
         open(unit=u, file='transport_times.txt', access='append')
         write(u, '(i6,3(1x,e16.9))') n, tw1 - tw0, tw2 - tw1, tw3 - tw2
         close(u)
c
c        worker tallies of this step
         write(fn, '(a,i3.3,a)') 'out_', n, '.bin'
         open(unit=u, file=fn, access='stream',
     1        form='unformatted', status='replace')
         write(u) ((edep(js,ks), ks=1,nr), js=1,nz)
         write(u) ((prdep(js,ks), ks=1,nr), js=1,nz)
         write(u) ((ecens(js,ks), ks=1,nr), js=1,nz)
         write(u) ((npcen(js,ks), ks=1,nr), js=1,nz)
         write(u) (((n_field(j,js,ks), j=1,nphfield), ks=1,nr),
     1             js=1,nz)
         write(u) (E_IC(j), j=1,num_nt)
         write(u) (nelectron(j), j=1,num_nt)
         write(u) ((fout(js,ks), ks=1,nphomax), js=1,nmu)
         write(u) ((edout(js,ks), ks=1,nphlcmax), js=1,nmu)
         write(u) (erlki(j), j=1,nz), (erlko(j), j=1,nz)
         write(u) (erlku(k), k=1,nr), (erlkl(k), k=1,nr)
         write(u) (Ed_in(k), k=1,nr)
         write(u) ndxout
         write(u) (dbufout(j), j=1,6*ndxout)
         write(u) (ibufout(j), j=1,6*ndxout)
         write(u) nfile
         write(u) (E_file(j), j=1,nfmax), (a1(j), j=1,nfmax)
         write(u) (I_file(j), j=1,nfmax), (F_file(j), j=1,nfmax)
         write(u) (P_file(j), j=1,nfmax)
         close(u)
         close(nunit_evt)
c
c        Fokker-Planck update (src/xec2d.f:86-87 -> update2d.f:7-327):
c        the master/worker job exchange of update collapses to calling
c        FP_calc for every zone in this one process.
         if ((T_const.eq.0).and.(ncycle.gt.0)) then
            write(fn, '(a,i3.3,a)') 'fpin_', n, '.bin'
            open(unit=u, file=fn, access='stream',
     1           form='unformatted', status='replace')
            write(u) ncycle
            write(u) time, dt(1)
            write(u) ((tea(js,ks), ks=1,nr), js=1,nz)
            write(u) ((tna(js,ks), ks=1,nr), js=1,nz)
            write(u) ((n_e(js,ks), ks=1,nr), js=1,nz)
            write(u) ((B_field(js,ks), ks=1,nr), js=1,nz)
            write(u) ((Eloss_sy(js,ks), ks=1,nr), js=1,nz)
            write(u) ((ecens(js,ks), ks=1,nr), js=1,nz)
            write(u) ((ec_old(js,ks), ks=1,nr), js=1,nz)
            write(u) ((turb_lev(js,ks), ks=1,nr), js=1,nz)
            write(u) ((vol(js,ks), ks=1,nr), js=1,nz)
            write(u) ((f_pair(js,ks), ks=1,nr), js=1,nz)
            write(u) ((gmin(js,ks), ks=1,nr), js=1,nz)
            write(u) ((gmax(js,ks), ks=1,nr), js=1,nz)
            write(u) ((amxwl(js,ks), ks=1,nr), js=1,nz)
            write(u) ((p_nth(js,ks), ks=1,nr), js=1,nz)
            write(u) (((f_nt(js,ks,j), j=1,num_nt), ks=1,nr), js=1,nz)
            write(u) (((Pnt(js,ks,j), j=1,num_nt), ks=1,nr), js=1,nz)
            write(u) (((n_field(j,js,ks), j=1,nphfield), ks=1,nr),
     1                js=1,nz)
            close(u)
c           update, master part (update2d.f:142-151, :174-177), the
c           dT_max of photon_fill (:1912) and FP_bcast (:185)
            lnL = 20.d0
            dT_max = 0.d0
            if (ncycle.le.1) dT_max = df_T
            hr_st_total = 0.d0
            hr_total = 0.d0
            E_tot_old = 0.d0
            E_tot_new = 0.d0
            do 62 js = 1, nz
               do 61 ks = 1, nr
                  Te_new(js,ks) = tea(js,ks)
 61            continue
 62         continue
            do 70 zone = 1, nz*nr
               call FP_calc(zone)
 70         continue
c           store results for the next step (update2d.f:266-276)
            do 82 js = 1, nz
               do 81 ks = 1, nr
                  if (tna(js,ks).gt.1.) then
                     tea(js,ks) = Te_new(js,ks)
                     tea(js,ks) = dmin1(1.d3, tea(js,ks))
                     tea(js,ks) = dmax1(5.d0, tea(js,ks))
                  endif
 81            continue
 82         continue
            write(fn, '(a,i3.3,a)') 'fpout_', n, '.bin'
            open(unit=u, file=fn, access='stream',
     1           form='unformatted', status='replace')
            write(u) E_tot_old, E_tot_new, hr_total, hr_st_total, dT_max
            write(u) ((Te_new(js,ks), ks=1,nr), js=1,nz)
            write(u) ((tea(js,ks), ks=1,nr), js=1,nz)
            write(u) ((n_e(js,ks), ks=1,nr), js=1,nz)
            write(u) ((gmin(js,ks), ks=1,nr), js=1,nz)
            write(u) ((gmax(js,ks), ks=1,nr), js=1,nz)
            write(u) ((amxwl(js,ks), ks=1,nr), js=1,nz)
            write(u) ((p_nth(js,ks), ks=1,nr), js=1,nz)
            write(u) (((f_nt(js,ks,j), j=1,num_nt), ks=1,nr), js=1,nz)
            write(u) (((Pnt(js,ks,j), j=1,num_nt), ks=1,nr), js=1,nz)
            close(u)
         endif
c
c        advance in time (src/xec2d.f:100-107)
         dt(2) = dt(1)
         if (ncycle.gt.0) then
            time = time + dt(1)
         endif
         ncycle = ncycle + 1
 500  continue
      close(4)
      call MPI_FINALIZE(ierr)
      end
