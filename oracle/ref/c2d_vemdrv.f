c     c2d_vemdrv.f -- TEST INFRASTRUCTURE ONLY (oracle/ref).
c
c     Calls the reference's own volume_em (src/volume2d.f:10-394) on cell
c     states read from a binary file, so the C restatement
c     (oracle/c2d_vem_oracle.c) and the GPU kernel can be pinned to it:
c       c2d_vemdrv IN.bin OUT.bin
c     IN : int32 ncell (<= 99); f64 gnt(200); per cell f64 T_keV, n_e, B,
c          l_min, amxwl, gmin, gmax, p_nth, f_pair, f_nt(200)
c     OUT: f64 E_ph(400); per cell f64 kappa_tot(400), eps_tot(400),
c          eps_th(400), Eloss_cy, Eloss_th  (the raw sums volume_em leaves
c          in COMMON, before imcgen2d's dt*vol / dt*zsurf scaling)
c
      program c2d_vemdrv
      implicit none
      include 'mpif.h'
      include 'general.pa'
      include 'commonblock.f'
      integer n, u, c, i
      double precision st(9)
      character*256 fin, fnout
c
      call getarg(1, fin)
      call getarg(2, fnout)
      u = 41
      pair_switch = 0
      open(unit=u, file=fin, access='stream', form='unformatted',
     1     status='old')
      open(unit=u+1, file=fnout, access='stream', form='unformatted',
     1     status='replace')
      read(u) n
      read(u) (gnt(i), i=1,num_nt)
      do c = 1, n
         read(u) (st(i), i=1,9)
         read(u) (f_nt(1,c,i), i=1,num_nt)
         amxwl(1,c) = st(5)
         gmin(1,c) = st(6)
         gmax(1,c) = st(7)
         p_nth(1,c) = st(8)
         f_pair(1,c) = st(9)
         call volume_em(1, c, st(1), st(2), st(3), st(4))
         if (c.eq.1) write(u+1) (E_ph(i), i=1,n_vol)
         write(u+1) (kappa_tot(i,1,c), i=1,n_vol)
         write(u+1) (eps_tot(i,1,c), i=1,n_vol)
         write(u+1) (eps_th(i,1,c), i=1,n_vol)
         write(u+1) Eloss_cy(1,c), Eloss_th(1,c)
      enddo
      close(u)
      close(u+1)
      end
