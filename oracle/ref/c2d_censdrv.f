c     c2d_censdrv.f -- TEST INFRASTRUCTURE ONLY (oracle/ref).
c
c     Runs the reference's own census record writer/reader
c     (src/census2d.f:1-76, write_cens / read_cens) so that the engine's
c     census_io.py can be pinned to the reference's file format:
c       c2d_censdrv w IN.bin OUT.txt   - N, d(6,N), i(6,N) -> write_cens
c       c2d_censdrv r IN.txt N OUT.bin - read_cens of N records -> binary
c
      program c2d_censdrv
      implicit none
      include 'mpif.h'
      include 'general.pa'
      include 'commonblock.f'
      integer n, u, i
      character*8 mode
      character*256 fin, fnout, arg
c
      call getarg(1, mode)
      call getarg(2, fin)
      u = 41
      if (mode(1:1).eq.'w') then
         call getarg(3, fnout)
         open(unit=u, file=fin, access='stream', form='unformatted',
     1        status='old')
         read(u) n
         read(u) (dbufout(i), i=1,6*n)
         read(u) (ibufout(i), i=1,6*n)
         close(u)
         open(unit=u+1, file=fnout, status='replace')
         call write_cens(n, u+1)
         close(u+1)
      else
         call getarg(3, arg)
         read(arg, *) n
         call getarg(4, fnout)
         open(unit=u, file=fin, status='old')
         call read_cens(n, u)
         close(u)
         open(unit=u+1, file=fnout, access='stream',
     1        form='unformatted', status='replace')
         write(u+1) (dbufout(i), i=1,6*n)
         write(u+1) (ibufout(i), i=1,6*n)
         close(u+1)
      endif
      end
