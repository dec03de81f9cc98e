#!/usr/bin/env bash
# oracle/ref/build_shim.sh — TEST INFRASTRUCTURE ONLY (this container).
#
# Links the reference's OWN Fortran host — its main program
# (src/compton2d.f), reader, setup, xec, imcgen2d, graphics, write_record,
# the MPI plumbing ... every object of src/Makefile — with the drop-in
# shim examples/c2d_shim.f, which defines the five per-step entry points
# imcfield2d, imcvol2d, imcsurf2d, imcredist and update over the engine's
# C-ABI (libcompton2d.so).  The reference objects keep their own
# definitions of those five names, weakened with objcopy so the shim's
# strong ones win at link time; nothing else in them changes.
#
# Objects come from oracle/ref/build_ref.sh (oracle/_ref/obj); outputs go
# ONLY to oracle/_ref/ (git-ignored, never shipped to the GPU box):
#   shim/compton2d_gpu      the reference host + shim over libcompton2d.so
#   shim/compton2d_standin  the same, linked against oracle/c2d_standin.c
#                           (the C-ABI over the C oracle in its reference
#                           mode: runs here, without a GPU)
#   shim/compton2d_ref      the unmodified reference (its main + every
#                           object), for the comparison
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
REF="$HERE/../_ref"
OUT="$REF/shim"
SRC="${C2D_REFERENCE_SRC:-/root/reference/src}"
FC="${FC:-/opt/rocm/lib/llvm/bin/flang}"
MPI_INC="${MPI_INC:-/opt/conda/include}"
MPI_LIB="${MPI_LIB:-/opt/conda/lib}"
FFLAGS="${FFLAGS:--O2}"
if [ ! -f "$REF/obj/xec2d.o" ]; then bash "$HERE/build_ref.sh" > /dev/null; fi
mkdir -p "$OUT/mod"

OBJS="reader setup2d xec2d imcgen2d volume2d gamma1_2d nontherm2d imcsurf2d_para
      planck2d pp2d imctrk2d census2d compb_2d comtot2d imcdate2d ref_matrix
      imcleak2d graphics2d imcvol2d_para imcfield2d imcredist icloss2d update2d
      rand fp_mpi surf_mpi vol_mpi write_record read_record"
declare -A WEAK=([imcfield2d]=imcfield2d_ [imcvol2d_para]=imcvol2d_
                 [imcsurf2d_para]=imcsurf2d_ [imcredist]=imcredist_ [update2d]=update_)
objs=""
for f in $OBJS; do
  if [ -n "${WEAK[$f]:-}" ]; then
    objcopy --weaken-symbol="${WEAK[$f]}" "$REF/obj/$f.o" "$OUT/$f.weak.o"
    objs="$objs $OUT/$f.weak.o"
  else
    objs="$objs $REF/obj/$f.o"
  fi
done
# the reference's main program (src/compton2d.f), unchanged
"$FC" -c $FFLAGS -I"$MPI_INC" -I"$SRC" -module-dir "$OUT/mod" "$SRC/compton2d.f" -o "$OUT/compton2d.o"
"$FC" -c $FFLAGS -module-dir "$OUT/mod" "$REPO/include/compton2d_mod.f90" -o "$OUT/compton2d_mod.o"
"$FC" -c $FFLAGS -I"$MPI_INC" -I"$SRC" -I"$OUT/mod" -module-dir "$OUT/mod" \
  "$REPO/examples/c2d_shim.f" -o "$OUT/c2d_shim.o"
LIB="$REPO/compton2d_amd"
"$FC" -o "$OUT/compton2d_gpu" "$OUT/c2d_shim.o" "$OUT/compton2d_mod.o" "$OUT/compton2d.o" $objs \
  -L"$LIB" -lcompton2d -Wl,-rpath,"$LIB" -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi
echo "build_shim: $OUT/compton2d_gpu"

# the stand-in library: the C-ABI symbols the shim calls, over the oracle
STANDIN="$REF/standin"
mkdir -p "$STANDIN"
gcc -O2 -fPIC -ffp-contract=off -fno-fast-math -fno-math-errno -std=gnu11 -w -shared \
  -o "$STANDIN/libcompton2d.so" "$REPO/oracle/c2d_standin.c" "$REPO/oracle/c2d_oracle.c" \
  "$REPO/oracle/c2d_fp_oracle.c" "$REPO/oracle/c2d_obs_oracle.c" -lm
"$FC" -o "$OUT/compton2d_standin" "$OUT/c2d_shim.o" "$OUT/compton2d_mod.o" "$OUT/compton2d.o" $objs \
  -L"$STANDIN" -lcompton2d -Wl,-rpath,"$STANDIN" -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi
echo "build_shim: $OUT/compton2d_standin"
# the unmodified reference
refobjs=""
for f in $OBJS; do refobjs="$refobjs $REF/obj/$f.o"; done
"$FC" -o "$OUT/compton2d_ref" "$OUT/compton2d.o" $refobjs \
  -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi
echo "build_shim: $OUT/compton2d_ref"
