#!/usr/bin/env bash
# oracle/ref/build_ref.sh — TEST INFRASTRUCTURE ONLY.
#
# Builds the reference Fortran (bbw7561135/Compton2d, src/ snapshot) from
# its sources where they lie under /root/reference/src, with the image's
# own toolchain (AMD flang 22 + MPICH from /opt/conda),
# plus the serial driver oracle/ref/c2d_refdrv.f.  Outputs go ONLY to
# oracle/_ref/ (git-ignored).  Nothing here is needed on the GPU box: the
# tests there use the committed fixtures in tests/golden/.
#
# Object list = src/Makefile:39-68 minus the MPI main program compton2d.o.
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/../_ref"
SRC="${C2D_REFERENCE_SRC:-/root/reference/src}"
FC="${FC:-/opt/rocm/lib/llvm/bin/flang}"
MPI_INC="${MPI_INC:-/opt/conda/include}"
MPI_LIB="${MPI_LIB:-/opt/conda/lib}"
FFLAGS="${FFLAGS:--O2}"

if [ ! -d "$SRC" ]; then
  echo "build_ref: reference sources not found at $SRC" >&2
  exit 2
fi
mkdir -p "$OUT/obj" "$OUT/mod"

OBJS="reader setup2d xec2d imcgen2d volume2d gamma1_2d nontherm2d imcsurf2d_para
      planck2d pp2d imctrk2d census2d compb_2d comtot2d imcdate2d ref_matrix
      imcleak2d graphics2d imcvol2d_para imcfield2d imcredist icloss2d update2d
      rand fp_mpi surf_mpi vol_mpi write_record read_record"

pids=()
for f in $OBJS; do
  o="$OUT/obj/$f.o"
  if [ ! -f "$o" ] || [ "$SRC/$f.f" -nt "$o" ]; then
    "$FC" -c $FFLAGS -I"$MPI_INC" -I"$SRC" -module-dir "$OUT/mod" \
      "$SRC/$f.f" -o "$o" &
    pids+=($!)
    if [ ${#pids[@]} -ge 8 ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
  fi
done
for p in "${pids[@]}"; do wait "$p"; done

"$FC" -c $FFLAGS -I"$MPI_INC" -I"$SRC" -module-dir "$OUT/mod" \
  "$HERE/c2d_refdrv.f" -o "$OUT/obj/c2d_refdrv.o"

objs=""
for f in $OBJS; do objs="$objs $OUT/obj/$f.o"; done
"$FC" -o "$OUT/c2d_refdrv" "$OUT/obj/c2d_refdrv.o" $objs \
  -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi
# the same driver over the 2012-11 snapshot's tracker (c2d_config.trk_variant =
# C2D_TRK_2012_11): src_20121113/imctrk2d.f and its
# imcfield2d.f (the census |wmu| clamp) in place of src/'s; every other
# object, and the COMMON blocks (commonblock.f, general.pa: identical in both
# snapshots), are src/'s
SRC12="${C2D_REFERENCE_SRC12:-$(dirname "$SRC")/src_20121113}"
if [ -d "$SRC12" ]; then
  mkdir -p "$OUT/obj/v2012"
  for f in imctrk2d imcfield2d; do
    "$FC" -c $FFLAGS -I"$MPI_INC" -I"$SRC" -module-dir "$OUT/mod" "$SRC12/$f.f" -o "$OUT/obj/v2012/$f.o"
  done
  objs12=""
  for f in $OBJS; do
    case $f in imctrk2d|imcfield2d) objs12="$objs12 $OUT/obj/v2012/$f.o" ;; *) objs12="$objs12 $OUT/obj/$f.o" ;; esac
  done
  "$FC" -o "$OUT/c2d_refdrv_2012" "$OUT/obj/c2d_refdrv.o" $objs12 \
    -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi
  echo "build_ref: $OUT/c2d_refdrv_2012"
fi
"$FC" -c $FFLAGS -I"$MPI_INC" -I"$SRC" -module-dir "$OUT/mod" \
  "$HERE/c2d_censdrv.f" -o "$OUT/obj/c2d_censdrv.o"
"$FC" -o "$OUT/c2d_censdrv" "$OUT/obj/c2d_censdrv.o" "$OUT/obj/census2d.o" \
  -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi
"$FC" -c $FFLAGS -I"$MPI_INC" -I"$SRC" -module-dir "$OUT/mod" \
  "$HERE/c2d_vemdrv.f" -o "$OUT/obj/c2d_vemdrv.o"
"$FC" -o "$OUT/c2d_vemdrv" "$OUT/obj/c2d_vemdrv.o" "$OUT/obj/volume2d.o" \
  -L"$MPI_LIB" -Wl,-rpath,"$MPI_LIB" -lmpifort -lmpi
echo "build_ref: $OUT/c2d_refdrv $OUT/c2d_censdrv $OUT/c2d_vemdrv"

# The post-processing tools (postprocessing/pspt.c, plcm.c: K&R C reading an
# input deck on stdin) for the observer-frame binning fixtures.
PP="${C2D_REFERENCE_PP:-$(dirname "$SRC")/postprocessing}"
for t in pspt plcm; do
  gcc -O2 -std=gnu89 -w "$PP/$t.c" -o "$OUT/$t" -lm 2>/dev/null
done
echo "build_ref: $OUT/pspt $OUT/plcm"
