set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for v in fpprof: fpsec:--sections fpmemo:--memo; do
  t=${v%%:*}; a=${v#*:}
  C2D_LIBRARY=$PWD/compton2d_amd/sweep/$t/libcompton2d.so timeout -k 10 200 python tools/fp_prof.py --nz 30 --nr 9 --vary --mode fast $a > $O/$t.out 2> $O/$t.err || exit 1
  cat $O/$t.out
done
