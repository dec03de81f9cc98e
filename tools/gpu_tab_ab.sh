set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
for tag in tab1024 tab512; do
  C2D_LIBRARY=$PWD/compton2d_amd/sweep/$tag/libcompton2d.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k fast -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/par_$tag.log 2>&1 || { echo "$tag parity FAILED"; tail -15 gpurun_out/ab/par_$tag.log; }
done
bash tools/gpu_ab.sh base tab1024 tab512
