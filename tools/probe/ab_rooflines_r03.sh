set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_ps_golden.py tests/test_gpu_payload.py -m gpu -p no:cacheprovider > gpurun_out/${TAG:-r03c}_pt.log 2>&1; rc=$?; tail -1 gpurun_out/${TAG:-r03c}_pt.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  CFA_LIB=$PWD/federated_amd/lib_prev/libcfa.so timeout -k 10 300 python tools/kernel_rooflines.py > gpurun_out/${TAG:-r03c}_rl_prev_$r.log 2>&1 || exit 1
  timeout -k 10 300 python tools/kernel_rooflines.py > gpurun_out/${TAG:-r03c}_rl_new_$r.log 2>&1 || exit 1
done
echo done
