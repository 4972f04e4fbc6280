set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider > gpurun_out/pt_ab.log 2>&1; tail -1 gpurun_out/pt_ab.log
for r in 1 2; do
  CFA_LIB=$PWD/federated_amd/lib_prev/libcfa.so timeout -k 10 300 python tools/kernel_rooflines.py > gpurun_out/rl_prev_$r.log 2>&1 || exit 1
  timeout -k 10 300 python tools/kernel_rooflines.py > gpurun_out/rl_new_$r.log 2>&1 || exit 1
done
echo done
