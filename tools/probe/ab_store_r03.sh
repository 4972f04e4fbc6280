#!/usr/bin/env bash
# Same-box A/B of the streaming mix's store policy (round 3): nt buffer store (this library)
# against the sc1 write-through store (federated_amd/lib_prev, built from the commit before),
# alternating processes: the default bench line (no baselines), every streaming entry point's
# roofline (tools/kernel_rooflines.py), and ring rounds at the N > 1 slice sizes
# (tools/probe/slice_shape.py, K = 8). Output: gpurun_out/${TAG}_*.
set -u
TAG=${1:-abst}
mkdir -p gpurun_out
export SLICE_SIZES=1000000,3125056,6250048,12500000 SLICE_BPC=1 SLICE_VEC=1 SLICE_CANDIDATES=2 SLICE_PASSES=5 SLICE_HALF=4
for r in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export CFA_LIB=$PWD/federated_amd/lib_prev/libcfa.so; else unset CFA_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-live-traffic --no-e2e \
      > gpurun_out/${TAG}_bench_${lib}_$r.json 2>/dev/null || exit $?
    timeout -k 10 300 python tools/kernel_rooflines.py > gpurun_out/${TAG}_rooflines_${lib}_$r.jsonl 2>/dev/null || exit $?
    timeout -k 10 200 python tools/probe/slice_shape.py > gpurun_out/${TAG}_slice_${lib}_$r.jsonl 2>/dev/null || exit $?
  done
done
echo done
