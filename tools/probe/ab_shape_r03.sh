#!/usr/bin/env bash
# Same-box A/B of the mix kernel's size-dependent default launch shape (round 3): this library
# against the previous one (federated_amd/lib_prev, built from the commit before the change),
# alternating processes: the ring rounds of tools/probe/slice_shape.py at K = 2/4/8/16 (and K = 8
# on scattered rows, no reuse between consecutive mixes) and the
# drop-in host pipeline (tools/probe/pipeline_threshold.py --native-only), whose 128K-element
# chunks are now launched with four workgroups per CU.
set -u
TAG=${1:-ab}
mkdir -p gpurun_out
export SLICE_SIZES=500000,1000000,2000000,3125056,6250048,9000000 SLICE_BPC=1 SLICE_VEC=1 SLICE_CANDIDATES=2 SLICE_PASSES=5
for r in 1 2; do
  for lib in new prev; do
    if [ $lib = prev ]; then export CFA_LIB=$PWD/federated_amd/lib_prev/libcfa.so; else unset CFA_LIB; fi
    for h in 1 2 4 8; do
      SLICE_HALF=$h timeout -k 10 200 python tools/probe/slice_shape.py > gpurun_out/${TAG}_shape_${lib}_k$((2*h))_$r.jsonl 2>/dev/null || exit $?
    done
    SLICE_HALF=4 SLICE_PATTERN=scattered timeout -k 10 200 python tools/probe/slice_shape.py \
      > gpurun_out/${TAG}_shape_${lib}_k8_scattered_$r.jsonl 2>/dev/null || exit $?
    timeout -k 10 200 python tools/probe/pipeline_threshold.py --native-only > gpurun_out/${TAG}_pipe_${lib}_$r.log 2>&1 || exit $?
  done
done
echo done
