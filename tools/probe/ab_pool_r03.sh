#!/usr/bin/env bash
# Same-box A/B of the drop-in host pipeline (cfa_host_mix_f32) with the copy pool's round-3
# claim/close protocol (run() returns once the jobs are done and no helper is inside the job list,
# without waiting for idle helpers to check in) against the previous pool (federated_amd/lib_prev),
# alternating processes.
set -u
TAG=${1:-pool}
mkdir -p gpurun_out
for r in 1 2 3 4 5 6; do
  order="new prev"; [ $((r % 2)) -eq 0 ] && order="prev new"  # alternate which library goes first
  for lib in $order; do
    if [ $lib = prev ]; then export CFA_LIB=$PWD/federated_amd/lib_prev/libcfa.so; else unset CFA_LIB; fi
    timeout -k 10 200 python tools/probe/pipeline_threshold.py --native-only > gpurun_out/${TAG}_pipe_${lib}_$r.log 2>&1 || exit $?
  done
done
echo done
