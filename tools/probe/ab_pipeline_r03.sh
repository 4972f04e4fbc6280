#!/usr/bin/env bash
# Same-box A/B of the drop-in host pipeline (cfa_host_mix_f32): round 3's library against round 2's
# (federated_amd/lib_prev, built from commit cbfea0c), alternating processes. Round 2's pool can
# deadlock (the bug round 3 fixed), so every run has its own time limit.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python tools/probe/pipeline_threshold.py --native-only > gpurun_out/r03h_pipe_new_$r.log 2>&1 || exit $?
  CFA_LIB=$PWD/federated_amd/lib_prev/libcfa.so timeout -k 10 200 python tools/probe/pipeline_threshold.py --native-only > gpurun_out/r03h_pipe_prev_$r.log 2>&1 || exit $?
done
echo done
