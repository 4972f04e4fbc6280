#!/usr/bin/env bash
# Batch-split sweep of the CFA-GE gradient launch (GPU box): rocprofv3 kernel stats of the config-3
# population rounds at each forced split (CFA_GRAD_SPLIT); results under gpurun_out/split_<sp>/.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for sp in 1 2 3 4 6 8 12 24; do
  CFA_GRAD_SPLIT=$sp timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/split_$sp -o s --output-format csv -- python3 tools/bench_configs.py c3 > gpurun_out/split_$sp.log 2>&1 || exit 1
  echo "sp=$sp done"
done
