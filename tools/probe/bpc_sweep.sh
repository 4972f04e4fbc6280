#!/usr/bin/env bash
# Workgroups per CU for every streaming entry (CFA_BLOCKS_PER_CU overrides the library default
# of 2 for all of them), two interleaved rounds of tools/kernel_rooflines.py per setting.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for b in 2 3 4; do
    CFA_BLOCKS_PER_CU=$b timeout -k 10 300 python tools/kernel_rooflines.py > gpurun_out/bpc${b}_$r.log 2>&1 || exit 1
  done
done
echo done
