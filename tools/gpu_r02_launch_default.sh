#!/usr/bin/env bash
# The mix kernel's new default shape (1 workgroup per CU, per-fan-in float4 per lane) against the
# round-1 default (CFA_BLOCKS_PER_CU=2: 2 workgroups per CU, auto vec), alternating processes; the
# whole GPU suite first; then the launch sweep at K = 4 and 8 on this box.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider > $OUT/ld_pytest.log 2>&1 || { tail -20 $OUT/ld_pytest.log; exit 1; }
tail -1 $OUT/ld_pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic > $OUT/ld_new_$r.log 2>&1 || exit 1
  CFA_BLOCKS_PER_CU=2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic > $OUT/ld_old_$r.log 2>&1 || exit 1
  echo "$r: $(grep -h '^{' $OUT/ld_new_$r.log | cut -c90-120) | $(grep -h '^{' $OUT/ld_old_$r.log | cut -c90-120)"
done
for h in 2 4; do TUNE_HALF=$h timeout -k 10 200 python tools/probe/tune_placed.py > $OUT/tune_placed_c_h$h.jsonl 2>/dev/null || exit 1; done
echo done
