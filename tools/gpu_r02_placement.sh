#!/usr/bin/env bash
# Placement-calibrated population stacks: the new GPU test, then bench.py A/B (plain allocation
# vs the fastest of 4 candidates per stack), alternating processes on one box.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "!! stop"; exit $rc; fi
}
step pytest_placement 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_population.py -k placement -p no:cacheprovider
for r in 1 2; do
  step bench_plain_$r 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic --placement-candidates 1
  step bench_placed_$r 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-traffic --placement-candidates 4
done
echo "== done"
