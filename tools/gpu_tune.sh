#!/usr/bin/env bash
# GPU session: GPU tests, launch-shape sweep, PMC traffic passes on the bench command.
set -u
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "!! stop"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step tune 600 python tools/tune_mix.py
BENCH="bench.py --steps 5 --warmup 1 --no-cpu-baseline"
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_$TAG" -o fetch --output-format csv -- python3 $BENCH
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_$TAG" -o write --output-format csv -- python3 $BENCH
ls -R "$OUT/pmc_$TAG" | head -20
echo "== done"
