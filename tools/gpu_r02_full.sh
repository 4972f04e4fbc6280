#!/usr/bin/env bash
# Round-2 GPU session: the whole GPU test suite, smoke, and the default bench line (N = 1).
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "!! stop"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 400 python bench.py --steps 20 --warmup 3
echo "== done"
