#!/usr/bin/env bash
# Round-2 session-3 re-entry check on a fresh box: whole GPU suite, smoke, the default bench line.
set -u
OUT=gpurun_out; mkdir -p $OUT; cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "!! stop"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 500 python bench.py --steps 20 --warmup 3
echo "== done"
