#!/usr/bin/env bash
# Round-2 GPU session: the host-path GPU tests (HostMixer, drop-in golden replays), then the
# drop-in latency breakdown with the zero-copy default and with it off.
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
step pytest_gpu 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -p no:cacheprovider
step dropin 200 python tools/dropin_latency.py
step dropin_off 200 python tools/dropin_latency.py --zero-copy-off
echo "== done"
