#!/usr/bin/env bash
# A/B of the completion word on config 3's CFA-GE call pieces (tools/probe/c3_calls.py),
# alternating processes on one box. Output: gpurun_out/ab_signal_c3.jsonl
set -u
OUT=gpurun_out; mkdir -p "$OUT"; cd "${GRAFT_REPO_ROOT:-.}"
for i in 1 2 3; do
  timeout -k 10 120 python tools/probe/c3_calls.py >> "$OUT/ab_signal_c3.jsonl" || exit $?
  timeout -k 10 120 python tools/probe/c3_calls.py --signal-off >> "$OUT/ab_signal_c3.jsonl" || exit $?
done
