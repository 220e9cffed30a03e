#!/bin/bash
# Round-3 GPU session: each GPU step under its own time limit; a fault, abort or timeout ends the
# session (exit codes 124/134/137/139), an ordinary test failure does not.
set -u
OUT=${1:-gpurun_out/r3}
shift || true
mkdir -p "$OUT"
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "$OUT/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc $rc in $name: stopping"; exit $rc;; esac
  return 0
}
PYT="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
for s in "$@"; do eval "$s" || exit $?; done
