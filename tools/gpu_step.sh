#!/bin/bash
# Shared helper for GPU job scripts: run one GPU step under its own time limit; a test
# failure (pytest rc 1) lets the script go on, anything else (timeout, abort, fault) ends it.
step() {
  local secs=$1 log=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"
  tail -3 "$log"
  if [ $rc -gt 1 ]; then
    echo "stopping after rc=$rc"
    exit $rc
  fi
}
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
