#!/bin/bash
# Run one GPU step under its own time limit; classify the exit status.
# usage: tools/box_step.sh <seconds> <logfile> <cmd...>
# exit 0: ok or ordinary failure (logged); exit 99: fault-class status -> caller must stop.
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[box_step] rc=$rc cmd=$*" >> "$log"
case $rc in
  0|1|2|5) exit 0 ;;     # success / test failures / usage / no tests
  *) echo "[box_step] FAULT-CLASS rc=$rc for: $*"; exit 99 ;;
esac
