#!/bin/bash
# GPU box: run one step under its own time limit with a heartbeat file (long oracle comparisons
# print nothing for minutes), output to gpurun_out/<tag>/<name>.log; crash-class exits stop.
#   bash tools/gpu_run.sh TAG NAME SECONDS CMD...
set -u
TAG=$1 NAME=$2 SECS=$3
shift 3
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
(while true; do date +%T > $O/heartbeat.txt; sleep 20; done) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
echo "== $NAME ($(date +%T))"
timeout -k 10 "$SECS" "$@" > "$O/$NAME.log" 2>&1
rc=$?
echo "== $NAME rc=$rc"
tail -n 15 "$O/$NAME.log"
exit $rc
