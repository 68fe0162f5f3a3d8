#!/bin/bash
# usage: gpq.sh LOG TIMEOUT 'command' -- queue a gpurun call, retrying only while no GPU slot is free (exit 3)
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  timeout $((TO + 1500)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  echo "exit $rc" >> $LOG
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
