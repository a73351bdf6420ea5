#!/bin/bash
# usage: gpr.sh LOG TIMEOUT CMD  -- retries gpurun only when no box could be prepared (rc 3)
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  echo "EXIT $rc (try $i)" >> $LOG
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 90
done
