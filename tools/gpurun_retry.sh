#!/bin/bash
# retries a gpurun call only when it reports exit 3 (no box / transient
# infrastructure: nothing ran, nothing charged); any other result returns
LOG=$1; shift
for i in 1 2 3 4 5 6; do
  timeout 3000 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $LOG; then echo "EXIT $rc" >> $LOG; exit $rc; fi
  echo "transient try $i" >> /tmp/gpurun_transients.log
  sleep 60
done
echo "EXIT $rc (gave up)" >> $LOG
