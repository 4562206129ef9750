#!/bin/bash
# retries a gpurun call only when it reports exit 3 / a transient status (no
# box, infrastructure: nothing ran, nothing charged); any other result returns.
# usage: gpurun_retry.sh LOG CMD [TRIES] [WAIT_S]
LOG=$1; CMD=$2; TRIES=${3:-12}; WAIT=${4:-180}
for i in $(seq 1 $TRIES); do
  timeout 3000 /usr/local/graft/bin/gpurun --timeout 1200 -- "$CMD" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $LOG; then echo "EXIT $rc" >> $LOG; exit $rc; fi
  w=$WAIT
  s=$(grep -oE "retry in [0-9]+s" $LOG | grep -oE "[0-9]+" | tail -1)
  [ -n "$s" ] && [ "$s" -gt "$w" ] && w=$((s + 15))
  echo "transient try $i, waiting ${w}s" >> /tmp/gpurun_transients.log
  sleep $w
done
echo "EXIT $rc (gave up)" >> $LOG
