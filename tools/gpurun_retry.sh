#!/bin/bash
# submit a gpurun call, re-submitting (at most 8 times, 150 s apart) only when gpurun reports an infrastructure
# failure (no box / backing off / box lost before the command ran: status=transient, nothing charged)
# usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUTF=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUTF 2>&1
  grep -q "status=transient" $OUTF || exit 0
  sleep 150
done
