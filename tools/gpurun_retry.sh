#!/bin/bash
# submit a gpurun call, re-submitting (at most 10 times) only when gpurun reports an infrastructure failure
# (status=transient: no box / backing off / box lost before the command ran; nothing charged), after the wait
# gpurun names ("retry in Ns"), else 150 s.   usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUTF=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUTF 2>&1
  grep -q "status=transient" $OUTF || exit 0
  W=$(grep -oE "retry in [0-9]+s" $OUTF | grep -oE "[0-9]+" | tail -1)
  sleep $(( ${W:-150} + 10 ))
done
