#!/bin/bash
# usage: gpu_try.sh OUT TIMEOUT CMD -- retries only while gpurun reports that no box ran the command
# (host side: only a call that no box ran is tried again; a call that ran is never repeated)
out=$1; lim=$2; cmd=$3
for a in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $lim -- "$cmd" > $out 2>&1
  if grep -q "status=transient" $out; then
    w=$(grep -o "retry in [0-9]*s" $out | grep -o "[0-9]*" | head -1); w=${w:-150}
    sleep $((w + 10)); continue
  fi
  break
done
echo "attempts=$a" >> $out
