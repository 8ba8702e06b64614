#!/bin/bash
# tools/gpu_queue.sh LOG CMD: queue a gpurun call: retries only while the pool has no free box/slot (exit 3: nothing ran)
log=$1; shift
for i in $(seq 1 12); do
  timeout 3000 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > $log 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "EXIT $rc" >> $log; exit 0; fi
  sleep 90
done
echo "EXIT 3 (gave up)" >> $log
