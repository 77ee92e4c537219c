#!/bin/bash
# (host side) retry a gpurun call only while the pool has no free box (rc 3 / transient); any other outcome ends it
for i in $(seq 1 30); do
  timeout 3300 /usr/local/graft/bin/gpurun --timeout ${GPU_T:-1200} -- "$1"
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q '"status": "transient"' /root/repo/gpurun_out/.last_call.json 2>/dev/null; then exit $rc; fi
  sleep 90
done
exit 3
