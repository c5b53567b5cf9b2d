#!/bin/bash
# gpurun with a wait-and-resubmit ONLY when the pool reports an infrastructure problem
# (status=transient / exit 3: no box, nothing ran).  A command that ran is never resubmitted.
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun "$@" > /tmp/gr_last.log 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|no box\|no slot" /tmp/gr_last.log || [ $rc -eq 3 ]; then
    echo "[gr] infrastructure not ready (attempt $attempt), waiting" >&2
    sleep 75
    continue
  fi
  cat /tmp/gr_last.log
  exit $rc
done
cat /tmp/gr_last.log
exit 3
