#!/bin/bash
# Re-submit a gpurun call while the GPU service reports an infrastructure event (no box, box
# taken away / unresponsive while being prepared: status=transient, nothing ran, nothing
# charged).  Any run that actually executed — pass or fail — is returned as is, never retried.
#   tools/gpurun_retry.sh <timeout_s> '<command>'
T=$1; shift
for attempt in $(seq 1 ${RETRIES:-10}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out" | grep -v "every call sends" | tail -12
  if echo "$out" | grep -q "status=transient\|backing off\|no free box"; then
    echo "[retry] attempt $attempt: infrastructure event, retrying in 60 s"
    sleep 60
    continue
  fi
  exit $rc
done
exit 3
