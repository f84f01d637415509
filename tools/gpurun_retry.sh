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
  if echo "$out" | grep -q "status=transient\|backing off\|no free box\|slot(s) on this pod are busy"; then
    # honour the service's own back-off hint ("retry in Ns"): retrying earlier only extends it
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
    w=$(( ${w:-60} + 15 ))
    echo "[retry] attempt $attempt: infrastructure event, retrying in $w s"
    sleep $w
    continue
  fi
  exit $rc
done
exit 3
