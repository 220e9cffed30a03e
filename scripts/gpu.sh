#!/bin/bash
# build in-tree (the library's source hash must match the tree that travels), then one gpurun call.
# A call gpurun could not place (no box free / backing off: nothing ran, nothing charged) is
# placed again after a pause; a call that ran is never repeated.
cd /root/repo
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
  # (re)build right before each attempt: sources edited while waiting must not travel with a stale library
  python -c "import __graft_entry__ as g; g.build()" > /tmp/build.log 2>&1 || { tail -30 /tmp/build.log; exit 1; }
  timeout 2700 /usr/local/graft/bin/gpurun --timeout ${GT:-1200} -- "$@" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_last.log && ! grep -q "run [1-9]" /tmp/gpurun_last.log; then
    echo "attempt $attempt: not placed ($(grep -o 'no free box\|backing off' /tmp/gpurun_last.log | head -1)); waiting"
    sleep 90
    continue
  fi
  cat /tmp/gpurun_last.log
  exit $rc
done
cat /tmp/gpurun_last.log
exit 3
