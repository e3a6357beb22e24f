#!/bin/bash
# retry only while no box / slot is free (exit 3 or a "transient" status); any real run ends the loop
OUT=$1; shift
for i in $(seq 1 40); do
  timeout 1700 /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  rc=$?
  if grep -q "status=transient" $OUT && ! grep -q "status=ok\|status=fail" $OUT; then sleep 200; continue; fi
  break
done
echo "RC=$rc" >> $OUT
