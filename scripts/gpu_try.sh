#!/bin/bash
# Submit one gpurun command; re-submit ONLY while the pool ran nothing (status=transient, nothing charged).
# Stops at the first call that actually ran (whatever its result).  $1 = command, $2 = output file, $3 = max tries
cmd="$1"; out="$2"; n=${3:-10}
for i in $(seq 1 $n); do
  timeout 1700 /usr/local/graft/bin/gpurun --timeout 1200 -- "$cmd" > "$out" 2>&1
  if grep -q "status=transient" "$out" && grep -qE "charged=(0\.0s|Nones)" "$out"; then
    w=$(grep -oE "retry in [0-9]+s" "$out" | grep -oE "[0-9]+" | head -1); w=${w:-240}; [ $w -lt 240 ] && w=240
    echo "try $i: nothing ran; waiting $((w+10))s" >> "$out.tries"
    sleep $((w+10)); continue
  fi
  echo "try $i: ran" >> "$out.tries"; break
done
