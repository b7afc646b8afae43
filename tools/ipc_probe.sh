#!/bin/bash
# Two processes of tools/ipc_probe on one device (GPU box): can they map each
# other's buffers (hipIpcOpenMemHandle) and hand off data with device flags?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
D=$(mktemp -d /tmp/ipcprobe.XXXXXX)
ITERS=${ITERS:-2000}
for M in ${MODES:-0 1 2}; do
for B in ${BYTES:-65536 2097152 8388608}; do
  rm -f "$D"/h* "$D"/d*
  timeout -k 5 60 ./tools/ipc_probe 0 "$D" "$ITERS" "$B" 0 "$M" > "$D/o0" 2>&1 &
  p0=$!
  timeout -k 5 60 ./tools/ipc_probe 1 "$D" "$ITERS" "$B" 0 "$M" > "$D/o1" 2>&1 &
  p1=$!
  wait $p0; r0=$?
  wait $p1; r1=$?
  cat "$D/o0" "$D/o1"
  echo "mode=$M bytes=$B rc0=$r0 rc1=$r1"
  if [ $r0 -ne 0 ] || [ $r1 -ne 0 ]; then rm -rf "$D"; exit 1; fi
done
done
rm -rf "$D"
