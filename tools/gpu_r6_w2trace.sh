#!/bin/bash
# the world-2 gated graphed engine (IPC-only smddp, 2 ranks on cuda:0, batch 256
# at 224x224 as in test_graphed_engine_two_ranks_gated_buckets) with each rank under its own
# rocprofv3 --kernel-trace: with command-processor gates (hipStreamWaitValue32) no flag_gate_kernel
# may appear; then the same with MI355X_DP_GATE_WAIT=kernel for contrast.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6/w2trace
mkdir -p $OUT
run() {  # $1 tag, $2 port, extra env via the caller
  local pids=()
  for r in 0 1; do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$2 \
    MI355X_DP_SMDDP_IPC_ONLY=1 MI355X_DP_SMDDP_DEVICE=0 MI355X_DP_SMDDP_IPC_MB=4 \
    GRAPHED_BATCH=256 GRAPHED_SIZE=224 GRAPHED_BCAST=0 MI355X_DP_ENGINE_GRAPH_MAX_NUMEL=67108864 GPU_MAX_HW_QUEUES=6 \
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1_r$r -o $1_r$r -- python3 tools/graphed_world2.py \
      > $OUT/$1_r$r.log 2>&1 &
    pids+=($!)
  done
  local rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  return $rc
}
run cp 29611 || exit $?
MI355X_DP_GATE_WAIT=kernel run kernel 29612 || exit $?
for f in $(find $OUT -name '*kernel_stats.csv'); do
  echo "== $f"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r.get("Name", "")
    if "flag" in n or "ipc" in n.lower():
        print(n[:60], r.get("Calls"), r.get("TotalDurationNs"))
PY
done
grep -h '"rank"' $OUT/*.log | cut -c1-400
