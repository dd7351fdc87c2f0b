#!/bin/bash
# the default bench line (ResNet-152 / ViT secondaries, emulated 8-rank comm) on the final tree
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 700 python bench.py > gpurun_out/r6/bench_default_final.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r6/bench_default_final.log") if l.startswith("{")][-1])
print("rn50", d["value"], d["ms_per_step"])
for k, v in (d.get("secondary_models") or {}).items():
    print(k, v.get("img_s"), v.get("ms_per_step"))
e = d.get("emulated_comm_dp8") or {}
print("emulated_dp8", e.get("img_s"), e.get("ms_per_step"), e.get("comm_exposed_ms"))
PY
