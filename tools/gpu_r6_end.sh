#!/bin/bash
# round 6 end (final tree): full GPU suite, smoke(), default bench line (ResNet-152 / ViT secondaries,
# emulated 8-rank comm)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/end2
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/end2/gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r6/end2/gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6/end2/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r6/end2/smoke.log
timeout -k 10 700 python bench.py > gpurun_out/r6/end2/bench_default.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r6/end2/bench_default.log") if l.startswith("{")][-1])
print("rn50", d["value"], d["ms_per_step"])
for k, v in (d.get("secondary_models") or {}).items():
    print(k, v.get("img_s"), v.get("ms_per_step"))
e = d.get("emulated_comm_dp8") or {}
print("emulated_dp8", e.get("img_s"), e.get("ms_per_step"), e.get("comm_exposed_ms"))
PY
