#!/bin/bash
# round 6: fp32 BN diagnostics, then the whole GPU suite (every failure listed, not -x)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 120 python -u tools/diag_bnf.py > gpurun_out/r6/diag_bnf.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/diag_bnf.py --res 0 > gpurun_out/r6/diag_bnf_nores.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/gpu_full.log 2>&1
echo "pytest rc=$?"
tail -5 gpurun_out/r6/gpu_full.log
