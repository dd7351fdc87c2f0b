#!/bin/bash
# PMC passes over the ResNet-152 layer-3 expand conv (256 -> 1024 at 14x14, 1x1),
# panel kernel (MI355X_DP_PANEL=1, default) vs the 128-tile nt_kernel (0); counter-only runs
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6/pmc
mkdir -p $OUT
P1=SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,GRBM_COUNT,GRBM_GUI_ACTIVE
P2=FETCH_SIZE,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_WAVES
for mode in 1 0; do
  MI355X_DP_PANEL=$mode timeout -k 10 120 python3 tools/conv_probe.py --kind fwd --N 256 --C 256 --H 14 --K 1024 --R 1 --s 1 --iters 50 > $OUT/probe_p$mode.log 2>&1 || exit $?
  i=1
  for ctr in $P1 $P2; do
    MI355X_DP_PANEL=$mode timeout -s KILL 60 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d $OUT/p${mode}_$i -o run -- python3 tools/conv_probe.py --kind fwd --N 256 --C 256 --H 14 --K 1024 --R 1 --s 1 --iters 20 > $OUT/p${mode}_$i.log 2>&1 || exit $?
    i=$((i+1))
  done
  python3 tools/pmc_summary.py $(find $OUT/p${mode}_1 $OUT/p${mode}_2 -name '*counter_collection.csv') --top 3 > $OUT/summary_p$mode.md 2>&1
done
cat $OUT/probe_p1.log $OUT/probe_p0.log $OUT/summary_p1.md $OUT/summary_p0.md
