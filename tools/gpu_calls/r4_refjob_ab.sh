set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 300 python tools/reference_job.py --batch-size 32 --epochs 2 --tag "$1" "${@:2}" > gpurun_out/r4_refjob_$1.json 2> gpurun_out/r4_refjob_$1.err; }
run nocomm && run force_gated --env MI355X_DP_FORCE_COMM=1 && run force_ungated --env MI355X_DP_FORCE_COMM=1 --env MI355X_DP_GRAPH_GATES=0 && run nocomm2 && run force_gated2 --env MI355X_DP_FORCE_COMM=1
