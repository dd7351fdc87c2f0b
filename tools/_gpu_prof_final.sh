A="--model resnet18 --image-size 32 --batch 32 --graph --steps 300 --warmup 20"
bash tools/gpu_recipes.sh ab tnfa MI355X_DP_TN_SPLIT_FUSED "1 0" $A && \
bash tools/gpu_recipes.sh ab tnfb MI355X_DP_TN_SPLIT_FUSED "0 1" $A && \
bash tools/gpu_recipes.sh ab tnfc MI355X_DP_TN_SPLIT_FUSED "1 0" $A
