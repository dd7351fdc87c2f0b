for v in "" p1 p2; do
  for k in "fwd --N 256 --C 64 --H 56 --K 256 --R 1 --s 1" "dgrad --N 256 --C 256 --H 56 --K 64 --R 1 --s 1" "fwd --N 256 --C 128 --H 28 --K 512 --R 1 --s 1"; do
    echo "variant '$v' $(MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 60 python3 tools/conv_probe.py --kind $k --iters 20 2>&1 | grep TFLOP)"
  done
done
