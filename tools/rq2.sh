# development probe: ray-queue kernel scheduling modes at SPP (GPU box): tools/rq2.sh SPP
SPP=$1
for lib in nart_amd/lib/libnart_hip.so abbuild/b512/libnart_hip.so; do
  for qm in 2 1; do
    echo "$lib queue=$qm"; NART_HIP_LIB=$lib NART_QUEUE=$qm NART_VARIANT=3 timeout -k 10 120 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | cut -c1-100 || exit 1
  done
done
echo "k_render"; NART_VARIANT=0 timeout -k 10 120 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | cut -c1-100
