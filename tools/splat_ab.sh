# development probe: LDS splat variants vs col4 at SPP (GPU box): tools/splat_ab.sh LIB SPP "ENV..." ...
LIB=$1; SPP=$2; shift 2
NART_HIP_LIB=$LIB NART_SPLAT_MODE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "splat_bucket and lds or (rayqueue and framebuffer_glass_sphere_c1)" 2>&1 | tail -1
for e in "$@"; do echo "$e: $(env NART_HIP_LIB=$LIB $e timeout -k 10 120 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('splat_ms %.2f' % d['splat_ms'])")" || exit 1; done
