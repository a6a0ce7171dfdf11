# development probe: default-kernel parity subsets (GPU box, repo root)
mkdir -p gpurun_out/dbg1
timeout -k 10 600 python -X faulthandler -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "rayqueue or splat_bucket" > gpurun_out/dbg1/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/dbg1/parity.log; [ $rc -eq 0 ] || exit 1
for e in NART_PRIMARY=1 NART_SPLAT_MODE=3; do echo "$e"; env $e timeout -k 10 120 python tools/quick_perf.py -s 64 --reps 2 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms %.2f splat_ms %.2f' % (d['kernel_ms'], d['splat_ms']))" || exit 1; done
