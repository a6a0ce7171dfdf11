# development probe: scheduling knobs on the 1/8 C3 shard (rank 0), GPU box: tools/shard_sweep.sh "ENV=.. ENV2=.." ...
for e in "$@"; do
  echo "$e: $(env $e timeout -k 10 120 python tools/shard_perf.py --ns 8 --rank 0 --reps 2 2>/dev/null | grep '{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['worst']['kernel_ms'])")" || exit 1
done
