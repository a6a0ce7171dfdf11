# development probe: k_primary LDS budget (GPU box): kernel trace per NART_PRIMARY_LDS_KB value
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
for kb in "$@"; do
  NART_PRIMARY_LDS_KB=$kb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp$kb -o run -- python3 $R/tools/quick_perf.py -s 64 --reps 2 > $R/gpurun_out/pp$kb.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$R/gpurun_out/pp$kb/run_kernel_stats.csv')):
    if 'k_primary' in r['Name'] or 'k_render_rq' in r['Name']: print('$kb', r['Name'][:28], round(float(r['AverageNs'])/1e6, 2))"
done
