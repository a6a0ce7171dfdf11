"""Print the key numbers of bench.py JSON lines: python tools/bench_summary.py gpurun_out/b_*.log"""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [l for l in open(f).read().splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
    except Exception as e:  # noqa: BLE001
        print(f, "no JSON line:", e)
        continue
    print("%-28s %10.1f Msamples/s  %8.1f ms/step  kernel %7.1f  splat %6.1f  latin %6.1f  parity %s" % (
        f.split("/")[-1], d["value"], d["ms_per_step"], d["kernel_ms_per_step"], d["splat_ms_per_step"],
        d["latin_ms_per_step"], d.get("parity", {}).get("bit_identical")))
