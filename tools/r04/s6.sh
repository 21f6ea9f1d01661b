#!/bin/bash
# the driver's bench command, its rocprofv3 kernel stats, then the PMC passes at the bench's warm-up
set -o pipefail
mkdir -p gpurun_out/r04; rm -rf gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 900 python3 bench.py > gpurun_out/r04/s6_bench.json 2> gpurun_out/r04/s6_bench.err || { tail gpurun_out/r04/s6_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04/s6_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('value', d['value'], 'ms_per_step', d['ms_per_step'], 'k_round', r['avg_launch_ms'], 'frac', r['frac']); print('secondary', json.dumps({k: {kk: v[kk] for kk in ('rounds_per_s','k_round_ms') if kk in v} for k, v in (d.get('secondary') or {}).items()}))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/s6_prof -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > gpurun_out/r04/s6_prof.log 2>&1 || exit 1
bash tools/pmc.sh 5 20 || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/pmc/summary.json')); print({k: d.get(k) for k in ('traffic_bytes','traffic_over_compulsory','l2_hit_rate','valu_busy_frac','ta_busy_frac','td_busy_frac')})"
