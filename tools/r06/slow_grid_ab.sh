set -o pipefail
O=gpurun_out/r06; mkdir -p $O
for pass in 1 2; do for g in 2048 768; do
  GH_SLOW_GRID=$g timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 40 > $O/s38_$g.json 2>> $O/s38.err || exit 1
  python3 - $g $pass <<'PY' | tee -a $O/s38_ab.txt
import json,sys
d=json.loads(open('gpurun_out/r06/s38_%s.json'%sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; s=d['secondary']
def val(x): return x.get('rounds_per_s', x.get('value'))
print('GH_SLOW_GRID=%s pass %s: %.1f rounds/s, fixed %.1f us; %s' % (sys.argv[1], sys.argv[2], d['value'], 1e3*(d['ms_per_step']-r['avg_launch_ms']), {k: round(val(v),1) for k,v in s.items() if isinstance(v, dict) and val(v)}))
PY
done; done
