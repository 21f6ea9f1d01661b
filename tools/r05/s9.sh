#!/bin/bash
# the REMOVE-taking nibble path as its own instantiation: tier tests, REMOVE
# and D7 parity, then an A/B of the steady round (GH_NIB_RMV=2 forces the
# REMOVE-taking instantiation every round) on the bench workload
set -o pipefail
mkdir -p gpurun_out/r05
O=gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier8.py -x -v --timeout 300 --timeout-method thread > $O/s9_tier8.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "remove or d7 or rejoin" > $O/s9_parity_rm.log 2>&1 || exit 1
for pass in 1 2; do
  for v in 1 2; do
    GH_NIB_RMV=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_rmv${v}_p$pass.json 2> $O/ab_rmv${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_rmv${v}_p$pass.json')); r=d['roofline']; print('rmv=$v pass=$pass', round(d['value'],1), 'rounds/s', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/ab_rmv.txt
  done
done
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tl9 -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/tl9.log 2>&1 || exit 1
python3 tools/r04/round_timeline.py $O/tl9 > $O/s9_timeline.txt || exit 1
tools/r05/probe3.sh || exit 1
for pass in 1 2; do
  for v in 1 2; do
    GH_ROUND_XMAP=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > $O/ab_xmap${v}_p$pass.json 2> $O/ab_xmap${v}_p$pass.err || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/ab_xmap${v}_p$pass.json')); r=d['roofline']; print('xmap=$v pass=$pass', round(d['value'],1), 'rounds/s', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/ab_xmap.txt
  done
done
