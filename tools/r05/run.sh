#!/bin/bash
# Round-5 GPU steps as one parameterised script (replaces the one-off sNN.sh
# files; run under gpurun from the repo root; every GPU step has its own time
# limit and the script stops at the first failure). Output: gpurun_out/r05/TAG_*
#   run.sh suite TAG                      the driver's GPU test command (-m gpu), then the smoke
#   run.sh tests TAG PYTEST_ARGS...       pytest -m gpu on the given tests / -k filters (-v, prints kept)
#   run.sh fullsize TAG -k EXPR           tests/test_gpu_fullsize.py --fullsize -k EXPR
#   run.sh bench TAG                      the driver's bench (--gpus 1 --steps 20 --warmup 5)
#   run.sh pmc TAG                        tools/pmc.sh 5 20 (PMC passes + kernel stats of the bench)
#   run.sh ab TAG VAR V1 V2 [PASSES]      bench A/B of the engine env switch VAR at V1 / V2, alternating
#   run.sh timeline TAG                   one steady round's kernels (tools/r04/round_timeline.py)
#   run.sh crash TAG                      the crash leg per round (tools/r05/crash_rounds.py 30)
#   run.sh exchange TAG LAYOUT            tools/shard_exchange.py 65536 8 3 with GH_EXCHANGE_ONLY=LAYOUT
#   run.sh probe TAG N                    tools/r05/probeN.sh (gprobe2 / 3 / 4 access-pattern probes)
# Steps of this round and the profiles they wrote: tools/r05/README.md.
set -o pipefail
O=gpurun_out/r05
mkdir -p $O
export TMPDIR=/tmp
cmd=$1; tag=$2; shift 2
T="--timeout 600 --timeout-method thread"
case "$cmd" in
  suite)
    ( time timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/${tag}_gpu_suite.log 2>&1 ) \
      2> $O/${tag}_suite_time.txt || exit 1
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/${tag}_smoke.log 2>&1 || exit 1 ;;
  tests)
    timeout -k 10 900 python -u -m pytest -x -v -s $T -m gpu "$@" > $O/${tag}_tests.log 2>&1 || exit 1 ;;
  fullsize)
    timeout -k 10 1100 python -u -m pytest tests/test_gpu_fullsize.py --fullsize -x -v -s $T "$@" \
      > $O/${tag}_fullsize.log 2>&1 || exit 1 ;;
  bench)
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${tag}_bench.json 2> $O/${tag}_bench.err || exit 1 ;;
  pmc)
    bash tools/pmc.sh 5 20 || exit 1
    cp -r gpurun_out/pmc $O/${tag}_pmc ;;
  ab)
    var=$1; v1=$2; v2=$3; passes=${4:-2}
    for pass in $(seq 1 $passes); do for v in $v1 $v2; do
      env "$var=$v" timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline \
        > $O/${tag}_ab_${v}_p$pass.json 2> $O/${tag}_ab.err || exit 1
      python3 -c "import json; d=json.load(open('$O/${tag}_ab_${v}_p$pass.json')); r=d['roofline']; print('$var=$v pass=$pass', round(d['value'],1), 'rounds/s', round(r['avg_launch_ms'],4), 'ms', round(r['frac'],3))" | tee -a $O/${tag}_ab.txt
    done; done ;;
  timeline)
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${tag}_tl -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/${tag}_tl.log 2>&1 || exit 1
    python3 tools/r04/round_timeline.py $O/${tag}_tl > $O/${tag}_timeline.txt || exit 1 ;;
  crash)
    timeout -k 10 300 python3 tools/r05/crash_rounds.py 30 > $O/${tag}_crash_rounds.jsonl 2>&1 || exit 1 ;;
  exchange)
    GH_EXCHANGE_ONLY=$1 timeout -k 10 300 python3 tools/shard_exchange.py 65536 8 3 > $O/${tag}_$1.txt 2>&1 || exit 1 ;;
  probe)
    bash tools/r05/probe$1.sh || exit 1 ;;
  *) sed -n 2,17p "$0"; exit 2 ;;
esac
