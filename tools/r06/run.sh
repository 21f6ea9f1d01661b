#!/bin/bash
# Round-6 GPU steps, one gpurun call each (run from the repo root; every GPU
# step has its own time limit and the steps stop at the first failure):
#   run.sh tests TAG T1 [T2 ...]   pytest node ids (tests/...::name), -m gpu, verbose with prints
#   run.sh suite TAG               the driver's GPU test command (-m gpu) + smoke
#   run.sh bench TAG [ARGS...]     the driver's bench (python3 bench.py --gpus 1 --steps 20 --warmup 5 ARGS)
#   run.sh pmc TAG                 tools/pmc.sh 5 20 (PMC passes + kernel stats of the bench)
#   run.sh ab TAG VAR [ARGS...]    bench A/B of env switch VAR=1 vs VAR=0, three alternating passes
#   run.sh timeline TAG            one steady round's kernels (rocprofv3 kernel trace)
#   run.sh py TAG SECONDS SCRIPT [ARGS...]   a tool script under a time limit
#   run.sh trace TAG MODE ROUNDS MARKER PER R1 [R2...]   tools/r06/slow_rounds.py MODE ROUNDS under a
#                                  rocprofv3 kernel trace, split per round by tools/r06/trace_rounds.py
# Output: gpurun_out/r06/TAG_*
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
export TMPDIR=/tmp
cmd=$1; tag=$2; shift 2
case "$cmd" in
  tests)
    timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu "$@" \
      > $O/${tag}_tests.log 2>&1; rc=$?
    grep -E "PASSED|FAILED|ERROR|passed|failed|Error" $O/${tag}_tests.log | cut -c1-300 | tail -20; exit $rc ;;
  suite)
    ( time timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu > $O/${tag}_gpu_suite.log 2>&1 ) \
      2> $O/${tag}_suite_time.txt || { tail -30 $O/${tag}_gpu_suite.log; exit 1; }
    tail -2 $O/${tag}_gpu_suite.log; cat $O/${tag}_suite_time.txt
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/${tag}_smoke.log 2>&1 || exit 1
    tail -2 $O/${tag}_smoke.log ;;
  bench)
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $O/${tag}_bench.json 2> $O/${tag}_bench.err \
      || { tail $O/${tag}_bench.err; exit 1; }
    tail -c 1500 $O/${tag}_bench.json ;;
  pmc)
    rm -rf gpurun_out/pmc
    bash tools/pmc.sh 5 20 || exit 1
    cp -r gpurun_out/pmc $O/${tag}_pmc; cat gpurun_out/pmc/summary.json | head -c 3000 ;;
  ab)
    var=$1; shift
    for pass in 1 2 3; do for v in 1 0; do
      env "$var=$v" timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary --steps 40 "$@" \
        > $O/${tag}_ab_$v.json 2> $O/${tag}_ab.err || { tail $O/${tag}_ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${tag}_ab_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$var=$v pass $pass: %.1f rounds/s, ms_per_step %.4f, k_round %.4f' % (d['value'], d['ms_per_step'], r['avg_launch_ms']))" | tee -a $O/${tag}_ab.txt
    done; done ;;
  timeline)
    timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/${tag}_tl -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $O/${tag}_tl.log 2>&1 || exit 1
    python3 tools/r04/round_timeline.py $O/${tag}_tl | tee $O/${tag}_timeline.txt ;;
  py)
    secs=$1; shift
    timeout -k 10 "$secs" python3 -u "$@" > $O/${tag}_py.log 2>&1; rc=$?
    tail -40 $O/${tag}_py.log; exit $rc ;;
  trace)
    mode=$1; rounds=$2; marker=$3; per=$4; shift 4
    timeout -s KILL 600 rocprofv3 --kernel-trace --output-format csv -d $O/${tag}_tr -o run -- \
      python3 tools/r06/slow_rounds.py $mode $rounds > $O/${tag}_rounds.jsonl 2> $O/${tag}_tr.log || { tail $O/${tag}_tr.log; exit 1; }
    python3 tools/r06/trace_rounds.py $O/${tag}_tr $marker $per "$@" > $O/${tag}_split.txt || exit 1
    cut -c1-150 $O/${tag}_rounds.jsonl | tail -8; head -60 $O/${tag}_split.txt ;;
  *) sed -n 2,14p "$0"; exit 2 ;;
esac
