#!/bin/bash
# Round-4 GPU steps (run under gpurun from the repo root; each GPU step has its own time limit):
#   run.sh suite                 the -m gpu suite without the full-size module
#   run.sh fullsize T1 [T2 ...]  full-size tests by name (tests/test_gpu_fullsize.py::T)
#   run.sh bench-pmc             the driver's bench, its rocprofv3 kernel stats, the PMC passes (tools/pmc.sh)
#   run.sh ab VAR                bench A/B of an engine env switch VAR=1 vs VAR=0, two alternating passes
#   run.sh timeline              one steady round's kernels under rocprofv3 (tools/r04/round_timeline.py)
#   run.sh exchange              tools/shard_exchange.py, all six legs
#   run.sh legs                  the crash leg and the two collapsed legs round by round
set -o pipefail
out=gpurun_out/r04/run
mkdir -p $out
export TMPDIR=/tmp
py="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
case "$1" in
  suite)
    timeout -k 10 900 $py tests --deselect tests/test_gpu_fullsize.py > $out/suite.log 2>&1; rc=$?
    tail -3 $out/suite.log; exit $rc ;;
  fullsize)
    shift; T=""; for t in "$@"; do T="$T tests/test_gpu_fullsize.py::$t"; done
    timeout -k 10 1150 $py -v -s $T > $out/fullsize.log 2>&1; rc=$?
    grep -E "PASSED|FAILED|passed|failed" $out/fullsize.log | cut -c1-200; exit $rc ;;
  bench-pmc)
    rm -rf gpurun_out/pmc
    timeout -k 10 900 python3 bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $out/prof.log 2>&1 || exit 1
    bash tools/pmc.sh 5 20 ;;
  ab)
    for pass in 1 2; do for v in 1 0; do
      env "$2=$v" timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary --steps 40 > $out/ab_$v.json 2> $out/ab.err || { tail $out/ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$out/ab_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$2=$v pass $pass: %.1f rounds/s, ms_per_step %.4f, k_round %.4f' % (d['value'], d['ms_per_step'], r['avg_launch_ms']))"
    done; done ;;
  timeline)
    timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $out/tl -o run -- \
      python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --files 0 > $out/tl.log 2>&1 || exit 1
    python3 tools/r04/round_timeline.py $out/tl ;;
  exchange)
    timeout -k 10 600 python -u tools/shard_exchange.py 65536 8 5 > $out/exchange.log 2>&1; rc=$?
    grep -v "^{" $out/exchange.log | cut -c1-220; exit $rc ;;
  legs)
    timeout -k 10 300 python3 -u tools/r04/crash_probe.py > $out/crash.log 2>&1 || exit 1
    timeout -k 10 300 python3 -u tools/r04/leg_probe.py ref 24 > $out/ref.log 2>&1 || exit 1
    timeout -k 10 300 python3 -u tools/r04/leg_probe.py ring 24 > $out/ring.log 2>&1 || exit 1
    tail -8 $out/crash.log; tail -3 $out/ref.log; tail -3 $out/ring.log ;;
  *) sed -n 2,9p "$0"; exit 2 ;;
esac
