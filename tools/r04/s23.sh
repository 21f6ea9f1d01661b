#!/bin/bash
# packed row records for the nibble path's staging: A/B on the bench (two passes), then the tier / parity suites and the full-size steady state
set -o pipefail
mkdir -p gpurun_out/r04/s23
for pass in 1 2; do for nrec in 1 0; do
  GH_DNW=$nrec timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary --steps 40 > gpurun_out/r04/s23/b_$nrec.json 2> gpurun_out/r04/s23/b.err || { tail gpurun_out/r04/s23/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/s23/b_$nrec.json').read().strip().splitlines()[-1]); r=d['roofline']; print('dnw $nrec pass $pass: value %.1f ms_per_step %.4f k_round %.4f' % (d['value'], d['ms_per_step'], r['avg_launch_ms']))"
done; done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests --deselect tests/test_gpu_fullsize.py > gpurun_out/r04/s23/suite.log 2>&1; rc=$?; tail -3 gpurun_out/r04/s23/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_fullsize.py::test_c3_fullsize_crash_1pct tests/test_gpu_fullsize.py::test_c3_fullsize_columns_g8 > gpurun_out/r04/s23/full.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04/s23/full.log | cut -c1-200; exit $rc
