#!/bin/bash
# A/B of library variants (tools/r04/build_variants.sh) on one box: the quick
# bench per library, AB_PASSES passes in alternating order.
#   tools/r04/ab.sh name... (default = the in-tree build)
set -o pipefail
mkdir -p gpurun_out/ab gpurun_out/r04
for pass in ${AB_PASSES:-1 2}; do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=p2p-file-system-with-gossip-detect-failure-management_amd/lib/libgossiphip.so
    else lib=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_$v.so; fi
    GOSSIPHIP_LIB=$lib timeout -k 10 180 python -u bench.py --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline \
      --no-secondary --files 0 > gpurun_out/ab/$v.$pass.json 2> gpurun_out/ab/$v.$pass.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/$v.$pass.json').read().strip().splitlines()[-1]); print('$v pass $pass', round(d['value'],1), 'rounds/s', round(d['roofline']['avg_launch_ms'],4), 'ms k_round', d['layout']['last_variant'])" | tee -a gpurun_out/ab/summary.txt
  done
done
