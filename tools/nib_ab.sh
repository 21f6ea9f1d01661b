#!/bin/bash
# A/B of the nibble path's lane shape (tools/build_nib_variants.sh): the
# quick bench per library, twice in alternating order.
#   tools/nib_ab.sh name... (default = the in-tree build)
set -o pipefail
mkdir -p gpurun_out/nib_ab
for pass in ${NIB_AB_PASSES:-1 2}; do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=p2p-file-system-with-gossip-detect-failure-management_amd/lib/libgossiphip.so
    else lib=p2p-file-system-with-gossip-detect-failure-management_amd/lib/variants/libgossiphip_$v.so; fi
    GOSSIPHIP_LIB=$lib timeout -k 10 180 python -u bench.py --steps ${NIB_AB_STEPS:-20} --warmup 5 --no-cpu-baseline --no-secondary \
      --files 0 > gpurun_out/nib_ab/$v.$pass.json 2> gpurun_out/nib_ab/$v.$pass.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/nib_ab/$v.$pass.json').read().strip().splitlines()[-1]); print('$v pass $pass', round(d['value'],1), 'rounds/s', round(d['roofline']['avg_launch_ms'],3), 'ms k_round', d['layout']['last_variant'])" | tee -a gpurun_out/nib_ab/summary.txt
  done
done
