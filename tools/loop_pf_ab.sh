#!/bin/bash
# Loop-pktio receive rate A/B of the header prefetch distance in the loop
# staging (ODP_AMD_LOOP_PF), interleaved on one box.  Usage: tools/loop_pf_ab.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/pf}
mkdir -p $OUT
trap 'rm -f $OUT/in_loop.pcap' EXIT
timeout -k 10 120 python - "$OUT" <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
from odp_amd import rules as R
from tests import rt_helpers as H
b, p = R.config3(32768)
H.write_pcap(sys.argv[1] + "/in_loop.pcap", [b.frame(i) for i in range(b.n)])
H.write_rules(sys.argv[1] + "/rules.txt", p)
PY
for rep in 1 2; do
  for pf in 16 48 96; do
    ODP_AMD_LOOP_PF=$pf ODP_AMD_RX_PROF=1 RX_COUNT_ONLY=1 RX_LOOP_ROUNDS=60 RX_POOL_NUM=65536 timeout -k 10 120 tests/_bin/rx_driver loop $OUT/rules.txt direct 4 0 1 $OUT/in_loop.pcap > $OUT/pf$pf.$rep.txt 2>&1 || { tail $OUT/pf$pf.$rep.txt; exit 1; }
    echo "pf $pf rep $rep: $(grep -E '^R ' $OUT/pf$pf.$rep.txt) $(grep -oE 'stage_ns [0-9]+' $OUT/pf$pf.$rep.txt)"
  done
done
