#!/bin/bash
# HIP API time inside the receive path: rocprofv3 HIP runtime trace of the
# rx_driver on config 3 traffic (pcap direct, loop); per-call statistics.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-rxh}
mkdir -p $OUT
timeout -k 10 120 python - "$OUT" 200000 <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
from odp_amd import rules as R
from tests import rt_helpers as H
b, p = R.config3(int(sys.argv[2]))
H.write_pcap(sys.argv[1] + "/in.pcap", [b.frame(i) for i in range(b.n)])
H.write_pcap(sys.argv[1] + "/in_loop.pcap", [b.frame(i) for i in range(min(b.n, 32768))])
H.write_rules(sys.argv[1] + "/rules.txt", p)
PY
cd /tmp && export TMPDIR=/tmp
RX_COUNT_ONLY=1 timeout -k 10 180 rocprofv3 --hip-trace --stats --output-format csv -d $OUT/pcap -o ht -- $ROOT/tests/_bin/rx_driver pcap:in=$OUT/in.pcap:loops=10 $OUT/rules.txt direct 4 0 1 > $OUT/pcap.log 2>&1 || { tail $OUT/pcap.log; exit 1; }
RX_COUNT_ONLY=1 RX_LOOP_ROUNDS=60 RX_POOL_NUM=65536 timeout -k 10 180 rocprofv3 --hip-trace --stats --output-format csv -d $OUT/loop -o ht -- $ROOT/tests/_bin/rx_driver loop $OUT/rules.txt direct 4 0 1 $OUT/in_loop.pcap > $OUT/loop.log 2>&1 || { tail $OUT/loop.log; exit 1; }
rm -f $OUT/in.pcap $OUT/in_loop.pcap $OUT/*/ht_hip_api_trace.csv
for f in $OUT/pcap $OUT/loop; do echo "== $f"; find $f -name "*hip_api_stats.csv" -exec cat {} \; | cut -d, -f1-5 | head -16; done
