#!/bin/bash
# Kernel durations inside the receive path (rocprofv3 kernel trace of the
# rx_driver on config 3 traffic, pcap direct and loop): classify, the
# receive chain's decide and deliver kernels.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-rxk}
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
RX_COUNT_ONLY=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/pcap -o kt -- $ROOT/tests/_bin/rx_driver pcap:in=$OUT/in.pcap:loops=10 $OUT/rules.txt direct 4 0 1 > $OUT/pcap.log 2>&1 || { tail $OUT/pcap.log; exit 1; }
RX_COUNT_ONLY=1 RX_LOOP_ROUNDS=60 RX_POOL_NUM=65536 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/loop -o kt -- $ROOT/tests/_bin/rx_driver loop $OUT/rules.txt direct 4 0 1 $OUT/in_loop.pcap > $OUT/loop.log 2>&1 || { tail $OUT/loop.log; exit 1; }
rm -f $OUT/in.pcap $OUT/in_loop.pcap
for f in $OUT/pcap $OUT/loop; do echo "== $f"; find $f -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -12; done
