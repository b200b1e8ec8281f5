#!/bin/bash
# Kernel trace of the runtime receive path (rx_driver rate mode on config 3
# traffic): per-kernel durations of the classify and delivery kernels.
# Usage (via gpurun): tools/rx_prof.sh OUTDIR [frames] [loops] [mode]
set -o pipefail
OUT=${1:-gpurun_out/rxprof}
ROOT=$(pwd)
mkdir -p $OUT
trap "rm -f $ROOT/$OUT/in.pcap" EXIT
timeout -k 10 120 python - "$OUT" ${2:-200000} <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
from odp_amd import rules as R
from tests import rt_helpers as H
b, p = R.config3(int(sys.argv[2]))
H.write_pcap(sys.argv[1] + "/in.pcap", [b.frame(i) for i in range(b.n)])
H.write_rules(sys.argv[1] + "/rules.txt", p)
PY
export RX_COUNT_ONLY=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/kt -o kt -- \
  $ROOT/tests/_bin/rx_driver pcap:in=$ROOT/$OUT/in.pcap:loops=${3:-10} $ROOT/$OUT/rules.txt ${4:-direct} 4 0 1 \
  > $ROOT/$OUT/run.txt 2>&1 || { tail $ROOT/$OUT/run.txt; exit 1; }
cat $(find $ROOT/$OUT/kt -name '*kernel_stats.csv' | head -1)
