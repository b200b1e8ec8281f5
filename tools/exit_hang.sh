#!/bin/bash
# Diagnostic: does rx_driver hang at process exit with program-specialised
# kernels (a hipRTC compile in flight when the process exits)?  Runs the
# config 2 receive case N times with MI_CLS_JIT=1 and N times with 0, each
# under its own time limit, and prints the exit codes (124 = hung).
set -o pipefail
OUT=${1:-gpurun_out/exit_hang}
N=${2:-6}
mkdir -p $OUT
trap 'rm -f $OUT/in.pcap' EXIT
timeout -k 10 120 python - "$OUT" <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
from odp_amd import rules as R
from tests import rt_helpers as H
b, p = R.config2(20000)
H.write_pcap(sys.argv[1] + "/in.pcap", [b.frame(i) for i in range(b.n)])
H.write_rules(sys.argv[1] + "/rules.txt", p)
PY
for jit in 1 0; do
  codes=""
  for i in $(seq $N); do
    MI_CLS_JIT=$jit RX_COUNT_ONLY=1 timeout -k 5 20 tests/_bin/rx_driver pcap:in=$OUT/in.pcap \
      $OUT/rules.txt sched 4 1 1 > $OUT/jit${jit}_$i.txt 2>&1
    codes="$codes $?"
  done
  echo "MI_CLS_JIT=$jit exit codes:$codes"
done
