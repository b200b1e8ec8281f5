#!/bin/bash
# Runtime receive rates on config 3 traffic with the per-phase profile;
# A/B: GPU delivery (default) vs host delivery (ODP_AMD_RX_GPU_DELIVER=0) vs
# pageable pools (ODP_AMD_PINNED_POOLS=0), synchronous bursts
# (ODP_AMD_RX_PIPELINE=0); the loop pktio (classified in place).
# Usage: tools/rx_rate.sh OUTDIR [frames] [loops]
set -o pipefail
OUT=${1:-gpurun_out/rx}
mkdir -p $OUT
trap 'rm -f $OUT/in.pcap $OUT/in_loop.pcap' EXIT
timeout -k 10 120 python - "$OUT" ${2:-200000} <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
from odp_amd import rules as R
from tests import rt_helpers as H
b, p = R.config3(int(sys.argv[2]))
H.write_pcap(sys.argv[1] + "/in.pcap", [b.frame(i) for i in range(b.n)])
# loop rounds: 32 k frames sent into the loop interface per round
H.write_pcap(sys.argv[1] + "/in_loop.pcap", [b.frame(i) for i in range(min(b.n, 32768))])
H.write_rules(sys.argv[1] + "/rules.txt", p)
PY
run() {  # name mode env...
  local name=$1 m=$2; shift 2
  env "$@" ODP_AMD_RX_PROF=1 RX_COUNT_ONLY=1 timeout -k 10 120 tests/_bin/rx_driver pcap:in=$OUT/in.pcap:loops=${LOOPS:-10} $OUT/rules.txt $m 4 0 1 > $OUT/$name.txt 2>&1 || { tail $OUT/$name.txt; exit 1; }
  echo "$name: $(grep -E '^(R|S|RXPROF|RXLOOP) ' $OUT/$name.txt | sed 's/pcap:in=[^ ]* //' | tr '\n' ' ')"
}
runloop() {  # name env...
  local name=$1; shift
  env "$@" ODP_AMD_RX_PROF=1 RX_COUNT_ONLY=1 RX_LOOP_ROUNDS=60 RX_POOL_NUM=65536 timeout -k 10 120 tests/_bin/rx_driver loop $OUT/rules.txt direct 4 0 1 $OUT/in_loop.pcap > $OUT/$name.txt 2>&1 || { tail $OUT/$name.txt; exit 1; }
  echo "$name: $(grep -E '^(R|S|RXPROF loop|RXLOOP) ' $OUT/$name.txt | tr '\n' ' ')"
}
LOOPS=${3:-10}
FRAMES=${2:-200000}
run direct direct NONE=1
run direct_host direct ODP_AMD_RX_GPU_DELIVER=0
run direct_pageable direct ODP_AMD_PINNED_POOLS=0
run sched sched NONE=1
run sched_host sched ODP_AMD_RX_GPU_DELIVER=0
run direct_sync direct ODP_AMD_RX_PIPELINE=0
runloop loop NONE=1
runloop loop_host ODP_AMD_RX_GPU_DELIVER=0
runloop loop_pageable ODP_AMD_PINNED_POOLS=0
