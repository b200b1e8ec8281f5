#!/bin/bash
# Host time of the receive delivery submit (MI_CLS_PROF: event wait, kernel
# launch, event record per submit) on the pcap direct receive of config 3
# traffic, with the per-phase receive profile (ODP_AMD_RX_PROF).
set -o pipefail
mkdir -p gpurun_out/rxp
timeout -k 10 120 python - gpurun_out/rxp 200000 <<'PY' || exit 1
import sys
sys.path.insert(0, ".")
from odp_amd import rules as R
from tests import rt_helpers as H
b, p = R.config3(int(sys.argv[2]))
H.write_pcap(sys.argv[1] + "/in.pcap", [b.frame(i) for i in range(b.n)])
H.write_rules(sys.argv[1] + "/rules.txt", p)
PY
MI_CLS_PROF=1 ODP_AMD_RX_PROF=1 RX_COUNT_ONLY=1 timeout -k 10 120 tests/_bin/rx_driver pcap:in=gpurun_out/rxp/in.pcap:loops=10 gpurun_out/rxp/rules.txt direct 4 0 1 > gpurun_out/rxp/direct.txt 2>&1
rc=$?; rm -f gpurun_out/rxp/in.pcap; grep -E "^(R|S|RXPROF|RXLOOP|MI_CLS_PROF)" gpurun_out/rxp/direct.txt; exit $rc
