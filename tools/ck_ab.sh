#!/bin/bash
# Checksum-path A/B on config 3 IMIX with valid checksums: kernel time per
# launch for pktin option sets (0x04 IPv4 header only: the general parser,
# no L4 sums; 0x7C0 drop only: fast parse; 0x3C all checksums; 0x3C on the
# SCTP mix), then SQ counters for 0x3C.  Usage (via gpurun): tools/ck_ab.sh
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
for a in "3 0x0" "3 0x04" "3 0x7C0" "3 0x3C" "35 0x3C"; do
  set -- $a
  r=$(timeout -k 10 120 python bench.py --config $1 --pktin-opt $2 --steps 10 --warmup 3 \
      --timed-only 2>/dev/null) || { echo "config $1 opt $2 failed"; exit 1; }
  echo "config $1 opt $2: $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
done
[ -n "$CK_COUNTERS" ] && tools/counters.sh ck "--config 3 --pktin-opt 0x3C --steps 5 --warmup 2 --timed-only"
exit 0
