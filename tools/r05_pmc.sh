#!/bin/bash
# round 5: PMC profiles (tools/profile.sh + tools/pmc_summary.py) of the
# bench workloads named on the command line (on the GPU box; summarise
# gpurun_out/prof_<TAG>_c<config>_<key> here afterwards), each as
#   <config>:<workload key>[:<ENV=VAL>][:<bench args>]
# e.g. 3:config3_n1000000  3:config3_generic_n1000000:MI_CLS_JIT=0
#      3:config3_checksums_n1000000::--pktin-opt 0x3C
set -o pipefail
TAG=${TAG:-r05}
for spec in "$@"; do
  IFS=: read -r cfg key envv extra <<< "$spec"
  echo "== $cfg $key env=[$envv] extra=[$extra]"
  if [ -n "$envv" ]; then export "$envv"; fi
  PROF_SUFFIX="_$key" PROF_EXTRA="$extra" tools/profile.sh $TAG $cfg 1000000 || exit 1
  if [ -n "$envv" ]; then unset "${envv%%=*}"; fi
done
