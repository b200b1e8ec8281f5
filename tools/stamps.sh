set -o pipefail
timeout -k 10 300 python -m odp_amd._build /tmp/vdiag DIAG_STAMPS WIN=${WINV:-128} > /dev/null || exit 1
for args in "--config 20" "--config 2" "--config 3" "--config 20 --n 250000"; do
  echo "== $args"
  ODP_AMD_LIB_DIR=/tmp/vdiag timeout -k 10 200 python bench.py $args --steps 3 --warmup 1 --no-cpu --no-extra 2>&1 >/dev/null | grep DIAG | tail -2 || exit 1
done
