set -o pipefail
timeout -k 10 300 python -m odp_amd._build /tmp/vso DIAG_STAGEONLY > /dev/null || exit 1
timeout -k 10 300 python -m odp_amd._build /tmp/vsl DIAG_STAGEONLY DIAG_FORCE_LO > /dev/null || exit 1
for d in /tmp/vso /tmp/vsl; do for c in 3 2; do
ODP_AMD_LIB_DIR=$d timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --timed-only > /tmp/t.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('/tmp/t.json')); print('$d config $c kernel_us', round(d['roofline']['kernel_ms']*1e3,2))"
done; done
mkdir -p gpurun_out/r02f
for d in /tmp/vso /tmp/vsl $(pwd)/odp_amd; do
  ( cd /tmp && export TMPDIR=/tmp && ODP_AMD_LIB_DIR=$d timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02f/f$(basename $d) -o p -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 5 --warmup 2 --timed-only > /dev/null 2>&1 ) || exit 1
  python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('$GRAFT_REPO_ROOT/gpurun_out/r02f/f$(basename $d)/p_counter_collection.csv') for r in csv.DictReader(open(f)) if 'mi_cls' in r['Kernel_Name']]
print('$d FETCH_SIZE x2 MB', 2*sum(v)/len(v)*1024/1e6)"
done
