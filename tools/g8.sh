set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in base kv256 base kv256; do
  if [ "$v" = base ]; then unset SDSP_LIB_PATH; else export SDSP_LIB_PATH=$R/stratum-dsp_amd/lib_exp/lib_$v.so; fi
  O=$R/gpurun_out/ab_kvs_$v
  SDSP_SERIAL_STREAMS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o s -- python3 $R/bench.py --tracks 32 --steps 2 --warmup 1 --no-cpu-baseline --no-probe > $O.json 2> $O.err || { echo "$v failed"; tail -5 $O.err; exit 1; }
  python3 - "$O/s_kernel_stats.csv" "$v" "$O.json" <<'PY'
import csv, re, sys, json
for r in csv.DictReader(open(sys.argv[1])):
    if re.search('k_key_vote', r['Name']):
        print(f"{sys.argv[2]:8s} {r['Name'][:40]:40s} calls {r['Calls']:>3} avg {float(r['AverageNs'])/1e3:9.1f} us")
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
print(sys.argv[2], 'sine_30s', d.get('sine_30s'))
PY
done
