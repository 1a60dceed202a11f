set -e
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for i in 1 2; do
  SDSP_SERIAL_STREAMS=1 timeout -k 10 200 $B > gpurun_out/ab_serial_reuse_$i.json 2>/dev/null
  SDSP_SERIAL_STREAMS=1 SDSP_NO_ROW_REUSE=1 timeout -k 10 200 $B > gpurun_out/ab_serial_noreuse_$i.json 2>/dev/null
  timeout -k 10 200 $B > gpurun_out/ab_reuse_$i.json 2>/dev/null
  SDSP_NO_ROW_REUSE=1 timeout -k 10 200 $B > gpurun_out/ab_noreuse_$i.json 2>/dev/null
done
