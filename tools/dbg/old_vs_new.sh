set -u
mkdir -p gpurun_out/r04e
A="--mode inflate --stream-bytes 262144 --replicas 1 --corpus text --streams 512 --no-shard-sweep --no-e2e --no-cpu-baseline"
for lib in tools/dbg/libzsgpu_2299bd4.so zlib-streams-ts_amd/libzsgpu.so; do
 for o in "" "--option seg_bits=8192"; do
  ZS_LIB=$lib timeout -k 10 200 python3 bench.py $A $o > gpurun_out/r04e/old.log 2>&1 || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r04e/old.log').read().strip().split('\n')[-1]); print('$lib $o', d['ms_per_step'], {k:v for k,v in d['roofline']['phase_ms'].items() if v>0.05})"
 done
done
