# A/B of library builds on bench configs (gpurun): tools/dbg/lib_ab.sh "bench args" lib1 lib2 ...
set -u
mkdir -p gpurun_out/ab
A=$1; shift
for lib in "$@"; do
  ZS_LIB=$lib timeout -k 10 200 python3 bench.py $A --no-shard-sweep --no-e2e --no-cpu-baseline > gpurun_out/ab/x.log 2>&1 || { tail -3 gpurun_out/ab/x.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab/x.log').read().strip().split('\n')[-1]); print('$lib', d['ms_per_step'], {k:v for k,v in d['roofline']['phase_ms'].items() if v>0.05})"
done
