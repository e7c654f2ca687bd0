#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for n in ${LLM_NS:-64 256}; do for opt in ${LLM_OPTS:-512 1}; do
  timeout -k 10 200 python3 bench.py --mode inflate --stream-bytes 262144 --streams $n --replicas 1 --corpus text --no-shard-sweep --no-e2e --no-cpu-baseline --steps 5 --warmup 2 --option lane_large_min=$opt > gpurun_out/llm_${n}_$opt.log 2>&1 || { tail -3 gpurun_out/llm_${n}_$opt.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['verify'].get('mismatches'))" gpurun_out/llm_${n}_$opt.log $n $opt
done; done
