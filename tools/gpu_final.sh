# Round-end rehearsal: the GPU suite, smoke() and the default bench line of the committed tree.
mkdir -p gpurun_out/final
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gputests.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > gpurun_out/final/bench.log 2>&1
rc=$?
tail -2 gpurun_out/final/gputests.log; tail -1 gpurun_out/final/bench.log | cut -c1-400
exit $rc
