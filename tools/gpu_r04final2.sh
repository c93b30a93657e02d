set -e
# round-4 closing check on the final tree: smoke, GPU suite, default bench,
# configs (each step under its own time limit)
T=${1:-r04ai}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_round4.sh $T suite bench configs
