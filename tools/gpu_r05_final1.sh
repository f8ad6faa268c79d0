# round 5 final tree, part 1: the whole GPU suite, smoke, the bench lines of every
# BASELINE workload, the host-batch probe.  Every GPU step has its own limit;
# the first failure ends the script.
set -o pipefail
O=gpurun_out/${TAG:-r05f1}
mkdir -p $O
python -c "import bench; print(bench.device_tree_hash())" > $O/tree.txt
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo pytest-failed; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke-failed; tail $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { echo bench2-failed; tail $O/bench_cfg2.err; exit 1; }
for w in cfg3 cfg4 cfg5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 > $O/bench_$w.json 2> $O/bench_$w.err || { echo bench-$w-failed; tail $O/bench_$w.err; exit 1; }
done
timeout -k 10 300 python -u tools/host_batch_probe.py > $O/host_batch.log 2>&1 || { echo hb-failed; tail $O/host_batch.log; exit 1; }
python tools/show_bench.py $O/bench_cfg2.json
echo final1-done
