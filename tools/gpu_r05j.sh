# round 5, session j: host memory end to end on the current tree (tools/e2e_host.py), three runs
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
git_tree=$(python -c "import bench; print(bench.device_tree_hash())")
echo "device tree $git_tree" > $O/e2e_host.log
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/e2e_host.py >> $O/e2e_host.log 2>&1 || { echo e2e-failed; tail -20 $O/e2e_host.log; exit 1; }
done
cat $O/e2e_host.log
