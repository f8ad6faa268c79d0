# round 5, session u: JIT kernels sharing the unit's input planes through LDS in
# phases of 8 inputs (16 KiB) instead of all k at once (k20: 40 KiB, 2 waves per
# SIMD on the r = 20 decode), against the committed tree (scratch/base):
# cfg4 bench lines and the GPU JIT tests
set -o pipefail
O=gpurun_out/${TAG:-r05u}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_jit.py \
  "tests/test_gpu_parity.py::test_config4_1024_stripes_of_1mib" > $O/pytest_jit.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest_jit.log; exit 1; }
tail -2 $O/pytest_jit.log
for i in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=.; else d=scratch/base; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload cfg4 --steps 20 --no-cpu) > $O/cfg4_${t}_$i.json 2> $O/cfg4_${t}_$i.err \
      || { echo cfg4-$t-failed; tail -20 $O/cfg4_${t}_$i.err; exit 1; }
    python tools/show_bench.py $O/cfg4_${t}_$i.json | head -1
  done
done
