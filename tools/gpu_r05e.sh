# round 5, session e: matapply_bsr table forms with the block pointers in the
# arguments and the routine-address tables cached on the device per matrix:
# parity, then A/B against 732a84b (scratch/base) on the first_seen leg and the
# generic wide shapes
set -o pipefail
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py \
  "tests/test_gpu_parity.py::test_config3_256mib_roundtrip" "tests/test_gpu_parity.py::test_config4_1024_stripes_of_1mib" \
  tests/test_gpu_bsg.py tests/test_gpu_jit.py > $O/pytest_bsr.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest_bsr.log; exit 1; }
tail -2 $O/pytest_bsr.log
for i in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=.; else d=scratch/base; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload first_seen) > $O/fs_${t}_$i.json 2> $O/fs_${t}_$i.err \
      || { echo fs-$t-failed; tail -20 $O/fs_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/60,30/70,12/30,10/16,40/60,94/100,128/256,200/256,255/256 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
