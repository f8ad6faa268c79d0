set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rm -f gpurun_out/ab_store.log
timeout -k 10 600 bash tools/ab_store.sh "cfg2 cfg3" "ZFEC_HIP_STORE=nt" "ZFEC_HIP_STORE=auto" "ZFEC_HIP_STORE=auto ZFEC_HIP_JIT_STORE=18"
for v in nt auto; do echo "== ZFEC_HIP_STORE=$v" >> gpurun_out/e2e_ab.log; ZFEC_HIP_STORE=$v timeout -k 10 120 python tools/e2e_host.py >> gpurun_out/e2e_ab.log 2>&1; done
echo done
