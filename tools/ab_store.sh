#!/bin/bash
# A/B of the output store policy in the real bench, interleaved rounds.
#   usage: tools/ab_store.sh "cfg2 cfg5" "ZFEC_HIP_STORE=nt" "ZFEC_HIP_STORE=ntsc1" ...
# (register kernels: ZFEC_HIP_STORE=nt|ntsc1|auto; JIT kernels: ZFEC_HIP_JIT_STORE=2 (nt) | 18 (nt sc1))
mkdir -p gpurun_out
workloads=$1; shift
for rnd in 1 2; do
  for w in $workloads; do
    for v in "$@"; do
      echo "== round $rnd $w $v" >> gpurun_out/ab_store.log
      env $v timeout -k 10 200 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu > gpurun_out/ab_s.json 2>gpurun_out/ab_s.err || exit 1
      python -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_s.json') if l.startswith('{')][-1])
r=d['roofline']; q=d['decode_roofline']; b=d.get('batched_1MiB') or {}
L=b.get('layouts', {})
bs=' '.join('%s %.4f/%.4f' % (k, v['frac_of_peak'], v['frac_of_peak_warm']) for k, v in L.items())
print('value %.1f | enc cold %.4f ms frac %.4f warm %.4f | dec cold %.4f warm %.4f | 1MiB %s' % (d['value'], r['launch_ms'], r['frac'], r['frac_warm'], q['frac'], q['frac_warm'], bs or '-'))
" >> gpurun_out/ab_store.log
    done
  done
done
