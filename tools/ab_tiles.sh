#!/bin/bash
# A/B of K=20/M=60 JIT kernel shapes in the real bench (cfg4, sustained load):
# the default (10-row tiles on 4 waves, planes shared through LDS), 3 tiles of
# 13-14 rows (198 VGPRs, 2 waves/SIMD), and no LDS sharing (each wave transposes
# every input; the decode's 2-wave workgroups are then not LDS-limited).
mkdir -p gpurun_out
for rnd in 1 2; do
  for v in "ZFEC_HIP_JIT_TILE=10" "ZFEC_HIP_JIT_TILE=14 ZFEC_HIP_JIT_WAVES=2" "ZFEC_HIP_JIT_SHARE=0"; do
    echo "== round $rnd $v" >> gpurun_out/ab_tiles.log
    env $v timeout -k 10 150 python bench.py --workload cfg4 --steps 20 --warmup 3 --no-cpu --no-extra > gpurun_out/ab_t.json 2>gpurun_out/ab_t.err || exit 1
    python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_t.json') if l.startswith('{')][-1])
r=d['roofline']; q=d['decode_roofline']
print('value %.1f enc_ms %.4f warm %.4f pairs %.4f | dec_ms %.4f warm %.4f pairs %.4f | %s | %s' % (d['value'], r['launch_ms'], r['launch_ms_warm'], r['launch_ms_event_pairs'], q['launch_ms'], q['launch_ms_warm'], q['launch_ms_event_pairs'], r['kernel'], q['kernel']))
" >> gpurun_out/ab_tiles.log
  done
done
