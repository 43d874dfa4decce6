#!/bin/bash
# print the bench lines written by scripts/quick_all.sh <tag>
tag=${1:-q}
[ -f gpurun_out/${tag}_gpu.log ] && tail -1 gpurun_out/${tag}_gpu.log
for c in c2 c3 c4 c5; do
  [ -f gpurun_out/${tag}_$c.log ] || continue
  python3 -c "
import json
l=[x for x in open('gpurun_out/${tag}_$c.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$c', d['value'], 'step', d['ms_per_step'], 'kernel', d['roofline']['kernel_ms'])"
done
