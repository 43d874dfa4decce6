#!/bin/bash
# summary of scripts/ab.sh <tag> output
tag=$1
for f in gpurun_out/${tag}_*_gpu.log; do echo "$f: $(tail -1 $f)"; done
for f in gpurun_out/${tag}_*_C*.log; do
  python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', d['value'], 'kernel', d['roofline']['kernel_ms'])"
done
