#!/bin/bash
for pad in 0 4096 9216 16384; do
  echo "pad $pad: $(BSG_LDS_PAD_BYTES=$pad timeout -k 10 120 python bench.py --skip-cpu-baseline --steps 300 2>/dev/null | python3 -c 'import json,sys;d=json.load(sys.stdin);print(round(d["value"]/1e6,2),"M/s", round(d["roofline"]["kernel_avg_ms"]*1e3,1),"us")')"
done
