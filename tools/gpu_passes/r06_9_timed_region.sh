#!/bin/bash
# Round-6 GPU pass 9: the 20-step timed region's fixed costs -- HIP's spin wait, device
# kernargs -- at the driver's own settings (--steps 20 --warmup 5), three runs each.
set -uo pipefail
OUT=gpurun_out/r06i
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2 3; do
  for mode in spin default kernarg; do
    case $mode in
      spin) env_set="BENCH_HIP_SPIN=1" ;;
      default) env_set="BENCH_HIP_SPIN=0" ;;
      kernarg) env_set="BENCH_HIP_SPIN=1 HIP_FORCE_DEV_KERNARG=1" ;;
    esac
    env $env_set timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --skip-cpu-baseline --no-c5 > "$OUT/${mode}_$r.log" 2>&1 || exit 1
    python3 - "$OUT/${mode}_$r.log" "$mode" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(sys.argv[2], f"ms_per_step {d['ms_per_step']*1e3:.2f} us  kernel {d['roofline']['kernel_avg_ms']*1e3:.2f} us  value {d['value']/1e6:.1f} M  sched {d['config'].get('hip_schedule')}")
PY
  done
done
