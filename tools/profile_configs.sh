#!/bin/bash
# rocprofv3 kernel stats + separate PMC passes (HBM bytes, VALU) for the non-headline
# step kernels: VerticalCREnv 2048x32 (C3), DescentEnv 4096 (C5's env) and the Merge C4
# shards (512 / 1024 / 2048 envs, lookahead on).  GPU box, repo root:
#   bash tools/profile_configs.sh r03        -> gpurun_out/profcfg_<tag>/, then
#   python3 tools/profile_configs_summary.py gpurun_out/profcfg_<tag> <tag>
set -uo pipefail
TAG=${1:-r03}
OUT=gpurun_out/profcfg_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in "vertical 32 2048 30 1" "descent 1 4096 30 0" "merge 32 512 10 1" "merge 32 1024 10 1" "merge 32 2048 10 1"; do
  t=$(echo $c | tr ' ' '_')
  P="python3 tools/one_config.py $c 40"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$t/trace" -o run -- $P > /dev/null 2>&1 || { echo "trace fail $t"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$t/pmc_fetch" -o run -- $P > /dev/null 2>&1 || { echo "fetch fail $t"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$t/pmc_write" -o run -- $P > /dev/null 2>&1 || { echo "write fail $t"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$OUT/$t/pmc_valu" -o run -- $P > /dev/null 2>&1 || { echo "valu fail $t"; exit 1; }
  echo "done $t"
done
