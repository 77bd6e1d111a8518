set -o pipefail
mkdir -p gpurun_out/r03
export TMPDIR=/tmp
L=$PWD/bluesky-gym-hallucination_amd/bluesky_gym/_lib
BSG_LIBRARY=$L/libbsg_stamps.so timeout -k 10 180 python tools/stamps.py 4096 32 > gpurun_out/r03/stamps_4096.txt 2>&1 || { echo STAMPS_FAILED; tail gpurun_out/r03/stamps_4096.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/stamps_4096.txt | head -30
timeout -k 10 150 python tools/probe/substep_probe.py tools/probe/substep_probe > gpurun_out/r03/probe_now.txt 2>&1 || { echo PROBE_FAILED; exit 1; }
grep "substep cycles" -A1 gpurun_out/r03/probe_now.txt
for exe in substep_probe_base substep_probe; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 --output-format csv -d gpurun_out/r03/pmc_probe_$exe -o run -- tools/probe/$exe gpurun_out/substep_state.bin > /dev/null 2>&1 || { echo PMC_FAILED $exe; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for exe in ("substep_probe_base", "substep_probe"):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r03/pmc_probe_{exe}/*/run_counter_collection.csv") + glob.glob(f"gpurun_out/r03/pmc_probe_{exe}/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(exe, {k: round(min(v)) for k, v in sorted(agg.items())})
PY
timeout -k 10 300 python tools/ablate.py merge32_full_1024 merge32_full_2048 merge32_full_512 merge32_full > gpurun_out/r03/ablate_shards.txt 2>&1 || { echo ABL_FAILED; tail gpurun_out/r03/ablate_shards.txt; exit 1; }
grep " us " gpurun_out/r03/ablate_shards.txt
