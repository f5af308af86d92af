#!/usr/bin/env bash
# PMC counters of the shared-prefix attention kernels (one config, B=80 P=8000).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES"; do
    i=$((i + 1))
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$ROOT/gpurun_out/pmc$i" -o p \
        -- python3 "$ROOT/scripts/bench_kernels.py" prefix8k > "$ROOT/gpurun_out/pmc$i.log" 2>&1 || exit $?
done
python3 - "$ROOT/gpurun_out" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        k = "prefix" if "prefix_attn" in k else "suffix" if "decode_attn_kernel" in k else "combine" if "combine" in k else "other"
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
