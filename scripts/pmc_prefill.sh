#!/usr/bin/env bash
# PMC counters of the MFMA prefill-attention kernel (one arm of
# bench_prefill_attn.py): one rocprofv3 pass per counter set.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$ROOT/gpurun_out/pmcp$i" -o p \
        -- python3 "$ROOT/scripts/bench_prefill_attn.py" --arms mfma_v0_s2 --rounds 1 --iters 5 \
        > "$ROOT/gpurun_out/pmcp$i.log" 2>&1 || exit $?
done
python3 - "$ROOT/gpurun_out" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float)
n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/pmcp*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "prefill_attn_kernel" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for c, v in sorted(agg.items()):
    print(f"{c:28s} {v:.4g}  (over {n[c]} dispatch records)")
PY
find "$ROOT/gpurun_out" -path '*pmcp*' -name '*.csv' -size +20M -delete
