#!/usr/bin/env bash
# rocprofv3 kernel stats of the decode step at 320 rows (fp8 KV), then PMC of
# the weight-streaming GEMM kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/wgp
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--batch 256 --extra 64 --kv-dtype fp8 --iters 30 ${STEP_ARGS:-}"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o step \
    -- python3 "$ROOT/scripts/bench_step.py" $ARGS > "$ROOT/$OUT/prof.log" 2>&1 ) || exit 1
find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -int(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:120]}')
PY
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$ROOT/$OUT/pmc$i" -o p \
        -- python3 "$ROOT/scripts/bench_step.py" --batch 256 --extra 64 --kv-dtype fp8 --iters 10 > "$ROOT/$OUT/pmc$i.log" 2>&1 || exit $?
done
python3 - "$ROOT/$OUT" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        k = ("wgemm_" + k.split("wgemm_kernelILi")[1][:12]) if "wgemm_kernel" in k else \
            ("reduce" if "reduce_" in k else "attn" if "attn" in k else "gemm_lib" if "Cijk" in k else "other")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(agg.items()):
    print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
find "$ROOT/$OUT" -path '*pmc*' -name '*.csv' -size +20M -delete
