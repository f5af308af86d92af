#!/usr/bin/env bash
# PMC counters of the decode step's kernels (bench_step.py defaults, 20 steps):
# one rocprofv3 pass per counter set, summed per kernel family.  Extra
# arguments go to bench_step.py (e.g. --kv-dtype fp8); PMC_PROG names another
# script to profile instead (e.g. scripts/bench_pgemm.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp
i=0
PROG=${PMC_PROG:-scripts/bench_step.py}
PROG_ARGS=$([ -z "${PMC_PROG:-}" ] && echo "--iters 20")
SETS=${PMC_SETS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES;FETCH_SIZE SQ_INSTS_VMEM_RD"}
rm -rf "$ROOT"/gpurun_out/pmcd*
IFS=';' read -ra SETL <<< "$SETS"
for set in "${SETL[@]}"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$ROOT/gpurun_out/pmcd$i" -o p \
        -- python3 "$ROOT/$PROG" $PROG_ARGS "$@" > "$ROOT/gpurun_out/pmcd$i.log" 2>&1 || exit $?
done
python3 - "$ROOT/gpurun_out" <<'PY'
import csv, glob, re, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
for f in glob.glob(sys.argv[1] + "/pmcd*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")
        mode = re.search(r"wgemm_kernel<\d+, \d+, \d+, (\d)", k)
        tg = re.search(r"tgemm_kernel<\d+, (\d)", k)
        k = (("tgemm_" + ["bf16", "part", "swiglu", "head"][int(tg.group(1))]) if tg else
             "tgemm_head" if "tgemm_argmax_reduce" in k else
             "prefix" if "prefill_attn" in k else "decode_mfma" if "decode_attn_mfma" in k else
             "combine" if "combine" in k else "gemm_lib" if "Cijk" in k else "rmsnorm" if "rmsnorm" in k else
             "lm_head_argmax" if (mode and mode.group(1) == "3") or "lm_head_reduce" in k else
             "wgemm_swiglu" if mode and mode.group(1) == "2" else "wgemm" if "wgemm_kernel" in k else
             "wmx_swiglu" if "wmx_kernel<64, 1, 2" in k or "wmx_kernel<64, 2, 2" in k else
             "wmx" if "wmx_kernel" in k else
             ("pgemm_" + ["bf16", "resid", "swiglu", "qkv"][int(re.search(r"pgemm_kernel<(\d)", k).group(1))])
             if re.search(r"pgemm_kernel<\d", k) else
             "reduce" if "reduce_" in k else "mx_quant" if "mx_quant" in k else "other")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in sorted(agg.items()):
    print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
find "$ROOT/gpurun_out" -path '*pmcd*' -name '*.csv' -size +20M -delete
