#!/usr/bin/env bash
# One GPU session on the MI355X box: GPU tests, smoke, bench.py (with
# extra.enrichLocal), bench_enrich (fp8 / bf16 KV), batched prefill, decode
# step at 320 / 78 rows and its rocprofv3 kernel stats.  Every GPU step has its
# own time limit; a crash / abort / timeout ends the script (ordinary test
# failures do not).  Output goes to gpurun_out/round/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=gpurun_out/round
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="${STEPS:-pytest smoke bench enrich_fp8 enrich_bf16 prefill step prof}"

run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 3 "$OUT/$name.log"
    case $rc in
        0|1|5) return 0 ;;                 # ok / test failures / no tests collected
        *) echo "fatal rc=$rc in $name: stopping"; exit $rc ;;
    esac
}

for s in $STEPS; do
    case $s in
        pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
        smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run bench 900 python bench.py --steps 20 --warmup 5 ;;
        enrich_fp8) run enrich_fp8 900 python bench_enrich.py --kv-dtype fp8 ;;
        enrich_bf16) run enrich_bf16 900 python bench_enrich.py --kv-dtype bf16 ;;
        enrich_llama) run enrich_llama 900 python bench_enrich.py --preset llama3.2-1b-code --kv-dtype fp8 ;;
        enrich_llama_bf16) run enrich_llama_bf16 900 python bench_enrich.py --preset llama3.2-1b-code --kv-dtype fp8 \
                --prefill-dtype bf16 ;;
        enrich_llama257) run enrich_llama257 600 python bench_enrich.py --preset llama3.2-1b-code --classes 257 ;;
        enrich_llama_r512) run enrich_llama_r512 600 python bench_enrich.py --preset llama3.2-1b-code --max-rows 512 ;;
        enrich_llama_b384) run enrich_llama_b384 600 python bench_enrich.py --preset llama3.2-1b-code --batch 384 ;;
        prof_llama)
            ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof_llama" -o enrich -- python3 "$ROOT/bench_enrich.py" --preset llama3.2-1b-code \
                --classes 512 --warmup 4 > "$ROOT/$OUT/prof_llama.log" 2>&1 )
            rc=$?
            echo "=== prof_llama rc=$rc"
            find "$OUT/prof_llama" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            python3 scripts/kstats.py $(find "$OUT/prof_llama" -name '*kernel_stats.csv' | head -1) \
                > "$OUT/kstats_llama.txt" 2>&1
            head -30 "$OUT/kstats_llama.txt"
            [ $rc -eq 0 ] || exit $rc ;;
        prof_llama_fp8)
            ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof_llama_fp8" -o enrich -- python3 "$ROOT/bench_enrich.py" --preset llama3.2-1b-code \
                --classes 512 --warmup 4 --prefill-dtype fp8 --decode-dtype fp8 > "$ROOT/$OUT/prof_llama_fp8.log" 2>&1 )
            rc=$?
            echo "=== prof_llama_fp8 rc=$rc"
            find "$OUT/prof_llama_fp8" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            python3 scripts/kstats.py $(find "$OUT/prof_llama_fp8" -name '*kernel_stats.csv' | head -1) \
                > "$OUT/kstats_llama_fp8.txt" 2>&1
            head -30 "$OUT/kstats_llama_fp8.txt"
            [ $rc -eq 0 ] || exit $rc ;;
        prof_byte)
            ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof_byte" -o enrich -- python3 "$ROOT/bench_enrich.py" --classes 512 --warmup 4 \
                > "$ROOT/$OUT/prof_byte.log" 2>&1 )
            rc=$?
            echo "=== prof_byte rc=$rc"
            find "$OUT/prof_byte" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            python3 scripts/kstats.py $(find "$OUT/prof_byte" -name '*kernel_stats.csv' | head -1) \
                > "$OUT/kstats_byte.txt" 2>&1
            head -30 "$OUT/kstats_byte.txt"
            [ $rc -eq 0 ] || exit $rc ;;
        gaps_llama)  # GPU idle inside the timed engine run (verdict item 8): busy fraction + largest gaps
            ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
                -d "$ROOT/$OUT/gaps_llama" -o enrich -- python3 "$ROOT/bench_enrich.py" --preset llama3.2-1b-code \
                --classes 512 --warmup 4 > "$ROOT/$OUT/gaps_llama.log" 2>&1 )
            rc=$?
            echo "=== gaps_llama rc=$rc"
            [ $rc -eq 0 ] || exit $rc
            el=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['elapsed_s'])" \
                "$OUT/gaps_llama.log")
            python3 scripts/kernel_gaps.py $(find "$OUT/gaps_llama" -name '*kernel_trace.csv' | head -1) "$el" \
                > "$OUT/gaps_llama.txt" 2>&1
            find "$OUT/gaps_llama" -type f -delete 2>/dev/null
            cat "$OUT/gaps_llama.txt" ;;
        prefill) run prefill 300 python scripts/bench_prefill.py --seqs 12 ;;
        pgemm_test) run pgemm_test 300 python -u -m pytest tests/test_gpu_pgemm.py -x -v --timeout 120 \
                --timeout-method thread ;;
        pgemm_bench) run pgemm_bench 300 python scripts/bench_pgemm.py --preset llama3.2-1b-code --rows 24576 ;;
        enrich_llama_fp8) run enrich_llama_fp8 900 python bench_enrich.py --preset llama3.2-1b-code --kv-dtype fp8 \
                --prefill-dtype fp8 --decode-dtype fp8 ;;
        enrich_llama_pf8) run enrich_llama_pf8 900 python bench_enrich.py --preset llama3.2-1b-code --kv-dtype fp8 \
                --prefill-dtype fp8 ;;
        step_fp8)
            for r in "256 64" "448 64"; do set -- $r
                run step_bf16_$(($1 + $2)) 300 python scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --iters 60
                run step_fp8_$(($1 + $2)) 300 python scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 \
                    --decode-dtype fp8 --iters 60
            done ;;
        prof_prefill)
            ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof_prefill" -o pf -- python3 "$ROOT/scripts/bench_prefill.py" \
                --preset llama3.2-1b-code --prefix 1119 --tokens 561 --seqs 44 --iters 5 --prefill-dtype fp8 \
                > "$ROOT/$OUT/prof_prefill.log" 2>&1 )
            rc=$?
            echo "=== prof_prefill rc=$rc"
            find "$OUT/prof_prefill" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            cp $(find "$OUT/prof_prefill" -name '*kernel_stats.csv' | head -1) "$OUT/prefill_fp8_kernel_stats.csv"
            tail -2 "$OUT/prof_prefill.log"
            [ $rc -eq 0 ] || exit $rc ;;
        prefill_llama)
            run prefill_llama_bf16 300 python scripts/bench_prefill.py --preset llama3.2-1b-code --prefix 1119 \
                --tokens 561 --seqs 44 --iters 5
            run prefill_llama_fp8 300 python scripts/bench_prefill.py --preset llama3.2-1b-code --prefix 1119 \
                --tokens 561 --seqs 44 --iters 5 --prefill-dtype fp8 ;;
        pmc_llama) run pmc_llama 900 bash scripts/pmc_decode_step.sh --preset llama3.2-1b-code --batch 256 \
                --extra 64 --kv-dtype fp8 --prefix 1119 --ctx 700 ;;
        pmc_llama_fp8) run pmc_llama_fp8 900 bash scripts/pmc_decode_step.sh --preset llama3.2-1b-code \
                --batch 256 --extra 64 --kv-dtype fp8 --prefix 1119 --ctx 700 --decode-dtype fp8 ;;
        enrich_fp8_nofork) run enrich_fp8_nofork 900 python bench_enrich.py --kv-dtype fp8 --no-fork ;;
        step_llama)
            run step_llama533 300 python scripts/bench_step.py --preset llama3.2-1b-code --batch 512 --extra 21 \
                --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 60
            run step_llama268 300 python scripts/bench_step.py --preset llama3.2-1b-code --batch 256 --extra 12 \
                --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 60 ;;
        ckpt_test) run ckpt_test 900 python -u -m pytest tests/test_gpu_checkpoint_full.py -x -v -s --timeout 900 \
                --timeout-method thread ;;
        tgemm_test) run tgemm_test 600 python -u -m pytest tests/test_gpu_tgemm.py -x -q --timeout 120 \
                --timeout-method thread ;;
        tgemm_small) run tgemm_small 900 python scripts/bench_tgemm.py --rows 40 80 160 320 --only qkv,o,gu,down,head ;;
        wg_sweep) run wg_sweep 600 python scripts/bench_tgemm.py --rows 40 80 160 320 --only qkv,o,down --wg-sweep ;;
        tgemm_sweep) run tgemm_sweep 900 python scripts/bench_tgemm.py --rows 520 610 768 1024 --only gu,head --sweep ;;
        step_small)  # small-row latency (verdict item 5): 40 / 80 / 160 rows
            for r in "32 8" "64 16" "128 32"; do set -- $r
                run step_llama$(($1 + $2)) 300 python scripts/bench_step.py --preset llama3.2-1b-code --batch $1 \
                    --extra $2 --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 100
            done ;;
        kern_tests) run kern_tests 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_wgemm.py \
                tests/test_gpu_tgemm.py tests/test_gpu_pgemm.py tests/test_gpu_prefill.py tests/test_gpu_model.py \
                -x -q --timeout 120 --timeout-method thread ;;
        attn_ab)  # small-step attention plans: shared-prefix key splits x per-row minimum chunk, alternating
            for rep in 1 2; do for cfg in "0 256" "8 256" "0 128" "8 128"; do set -- $cfg
                for r in "32 8" "64 16" "128 32"; do set -- $cfg $r
                    DMCP_PREFIX_SPLITS=$([ $1 = 0 ] || echo $1) DMCP_DECODE_MIN_CHUNK=$2 \
                        run attn_ab_p$1_c$2_$(($3 + $4))_$rep 300 python scripts/bench_step.py \
                        --preset llama3.2-1b-code --batch $3 --extra $4 --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 100
                done; done; done
            for f in "$OUT"/attn_ab_*.log; do echo "$(basename $f .log) $(grep -h '^{' $f)"; done > "$OUT/attn_ab.txt" ;;
        psplit_byte)  # shared-prefix key splits at small steps on the byte preset (4,949-token prefix)
            for rep in 1 2; do for sp in 0 8; do for r in "32 8" "64 16" "128 32"; do set -- $r
                DMCP_PREFIX_SPLITS=$([ $sp = 0 ] || echo $sp) run psplit_byte_p${sp}_$(($1 + $2))_$rep 300 \
                    python scripts/bench_step.py --batch $1 --extra $2 --kv-dtype fp8 --prefix 4949 --ctx 2400 --iters 60
            done; done; done
            for f in "$OUT"/psplit_byte_*.log; do echo "$(basename $f .log) $(grep -h '^{' $f)"; done > "$OUT/psplit_byte.txt" ;;
        gaps_ab)  # engine idle: refill + admission under the launched step (1) vs at the iteration's top (0)
            for rep in 1 2; do for u in 0 1; do
                LOCAL_LLM_HOST_UNDER_STEP=$u run gaps_ab_u${u}_$rep 600 python bench_enrich.py --preset llama3.2-1b-code \
                    --classes 1024 --warmup 4
            done; done
            for f in "$OUT"/gaps_ab_*.log; do echo "$(basename $f .log) $(grep -h '^{' $f)"; done > "$OUT/gaps_ab.txt" ;;
        nt_ab)  # the weight-streaming GEMM's weight loads nt (aux 2) vs default policy, small / mid steps, alternating
            for rep in 1 2; do for aux in 0 2; do for r in "32 8" "64 16" "128 32" "256 64" "448 64"; do set -- $r
                run nt_ab_a${aux}_$(($1 + $2))_$rep 300 python scripts/bench_step.py --preset llama3.2-1b-code \
                    --batch $1 --extra $2 --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 100 --wgemm-aux $aux
            done; done; done
            for f in "$OUT"/nt_ab_*.log; do echo "$(basename $f .log) $(grep -h '^{' $f)"; done > "$OUT/nt_ab.txt" ;;
        split_ab)  # per-row attention plan in the engine: (min chunk, min splits) -- long rows cut into more waves
            for rep in 1 2; do for cfg in "256 1" "512 8" "256 8"; do set -- $cfg
                DMCP_DECODE_MIN_CHUNK=$1 DMCP_DECODE_MIN_SPLITS=$2 run split_ab_llama_c$1_s$2_$rep 600 \
                    python bench_enrich.py --preset llama3.2-1b-code --classes 1024 --warmup 4
                DMCP_DECODE_MIN_CHUNK=$1 DMCP_DECODE_MIN_SPLITS=$2 run split_ab_byte_c$1_s$2_$rep 600 \
                    python bench_enrich.py --classes 512 --warmup 4
            done; done
            for f in "$OUT"/split_ab_*.log; do echo "$(basename $f .log) $(grep -h '^{' $f)"; done > "$OUT/split_ab.txt" ;;
        head_ab)  # LM head parts of <= 256 rows (64-deep stages) vs <= 320 rows (32-deep), alternating
            run head_test 300 python -u -m pytest tests/test_gpu_tgemm.py -x -q --timeout 120 --timeout-method thread \
                -k "argmax"
            for rep in 1 2; do for hr in 256 320; do
                DMCP_TG_HEAD_ROWS=$hr run head_ab_tg_${hr}_$rep 300 python scripts/bench_tgemm.py --rows 520 610 640 \
                    --only head
                DMCP_TG_HEAD_ROWS=$hr run head_ab_step_${hr}_$rep 300 python scripts/bench_step.py \
                    --preset llama3.2-1b-code --batch 512 --extra 98 --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 60
            done; done
            for f in "$OUT"/head_ab_*.log; do grep -h '^{' $f | sed "s/^/$(basename $f .log) /"; done > "$OUT/head_ab.txt" ;;
        prof_step80)
            ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof_step80" -o step -- python3 "$ROOT/scripts/bench_step.py" \
                --preset llama3.2-1b-code --batch 64 --extra 16 --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 60 \
                > "$ROOT/$OUT/prof_step80.log" 2>&1 )
            rc=$?
            echo "=== prof_step80 rc=$rc"
            find "$OUT/prof_step80" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            cp $(find "$OUT/prof_step80" -name '*kernel_stats.csv' | head -1) "$OUT/step80_kernel_stats.csv"
            [ $rc -eq 0 ] || exit $rc ;;
        ckpt_enrich)  # a written 16-layer, 128,256-id checkpoint through the engine, + its kernel trace
            run ckpt_enrich 900 python bench_enrich.py --checkpoint /tmp/dmcp_ckpt --write-checkpoint --classes 1024
            ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof_ckpt" -o enrich -- python3 "$ROOT/bench_enrich.py" --checkpoint /tmp/dmcp_ckpt \
                --classes 512 --warmup 4 > "$ROOT/$OUT/prof_ckpt.log" 2>&1 )
            rc=$?
            echo "=== prof_ckpt rc=$rc"
            find "$OUT/prof_ckpt" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            cp $(find "$OUT/prof_ckpt" -name '*kernel_stats.csv' | head -1) "$OUT/ckpt_kernel_stats.csv"
            python3 scripts/kstats.py "$OUT/ckpt_kernel_stats.csv" > "$OUT/kstats_ckpt.txt" 2>&1
            head -30 "$OUT/kstats_ckpt.txt"
            [ $rc -eq 0 ] || exit $rc ;;
        step_llama3)  # the verdict's three operating points: 320 / 610 / 768 rows
            for r in "256 64" "512 98" "512 256"; do set -- $r
                run step_llama$(($1 + $2)) 300 python scripts/bench_step.py --preset llama3.2-1b-code --batch $1 \
                    --extra $2 --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 60
            done ;;
        prof_step610)
            ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof_step610" -o step -- python3 "$ROOT/scripts/bench_step.py" \
                --preset llama3.2-1b-code --batch 512 --extra 98 --kv-dtype fp8 --prefix 1119 --ctx 700 --iters 40 \
                > "$ROOT/$OUT/prof_step610.log" 2>&1 )
            rc=$?
            echo "=== prof_step610 rc=$rc"
            find "$OUT/prof_step610" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            cp $(find "$OUT/prof_step610" -name '*kernel_stats.csv' | head -1) "$OUT/step610_kernel_stats.csv"
            python3 scripts/kstats.py "$OUT/step610_kernel_stats.csv" > "$OUT/kstats_step610.txt" 2>&1
            head -25 "$OUT/kstats_step610.txt"
            [ $rc -eq 0 ] || exit $rc ;;
        step)
            run step320 300 python scripts/bench_step.py --batch 256 --extra 64 --kv-dtype fp8 --iters 100
            run step78 300 python scripts/bench_step.py --batch 64 --extra 14 --kv-dtype fp8 --iters 100 ;;
        prof)
            ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
                -d "$ROOT/$OUT/prof" -o step -- python3 "$ROOT/scripts/bench_step.py" --batch 256 --extra 64 \
                --kv-dtype fp8 --iters 50 > "$ROOT/$OUT/prof.log" 2>&1 )
            rc=$?
            echo "=== prof rc=$rc"
            find "$OUT/prof" -type f ! -name '*kernel_stats*' -delete 2>/dev/null
            python3 scripts/kstats.py $(find "$OUT/prof" -name '*kernel_stats.csv' | head -1) > "$OUT/kstats.txt" 2>&1
            head -25 "$OUT/kstats.txt"
            [ $rc -eq 0 ] || exit $rc ;;
    esac
done
echo "=== done"
