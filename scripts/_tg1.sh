set -o pipefail
O=gpurun_out/tg16; mkdir -p $O
for rep in 1 2; do
for r in "256 64" "448 64"; do set -- $r
  for t in 1 0; do
    timeout -k 10 200 python scripts/bench_step.py --preset llama3.2-1b-code --batch $1 --extra $2 --prefix 1119 --ctx 700 --kv-dtype fp8 --iters 60 --tghead $t >> $O/step.jsonl 2>> $O/step.err || exit $?
  done
done
for r in "512 98" "512 256"; do set -- $r
  for t in 1 0; do
    timeout -k 10 200 python scripts/bench_step.py --preset llama3.2-1b-code --batch $1 --extra $2 --prefix 1119 --ctx 700 --kv-dtype fp8 --iters 60 --tgemm $t >> $O/step.jsonl 2>> $O/step.err || exit $?
  done
done
done
python3 -c "
import json
for l in open('$O/step.jsonl'):
    r=json.loads(l); print(r['preset'], r['rows'], 'tgemm', r['tgemm'], 'head', r['tg_head'], r['device_ms'])
"
timeout -k 10 400 python bench_enrich.py --preset llama3.2-1b-code > $O/enrich_llama.jsonl 2> $O/enrich_llama.err || exit $?
timeout -k 10 500 python bench_enrich.py > $O/enrich_byte.jsonl 2> $O/enrich_byte.err || exit $?
python3 -c "
import json
for f in ('enrich_llama','enrich_byte'):
    r=json.loads(open('$O/'+f+'.jsonl').read().strip().splitlines()[-1]); print(f, r['value'], r['decode_step_ms'], r['rows_per_step'], r.get('generated_tokens_per_class'))
"
