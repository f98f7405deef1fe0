# Same-lease A/B of whole trees (library + Python) on the training bench:
# the trees alternate (A B C A B C ...) with --cpu-baseline 0; one JSON line
# per run, tagged with its tree and repetition.
# usage: tools/ab_tree.sh <reps> <tag> <tree> <tree> [tree ...]
mkdir -p gpurun_out
reps=$1; tag=$2; shift 2
: > gpurun_out/$tag.jsonl
for rep in $(seq 1 $reps); do
  for tree in "$@"; do
    echo "== rep $rep tree $tree" >&2
    (cd $tree && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0) \
      > gpurun_out/${tag}_last.out 2> gpurun_out/${tag}_last.err || { cat gpurun_out/${tag}_last.err >&2; exit 1; }
    tail -1 gpurun_out/${tag}_last.out | python -c "
import json,sys; d=json.loads(sys.stdin.read()); d['tree']='$tree'; d['rep']=$rep
print(json.dumps(d))" >> gpurun_out/$tag.jsonl
    python - <<PY >&2
import json
d=[json.loads(l) for l in open('gpurun_out/$tag.jsonl')][-1]
print(d['tree'], d['rep'], d['value'], 'img/s', d['ms_per_step'], 'ms', 'conv', d['roofline']['avg_us'], 'us', d.get('box', {}).get('box_mfma_tflops'))
PY
  done
done
