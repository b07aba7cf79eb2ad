# A/B of two builds of the library on ONE box: bench.py (bs=1, no secondary/cpu) alternately
# with TTS_LIB_PATH=$1 (A) and the in-tree build (B), $2 rounds.  usage: bash scripts/ab_bench.sh scripts/ab_lib/libtts_base.so 2
mkdir -p gpurun_out
A=$1; R=${2:-2}
for r in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then export TTS_LIB_PATH=$A; else unset TTS_LIB_PATH; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 3 > gpurun_out/ab_$v$r.json 2>/dev/null || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab_$v$r.json')); r=d['roofline']; print('$v', d['value'], r['decode_step']['ms'], {k: v['avg_ms'] for k, v in r['kernels'].items()})"
  done
done
