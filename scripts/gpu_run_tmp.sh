mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 280 -x > gpurun_out/r2l_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r2l_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'tts-max_amd')
from tts_amd import configs
from tts_amd.speechlm import MI355XSpeechLM
m = MI355XSpeechLM.synthetic(configs.TTS1, seed=0x5EED, max_batch=32, max_seq_len=718)
for k in ('qkv','qkv_attn','attention','o_proj'):
    print(k, m.bench_kernel(k, rows=1, ctx=452, iters=30))
print('attention32', m.bench_kernel('attention', rows=32, ctx=452, iters=30))
" || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/r2l_bench.json 2> gpurun_out/r2l_bench.err || exit $?
python -c "import json; d=json.load(open('gpurun_out/r2l_bench.json')); print(d['value'], d['roofline']['decode_step'], d['roofline']['per_step_share_ms'])"
