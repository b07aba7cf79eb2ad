#!/bin/bash
# round 6: why the 17..32-row screen is slow: recompute skipped (diag 1) vs on, units recomputed (diag 2)
set -u
O=gpurun_out
T=${1:-r6ab}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN_DIAG 32 1 > $O/${T}_ab_diag_32.txt 2>&1; rc=$?
cat $O/${T}_ab_diag_32.txt; fatal $rc diag32
TTS_HEAD_SCREEN_DIAG=2 timeout -k 10 300 python -u - tts1 > $O/${T}_count.txt 2>&1 <<'PY'
import sys
sys.path.insert(0, "tts-max_amd")
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.LM_ARCHS[sys.argv[1]]
vocab = configs.vocab_for(arch)
m = MI355XSpeechLM.synthetic(arch, max_batch=32, max_seq_len=720)
for rows in (16, 17, 32):
    ps = [synth.synthetic_prompt(vocab, u, 39, 150) for u in range(rows)]
    m.generate_batch(ps, max_length=len(ps[0]) + 20, min_new_tokens=20, eos_token_id=vocab.speech_end_id, repetition_penalty=1.1)
    print("rows", rows, "steps 20", flush=True)
PY
rc=$?; cat $O/${T}_count.txt; fatal $rc count
echo done
