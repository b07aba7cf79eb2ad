#!/bin/bash
# round 6: where the screened head's time goes: the recompute skipped (TTS_HEAD_SCREEN_DIAG=1,
# timing only) vs on, at TTS-1 1 / 8 rows and TTS-1-Max 8 rows; units recomputed per step (=2)
set -u
O=gpurun_out
T=${1:-r6y}
mkdir -p $O
export TMPDIR=/tmp
fatal() { if [ $1 -ne 0 ]; then echo "stop: rc=$1 in $2"; exit $1; fi; }
for r in 1 8; do
  timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN_DIAG $r 1 > $O/${T}_ab_diag_$r.txt 2>&1; rc=$?
  cat $O/${T}_ab_diag_$r.txt; fatal $rc diag$r
done
AB_ARCH=tts1-max timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN_DIAG 8 1 > $O/${T}_ab_diag_max8.txt 2>&1; rc=$?
cat $O/${T}_ab_diag_max8.txt; fatal $rc diagmax8
AB_ARCH=tts1-max timeout -k 10 600 python -u scripts/env_ab_probe.py TTS_HEAD_SCREEN_DIAG 1 1 > $O/${T}_ab_diag_max1.txt 2>&1; rc=$?
cat $O/${T}_ab_diag_max1.txt; fatal $rc diagmax1
for arch in tts1 tts1-max; do
  TTS_HEAD_SCREEN_DIAG=2 timeout -k 10 300 python -u - $arch > $O/${T}_count_$arch.txt 2>&1 <<'PY'
import sys
sys.path.insert(0, "tts-max_amd")
from tts_amd import configs, synth
from tts_amd.speechlm import MI355XSpeechLM
arch = configs.LM_ARCHS[sys.argv[1]]
vocab = configs.vocab_for(arch)
m = MI355XSpeechLM.synthetic(arch, max_batch=8, max_seq_len=720)
for rows in (1, 8):
    ps = [synth.synthetic_prompt(vocab, u, 39, 150) for u in range(rows)]
    m.generate_batch(ps, max_length=len(ps[0]) + 100, min_new_tokens=100, eos_token_id=vocab.speech_end_id, repetition_penalty=1.1)
    print("rows", rows, "steps 100", flush=True)
PY
  rc=$?; cat $O/${T}_count_$arch.txt; fatal $rc count
done
echo done
