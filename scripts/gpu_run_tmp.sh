mkdir -p gpurun_out && export TMPDIR=/tmp
for kr in "qkv_attn 1" "o_proj 1" "down 1" "lm_head 1" "qkv 32" "o_proj 32" "gate_up 32" "down 32" "attention 32" "lm_head 32"; do
  set -- $kr
  bash scripts/pmc_traffic.sh $1 $2 >> gpurun_out/pmc_all.log 2>&1 || exit $?
  echo "done $1 $2" 
done
find gpurun_out/pmc -name "*.csv" -size +2M -delete
