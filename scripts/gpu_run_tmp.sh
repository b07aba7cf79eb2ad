mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r2n_prof32 -o run -- python3 scripts/gen_probe.py 32 120 > gpurun_out/r2n_prof32.log 2>&1 || exit $?
python scripts/step_breakdown.py $(find gpurun_out/r2n_prof32 -name "*kernel_trace.csv") > gpurun_out/r2n_break32.txt
find gpurun_out/r2n_prof32 -name "*trace*" -delete
cat gpurun_out/r2n_break32.txt
