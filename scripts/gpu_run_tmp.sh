mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_config1.py tests/test_gpu_persist.py -v --timeout 280 > gpurun_out/r2m_tests.log 2>&1; rc=$?
tail -8 gpurun_out/r2m_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-secondary > gpurun_out/r2m_bench.json 2> gpurun_out/r2m_bench.err || exit $?
tail -3 gpurun_out/r2m_bench.err
python -c "import json; d=json.load(open('gpurun_out/r2m_bench.json')); print(d['value'], d['cpu_baseline'])"
