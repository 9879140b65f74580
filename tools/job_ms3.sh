export MDA_STREAMS=1
timeout -k 10 600 python -X faulthandler -m pytest tests/test_engine_gpu.py tests/test_inception_gpu.py -v -x -p no:cacheprovider > gpurun_out/ms3.log 2>&1
echo "rc=$?"
