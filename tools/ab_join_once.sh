source tools/gpu_round.sh
step t_join timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_ext_overlap_gpu.py tests/test_dp_engine_gpu.py tests/test_inception_gpu.py tests/test_rccl_gpu.py -x -q --timeout 300 --timeout-method thread || exit 1
bash tools/gpu_session.sh ab "" "engine.lowering.LoweredProgram.JOIN_AT_FINALIZE=True" 3 MTL || exit 1
for f in A1 B1 A2 B2 A3 B3; do grep -o '"value": [0-9.]*' gpurun_out/ab_MTL_$f.log; done | tr '\n' ' '; echo
bash tools/gpu_session.sh ab "" "engine.lowering.LoweredProgram.JOIN_AT_FINALIZE=True" 2 multi_classifier || exit 1
for f in A1 B1 A2 B2; do grep -o '"value": [0-9.]*' gpurun_out/ab_multi_classifier_$f.log; done | tr '\n' ' '; echo
