set -u
O=gpurun_out/r5az; mkdir -p $O
V=RTAMD_LIB_PATH=$PWD/3d-ray-tracer-vulkan_amd/lib/variants/librtamd_scalar.so
env $V timeout -k 10 600 python -u -m pytest tests/test_gpu_accel.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -m gpu > $O/pytest_scalar.log 2>&1 || exit $?
bash tools/ab_env.sh $O/ab3 3 "-" "$V" -- --steps 200 --warmup 5 || exit $?
bash tools/ab_env.sh $O/ab5 2 "-" "$V" -- --config 5 --steps 20 --warmup 3 || exit $?
bash tools/ab_env.sh $O/ab6 2 "-" "$V" -- --config 6 --steps 200 --warmup 5 || exit $?
