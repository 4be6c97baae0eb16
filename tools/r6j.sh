set -o pipefail
mkdir -p gpurun_out/r6j
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread "tests/test_gpu_sharded.py::test_two_process_host_transport" "tests/test_gpu_sharded.py::test_rccl_world1_join" > gpurun_out/r6j/tests.log 2>&1 || exit 1
bash tools/r6i_ab.sh
