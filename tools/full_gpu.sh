set -o pipefail
mkdir -p gpurun_out/${OUT:-final}
timeout -k 10 1500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${OUT:-final}/gpu_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/${OUT:-final}/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${OUT:-final}/smoke.log 2>&1 && echo smoke ok >> gpurun_out/${OUT:-final}/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${OUT:-final}/bench.log 2>&1
