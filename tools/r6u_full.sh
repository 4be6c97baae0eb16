# the whole GPU suite and smoke at the current tree, then the metric / templated circuits checked
set -o pipefail
mkdir -p gpurun_out/r6u
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/r6u/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6u/smoke.log 2>&1 || exit 1
