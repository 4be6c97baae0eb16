set -o pipefail
# The round-end checks on one GPU box: the GPU test suite, smoke(), the default bench line.
# A step that times out, aborts or faults ends the script (no further GPU step after it).
O=gpurun_out/${OUT:-final}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/gpu_tests.log
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo smoke ok >> $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
