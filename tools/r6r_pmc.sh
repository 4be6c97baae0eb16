# the metric circuit's PMC passes (FETCH_SIZE, WRITE_SIZE, write requests) over one host -> host step only
set -e
OUT=gpurun_out/round6p
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link --no-hbm --no-write --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o f -- $B > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o w -- $B > $OUT/pmc_write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/pmc_wrreq -o q -- $B > $OUT/pmc_wrreq.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_writer.py > $OUT/writer_tests.log 2>&1
RS_PROF=1 timeout -k 10 300 python -u tools/writer_bench.py --reps 2 > $OUT/writer.txt 2> $OUT/writer.err
