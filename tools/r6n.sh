set -o pipefail
mkdir -p gpurun_out/r6n
timeout -k 10 120 tools/micro/linkpar > gpurun_out/r6n/linkpar.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/writer_bench.py --reps 3 > gpurun_out/r6n/writer.txt 2>&1 || exit 1
