# HIP runtime knobs under /opt/rocm's runtime vs torch's bundled one (bench.py, metric circuit)
set -o pipefail
mkdir -p gpurun_out/r6k
A="--steps 30 --warmup 3 --no-cpu --no-flatten --no-templated --no-o1 --no-linear1m --no-link"
for i in 1 2; do
  for v in base blit wait torch; do
    case $v in
      base) timeout -k 10 200 python -u bench.py $A > gpurun_out/r6k/${v}_$i.json 2> gpurun_out/r6k/${v}_$i.err || exit 1;;
      blit) GPU_FORCE_BLIT_COPY_SIZE=65536 timeout -k 10 200 python -u bench.py $A > gpurun_out/r6k/${v}_$i.json 2> gpurun_out/r6k/${v}_$i.err || exit 1;;
      wait) ROC_ACTIVE_WAIT_TIMEOUT=5000 timeout -k 10 200 python -u bench.py $A > gpurun_out/r6k/${v}_$i.json 2> gpurun_out/r6k/${v}_$i.err || exit 1;;
      torch) timeout -k 10 200 python -u -c "import torch, runpy, sys; torch.zeros(1, device='cuda'); sys.argv = ['bench.py'] + '$A'.split(); runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/r6k/${v}_$i.json 2> gpurun_out/r6k/${v}_$i.err || exit 1;;
    esac
  done
  echo "round $i"
done
