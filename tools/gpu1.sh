cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && rocm-smi --showproductname > gpurun_out/smi.txt 2>&1; 
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench.py --replicas 1024 --pods 4096 --steps 2 --warmup 1 --cpu-seconds 5 --cpu-workers 4 > gpurun_out/bench_small.json 2> gpurun_out/bench_small.err && echo BENCH_OK
