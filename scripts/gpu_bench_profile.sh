set -e
mkdir -p gpurun_out/prof1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --batch 128 > gpurun_out/bench_b128.json 2> gpurun_out/bench_b128.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 64 --no-cpu-baseline > gpurun_out/bench_b64.json 2> gpurun_out/bench_b64.err
timeout -k 10 300 python bench.py --steps 10 --warmup 5 --batch 256 --no-cpu-baseline > gpurun_out/bench_b256.json 2> gpurun_out/bench_b256.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --batch 128 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/gpurun_out/prof1/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof1/bench.err
