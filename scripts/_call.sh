cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06
for rep in 1 2; do
PYTHONFAULTHANDLER=1 NCCL_DEBUG=WARN DNA_DDP_FORCE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b64 --no-data-pipeline > gpurun_out/r06/force$rep.json 2> gpurun_out/r06/force$rep.err
echo "force rc=$?"
head -c 300 gpurun_out/r06/force$rep.json; echo
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-b64 --no-data-pipeline > gpurun_out/r06/noforce$rep.json 2> gpurun_out/r06/noforce$rep.err
echo "noforce rc=$?"
head -c 300 gpurun_out/r06/noforce$rep.json; echo
done
