set -e
cd $GRAFT_REPO_ROOT
bash scripts/gpu.sh round r06 512
cat gpurun_out/r06/roofline_agreement.md
bash scripts/gpu.sh pmc r06pmc_final "gemmp|bwd3|fwd2|wgradp|ln.*bwd_kernel|ln.*fwd_kernel" -- python /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-b64 --no-data-pipeline
