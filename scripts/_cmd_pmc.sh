set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/pmc_kernel.sh gpurun_out/pmct "k_gather_tab|k_scatter_tab|k_bucket_fill" --steps 2 --warmup 1 --no-cpu-baseline || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmct > gpurun_out/pmct/summary.txt
find gpurun_out/pmct -name "*.csv" -delete
cat gpurun_out/pmct/summary.txt
