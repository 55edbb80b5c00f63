set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1es
timeout -k 10 400 python bench.py > gpurun_out/r1es/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/r1es/bench.log; exit 1; }
tail -1 gpurun_out/r1es/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r1es/prof -o es -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r1es/prof.log 2>&1 || { echo prof failed; exit 1; }
cd $GRAFT_REPO_ROOT
bash scripts/pmc_traffic.sh gpurun_out/r1es/pmc --steps 3 --warmup 1 --no-cpu-baseline --no-degrid || exit 1
echo all done
