# LJ- and Twitter-shaped benches with the current defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cl2
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --graph lj --steps 20 --warmup 3 > gpurun_out/cl2/lj.log 2>&1 && \
timeout -k 10 400 python -u bench.py --graph twitter --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/cl2/tw.log 2>&1
