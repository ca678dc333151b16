# Chung-Lu configs: the new parity tests, then the LJ- and Twitter-shaped bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-cl}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "chunglu or lj_shaped" > gpurun_out/${T}_pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --graph lj --steps 20 --no-cpu-baseline > gpurun_out/${T}_bench_lj.log 2>&1 && \
timeout -k 10 500 python -u bench.py --graph twitter --steps 10 --no-cpu-baseline > gpurun_out/${T}_bench_twitter.log 2>&1
