# Class-count policy check: GPU suite, then s26 and LJ benches with the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pol
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pol/pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/pol/s26.log 2>&1 && \
timeout -k 10 200 python -u bench.py --graph lj --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/pol/lj.log 2>&1
