# Baseline GPU pass: parity tests, the default bench line, rocprofv3 kernel trace + PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-base}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && \
TAG=$TAG STEPS=10 bash tools/profile.sh
