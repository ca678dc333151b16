# The driver's round-end sequence on a clean in-tree build: GPU tests, smoke(), default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/roundend; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
