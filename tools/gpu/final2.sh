# Default build with the 128-slot staging window (18430 hot slots): GPU parity suite, smoke(),
# the default bench line with the CPU baseline, then the rocprofv3 trace + PMC passes (tools/profile.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/final2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 1
TAG=final2 STEPS=10 bash tools/profile.sh
