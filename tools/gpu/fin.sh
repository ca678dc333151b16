# k_finalize grid sized by the long-row count (16..512 workgroups): GPU tests, s20 / LJ / s26 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/fin; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/ -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 150 python -u bench.py --scale 20 --steps 100 --warmup 10 --no-cpu-baseline > $O/rmat_s20.log 2>&1 && \
timeout -k 10 150 python -u bench.py --graph lj --steps 50 --warmup 5 --no-cpu-baseline > $O/lj.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/rmat_s26.log 2>&1
