# Round 2: GPU tests incl. the full-size headline parity tests, then the default bench line
# (with its oracle leg: parity_max_rel + cpu_baseline), and a host-core probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r2_parity1; mkdir -p $O
export TMPDIR=/tmp
{ nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; free -g; } > $O/host.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
