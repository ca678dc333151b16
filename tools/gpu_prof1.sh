set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/prof/counters.txt 2>&1 || true
TAG=v1 bash tools/profile.sh
