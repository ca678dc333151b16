# Profiles of the current layout (64 classes, grouped epilogue) + multi-part validation at s26.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=c64 bash tools/profile.sh || exit 1
timeout -k 10 500 python3 -u tools/group_bench.py --scale 26 --parts 2,8 --iters 5 > gpurun_out/prof/group_s26_c64.log 2>&1
