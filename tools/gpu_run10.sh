set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=v3 STEPS=10 bash tools/profile.sh
