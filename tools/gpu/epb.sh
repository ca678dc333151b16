# Grouped epilogue: grid cap (PR_EPI_BLOCKS) and a 5-workgroups-per-CU window (variant 5) at 64 classes, s26.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/epb; mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/$1.log 2>&1; }
PR_EPI_VAR=0 run v0_b2048 && PR_EPI_VAR=0 PR_EPI_BLOCKS=1024 run v0_b1024 && PR_EPI_VAR=0 PR_EPI_BLOCKS=4096 run v0_b4096 && \
PR_EPI_VAR=5 run v5_b2048 && PR_EPI_VAR=5 PR_EPI_BLOCKS=1280 run v5_b1280 && PR_EPI_VAR=5 PR_EPI_BLOCKS=2560 run v5_b2560 && \
PR_EPI_VAR=0 run v0_b2048_again
