# Row partition at P = 8 (all parts on one GPU, kernels summed): 64 vs 32 column classes per part.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/grp_cls; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/group_bench.py --scale 26 --parts 8 --iters 5 > $O/p8_c64.log 2>&1 && \
PR_CLASSES=32 timeout -k 10 400 python3 -u tools/group_bench.py --scale 26 --parts 8 --iters 5 > $O/p8_c32.log 2>&1
