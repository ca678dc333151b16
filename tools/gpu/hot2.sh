# Hot-set size sweep + diagnostic variants of k_spmv_hot (0 product, 1 all-LDS, 2 no stores).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-hot2}
for K in ${KS:-0 2048 4096 8192 12288 18432}; do PR_HOT_SLOTS=$K timeout -k 10 200 python -u tools/diag_spmv.py --scale 26 --layout split --variants ${VARS:-0,1,2} --rounds 3 --iters 5 > gpurun_out/${T}_diag_k$K.log 2>&1 || exit 1; done
