cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad_x3_forms or large_grids or conv_fwd_bwd" 2>&1 | tail -2 || exit 1
OFLOW_TUNE=4=2 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_fwd_bwd" 2>&1 | tail -1 || exit 1
OFLOW_TUNE=4=2,5=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv_fwd_bwd" 2>&1 | tail -1 || exit 1
bash tools/gpu_abtune.sh "dec3.c0,dec3.c1,dec3.c2,dec3.c3,dec3.c4,dec2.c1,dec1.c1,enc.l2,enc.l3,enc.l4" 1 "mi1:5=1" "all2:4=2" "all1:4=2,5=1" "old:4=0"
